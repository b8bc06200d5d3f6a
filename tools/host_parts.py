#!/usr/bin/env python3
"""Host cost inside the SLAM frame's parts (GPU only): cProfile over N frames after a warm-up,
then the callees of the frame loop's parts (read_and_preprocess, NeuralPoints.update, tracking,
process_frame, mapping, ...) with their cumulative times per frame, so the call sites that cost
host time (and the syncs, `item` / `nonzero` / `Event.synchronize`) are visible per part."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import FrameLoop, Q_SCALE, lidar_scan, slam_poses, street_scene  # noqa: E402

PARTS = ("frame", "read_and_preprocess", "update", "tracking", "process_frame", "mapping", "_dense_loop",
         "_step_plan", "reset_local_map", "query_certainty", "sample", "_build_occupancy", "grid_view",
         "voxel_down_sample", "_views", "_packed_pool", "_grid_view", "mlp_view", "_build_compact", "records",
         "_batch_sizes", "draw_shapes", "run", "assign_local_to_global")


def main(warm=10, n=16):
    dev = "cuda"
    rng = np.random.default_rng(21)
    scene = street_scene(rng)
    poses = slam_poses(warm + 2 * n)
    scans = [torch.from_numpy(lidar_scan(T, scene, rng).astype(np.float32) / np.float32(Q_SCALE)).to(dev)
             for T in poses]
    cfg = P.Config(device=dev, reg_iter_n=20, track_on=True)
    nm = P.NeuralPoints(cfg)
    torch.manual_seed(42)
    dec = P.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1).to(dev)
    loop = FrameLoop(cfg, nm, dec, P.Tracker(cfg, nm, dec), P.Mapper(cfg, None, nm, dec), build_index=True)
    for k in range(warm):
        loop.frame(scans[k])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(warm, warm + n):
        loop.frame(scans[k])
    torch.cuda.synchronize()
    print(f"unprofiled: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per frame (frames {warm}..{warm + n - 1})")
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pr.enable()
    for k in range(warm + n, warm + 2 * n):
        loop.frame(scans[k])
    pr.disable()
    torch.cuda.synchronize()
    print(f"profiled: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per frame")
    st = pstats.Stats(pr)
    st.calc_callees()
    callees = st.all_callees
    for name in PARTS:
        for func, (cc, nc, tt, ct, callers) in st.stats.items():
            if func[2] != name:
                continue
            print(f"== {name} ({os.path.basename(func[0])}:{func[1]}): {nc / n:.1f} calls, self {tt / n * 1e3:.3f}, "
                  f"cumulative {ct / n * 1e3:.3f} ms per frame")
            rows = sorted(callees.get(func, {}).items(), key=lambda kv: -kv[1][3])
            for cf, (ccc, cnc, ctt, cct) in rows:
                if cct / n * 1e3 < 0.004:
                    continue
                where = cf[2] if cf[0] == "~" else f"{os.path.basename(cf[0])}:{cf[1]}({cf[2]})"
                print(f"    {cnc / n:6.1f} calls  self {ctt / n * 1e3:7.3f}  cum {cct / n * 1e3:7.3f}  {where[:100]}")


if __name__ == "__main__":
    main()
