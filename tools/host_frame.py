"""Host cost of the SLAM leg's parts (GPU only): cProfile of process_frame over a few steady-state
frames of the street sequence (the same setup as bench.py's whole-frame leg)."""
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


def main(warm=10, prof=6):
    dev = "cuda"
    rng = np.random.default_rng(21)
    scene = street_scene(rng)
    poses = slam_poses(warm + prof)
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
    mapper = loop.mapper
    orig = mapper.process_frame
    pr = cProfile.Profile()
    wall = []

    def profiled(*a, **kw):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pr.enable()
        out = orig(*a, **kw)
        pr.disable()
        torch.cuda.synchronize()
        wall.append(time.perf_counter() - t0)
        return out
    mapper.process_frame = profiled
    for k in range(warm, warm + prof):
        loop.frame(scans[k])
    print("process_frame wall ms (profiled):", [round(w * 1e3, 3) for w in wall])
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
