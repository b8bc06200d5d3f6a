#!/usr/bin/env python3
"""Host cost of the whole SLAM frame (GPU only): per frame, the wall time of each part with the
device synchronised at the part boundaries (as bench.py's slam_frame leg) and the host time the
part's Python spent (perf_counter around the part, no sync inside); then a cProfile of whole frames
(tottime and cumulative).  A part whose host time is close to its wall time is host-bound."""
import cProfile
import os
import pstats
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import FrameLoop, Q_SCALE, lidar_scan, slam_poses, street_scene  # noqa: E402


def main(warm=10, n=12):
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
    walls, hosts = {}, {}
    for k in range(warm, warm + n):
        marks = []

        def mark(name):
            h = time.perf_counter()
            torch.cuda.synchronize()
            marks.append((name, h, time.perf_counter()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.frame(scans[k], timer=mark)
        prev = t0
        for name, h, w in marks:
            hosts.setdefault(name, []).append(h - prev)
            walls.setdefault(name, []).append(w - prev)
            prev = w
    print("part: wall ms (synchronised) / host ms (Python until the part's end, before its sync), medians")
    for name in walls:
        print(f"  {name:14s} {statistics.median(walls[name]) * 1e3:7.3f} {statistics.median(hosts[name]) * 1e3:7.3f}")
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pr.enable()
    for k in range(warm + n, warm + 2 * n):
        loop.frame(scans[k])
    pr.disable()
    torch.cuda.synchronize()
    print(f"profiled frames: {(time.perf_counter() - t0) / n * 1e3:.3f} ms per frame")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(70)


if __name__ == "__main__":
    main()
