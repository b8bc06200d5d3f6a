"""Attribute the time of bench.py's whole-frame leg (configs[0]): run the frame loop over a few
frames, then time the tracker's registration iterations part by part."""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd import query as Q  # noqa: E402
from pin_slam_amd import tracker as TR  # noqa: E402
from pin_slam_amd.synthetic import FrameLoop, Q_SCALE, lidar_scan, slam_poses, street_scene  # noqa: E402


def main(frames=8):
    dev = "cuda"
    rng = np.random.default_rng(21)
    scene = street_scene(rng)
    poses = slam_poses(frames)
    scans = [torch.from_numpy(lidar_scan(T, scene, rng).astype(np.float32) / np.float32(Q_SCALE)).to(dev)
             for T in poses]
    cfg = P.Config(device=dev, reg_iter_n=20, track_on=True)
    nm = P.NeuralPoints(cfg)
    torch.manual_seed(42)
    dec = P.Decoder(cfg, 64, 1, 1).to(dev)
    tracker = P.Tracker(cfg, nm, dec)
    mapper = P.Mapper(cfg, None, nm, dec)
    loop = FrameLoop(cfg, nm, dec, tracker, mapper, build_index=True)
    for k in range(frames - 1):
        loop.frame(scans[k])
    torch.cuda.synchronize()
    # the last frame's tracking, instrumented
    stats = {}

    def timed(name, fn):
        def wrap(*a, **kw):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn(*a, **kw)
            torch.cuda.synchronize()
            stats.setdefault(name, []).append(time.perf_counter() - t0)
            return out
        return wrap
    TR.fused_query_sdf = timed("query_sdf", Q.query_sdf)
    tracker._register = timed("_register", tracker._register)
    TR.transform_points = timed("transform", TR.transform_points)
    loop.read_and_preprocess(scans[frames - 1])
    src = loop.cur_source_points
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    T, _, _, valid = tracker.tracking(src, loop.cur_pose_guess_torch, None, None)
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    print(f"source points {src.shape[0]}, tracking {total * 1e3:.3f} ms, valid {valid}")
    for k, v in stats.items():
        print(f"  {k:18s} n={len(v):3d} mean {statistics.mean(v) * 1e3:.4f} ms  total {sum(v) * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
