#!/usr/bin/env python3
"""Where Mapper.process_frame's time goes (bench process_frame workload): sampler, map update,
pool append, window filter, certainty of the new samples -- wall time of each step with a sync."""
import os
import sys
import time
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_scan  # noqa: E402


def main():
    dev = "cuda"
    nm, dec, pts = surface_map(1000, device=dev, buffer_size=int(5e7))
    cfg = nm.config
    cfg.track_on = True
    T = 25
    nm.local_map_radius = 50.0
    nm.diff_travel_dist_local = 250.0
    nm.travel_dist = torch.arange(T, dtype=torch.float32, device=dev) * 2.0
    poses, frames = [], []
    for k in range(T):
        c = np.array([100.0 + 2.0 * k, 150.0, 1.7])
        pose = np.eye(4)
        pose[:3, 3] = c
        poses.append(pose)
        w = surface_scan(c[0], c[1], 50.0, 65536, seed=300 + k, device=dev)
        frames.append((w - torch.as_tensor(c, dtype=torch.float32, device=dev)).contiguous())
    ds = types.SimpleNamespace(odom_poses=poses, stop_status=False, gt_pose_provided=False)
    mapper = P.Mapper(cfg, ds, nm, dec)
    pose_t = [torch.as_tensor(p, device=dev) for p in poses]
    acc = {}
    orig_update = nm.update
    orig_sample = mapper.sampler.sample
    orig_cert = nm.query_certainty

    def timed(name, fn):
        def w(*a, **kw):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn(*a, **kw)
            torch.cuda.synchronize()
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
            return r
        return w
    nm.update = timed("update", orig_update)
    mapper.sampler.sample = timed("sample", orig_sample)
    nm.query_certainty = timed("certainty", orig_cert)
    for name in ("_pool_append", "_pool_compact", "_used_poses"):
        setattr(mapper, name, timed(name, getattr(mapper, name)))
    per_frame = []
    for k in range(T):
        if k == 5:
            acc.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        torch.cuda.synchronize()
        tf = time.perf_counter()
        mapper.process_frame(frames[k], None, pose_t[k], k)
        torch.cuda.synchronize()
        per_frame.append((time.perf_counter() - tf) * 1e3)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    n = T - 5
    print(f"total {tot / n * 1e3:.3f} ms/frame")
    for k, v in acc.items():
        print(f"  {k:14s} {v / n * 1e3:.3f} ms/frame")
    print("per frame ms:", " ".join(f"{v:.2f}" for v in per_frame))
    print("pool", mapper.pool_sample_count)


if __name__ == "__main__" and not os.environ.get("PROFILE"):
    main()


def profile():
    import cProfile
    import pstats
    cProfile.run("main()", "/tmp/pf.prof")
    st = pstats.Stats("/tmp/pf.prof")
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__" and os.environ.get("PROFILE"):
    profile()
