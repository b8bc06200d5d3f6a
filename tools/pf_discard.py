#!/usr/bin/env python3
"""The process_frame leg's slow frame (bench.py process_frame_leg, frame 29: the first window
filter whose pool exceeds pool_capacity, i.e. the capacity discards) under torch.profiler: per op
host / device time and the allocator's hipMalloc calls."""
import os
import sys
import time
import types

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_scan  # noqa: E402


def main(upto=29):
    dev = "cuda"
    nm, dec, pts = surface_map(1000, device=dev, buffer_size=int(5e7))
    cfg = nm.config
    cfg.bs_new_sample = 2048
    cfg.pool_filter_freq = 10
    cfg.track_on = True
    T = upto + 1
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
    for k in range(upto):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mapper.process_frame(frames[k], None, pose_t[k], k)
        torch.cuda.synchronize()
        print(f"frame {k}: {(time.perf_counter() - t0) * 1e3:.3f} ms, pool {mapper.pool_sample_count}", flush=True)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        t0 = time.perf_counter()
        mapper.process_frame(frames[upto], None, pose_t[upto], upto)
        torch.cuda.synchronize()
    print(f"frame {upto}: {(time.perf_counter() - t0) * 1e3:.3f} ms (profiled), pool {mapper.pool_sample_count}, "
          f"capacity {cfg.pool_capacity}")
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25, max_name_column_width=60))
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=15, max_name_column_width=60))


if __name__ == "__main__":
    main()
