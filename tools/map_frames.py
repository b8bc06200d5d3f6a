#!/usr/bin/env python3
"""bench.py's map_update leg alone, twice over (fresh map each time), printing every frame's time
(GPU only) -- to find where an outlier frame comes from (run under rocprofv3 --hip-trace to see the
runtime calls of the slow frame)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


class A:
    steps = 20
    no_cpu_baseline = True


for rep in range(2):
    r = bench.map_leg(A, "cuda", 1, 0)
    print(f"run {rep}: mean {r['ms_per_frame']:.3f} ms, median {r['median_ms_per_frame']:.3f} ms, frames "
          f"{r['frame_ms']}, map {r['map_points_before']} -> {r['map_points_after']}", flush=True)
    torch.cuda.synchronize()
