#!/usr/bin/env python3
"""Phase timestamps of the fused tile sort (experiment build -DPIN_SORT_STAMPS, PIN_LIB=...): per
block, s_memrealtime (100 MHz) at kernel entry, after the loads, after the LDS ranks, after the
returning atomics, after the grid barrier, after the totals' scan, after the placement."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd import _lib  # noqa: E402
from pin_slam_amd.query import query_sort  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402

nm, dec, pts = surface_map(1000, device="cuda")
q = surface_queries(pts, 262144, device="cuda")
gv = nm.grid_view("global", True)
for _ in range(20):
    query_sort(gv, q)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (128 * 8))()
_lib.load().pin_debug_sort_stamps(buf)
a = np.array(buf, dtype=np.int64).reshape(128, 8)[:64, :7]
t0 = a[:, 0].min()
rel = (a - t0) * 10 / 1000.0   # us (100 MHz ticks)
names = ["entry", "loaded", "ranked", "atomics", "barrier", "scanned", "placed"]
print("phase end, us after the first block's entry: min / median / max over the 64 blocks")
for k, nme in enumerate(names):
    print(f"  {nme:8s} {rel[:, k].min():7.2f} {np.median(rel[:, k]):7.2f} {rel[:, k].max():7.2f}")
