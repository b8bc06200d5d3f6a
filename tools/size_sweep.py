#!/usr/bin/env python3
"""Headline query kernel time vs batch size (tile-sorted rows, HIP events): does the time scale
with the number of waves (throughput-bound) or step with wave generations (latency-bound)?"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pin_slam_amd import _lib  # noqa: E402
from pin_slam_amd.query import mlp_view, query_sort  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402


def main():
    dev = "cuda"
    nm, dec, pts = surface_map(bench.N_SIDE, device=dev, buffer_size=int(5e7))
    gv = nm.grid_view("global", True)
    hv, pv = nm._views("global", False)
    mv = mlp_view(dec, packed=True)
    for n in (16384, 65536, 131072, 196608, 262144, 393216, 524288, 1048576):
        q = surface_queries(pts, n, device=dev)
        q4 = query_sort(gv, q)
        sdf = torch.empty(n, device=dev)
        grad = torch.empty((n, 3), device=dev)
        nn = torch.empty(n, dtype=torch.int32, device=dev)

        def launch():
            _lib.call("pin_query_sdf_grid_sorted", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q4), n, 8, 1, 0,
                      _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn), None, None, _lib.stream())
        for _ in range(5):
            launch()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(30)]
        for a, b in ev:
            a.record()
            launch()
            b.record()
        torch.cuda.synchronize()
        t = statistics.median(a.elapsed_time(b) for a, b in ev) * 1e3
        print(f"n {n:8d} waves {n // 64:6d} generations(2/SIMD) {n / 64 / 2048:5.2f} kernel {t:7.1f} us "
              f"{n / t / 1e3:6.2f} Gq/s", flush=True)


if __name__ == "__main__":
    main()
