#!/usr/bin/env python3
"""Lean tile sort (PIN_SORT_LEAN) vs the standard sort, alone and streamed beside the query
kernel (QueryPipeline).  Per-step wall times over 200 batches."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd import _lib, query as Q  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    nm, dec, pts = surface_map(1000, buffer_size=int(5e7), nn_k=8, query_backend="grid")
    q = surface_queries(pts, 262144)
    n = q.shape[0]
    gv = nm.grid_view("global", True)
    ws = Q.order_workspace(n, q.device)
    q4 = torch.empty((n, 4), device=q.device)
    for flags, name in ((0, "standard"), (Q.SORT_LEAN, "lean")):
        us = timeit(lambda: _lib.call("pin_query_sort_ex", gv.ref(), _lib.ptr(q), n, _lib.ptr(q4), None, _lib.ptr(ws),
                                      flags, _lib.stream()))
        print(f"sort {name}: {us:.1f} us per call", flush=True)
    us = timeit(lambda: P.query_sdf(nm, dec, q, query_locally=False, want_grad=True, want_certainty=False,
                                    out_order="tile"))
    print(f"serial step (standard sort + query): {us:.1f} us", flush=True)
    pipe = P.QueryPipeline(nm, dec, n)

    def run(k):
        pipe.sort(q)
        for i in range(k):
            if i + 1 < k:
                pipe.sort(q)
            pipe.query()
    for k in (50, 200):
        run(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(k)
        torch.cuda.synchronize()
        print(f"streamed k={k}: {(time.perf_counter() - t0) / k * 1e6:.1f} us per batch", flush=True)


if __name__ == "__main__":
    main()
