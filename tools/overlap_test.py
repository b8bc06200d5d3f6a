#!/usr/bin/env python3
"""Does the tile sort of batch i+1 overlap the query kernel of batch i when it runs on a second
(high-priority) stream?  Wall time per batch, serial vs two streams."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pin_slam_amd import _lib  # noqa: E402
from pin_slam_amd.query import mlp_view, order_workspace  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402


def main():
    nm, dec, pts = surface_map(1000, buffer_size=int(5e7), nn_k=8, query_backend="grid")
    q = surface_queries(pts, 262144)
    n = q.shape[0]
    dev = q.device
    gv = nm.grid_view("global", True)
    hv, pv = nm._views("global", False)
    mv = mlp_view(dec)
    sdf = torch.empty(n, device=dev)
    grad = torch.empty((n, 3), device=dev)
    nn = torch.empty(n, dtype=torch.int32, device=dev)
    q4 = [torch.empty((n, 4), device=dev) for _ in range(2)]
    lib = _lib.load()

    def sort(b, s):
        ws = order_workspace(n, dev, stream_handle=s.value)
        lib.pin_query_sort(gv.ref(), _lib.ptr(q), n, _lib.ptr(q4[b]), None, _lib.ptr(ws), s)

    def query(b, s):
        lib.pin_query_sdf_grid_sorted(gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q4[b]), n, 8, 1, 0, _lib.ptr(sdf),
                                      _lib.ptr(grad), _lib.ptr(nn), None, None, s)

    main_s = torch.cuda.current_stream()
    mh = _lib.stream()
    for prio in (0, -1):
        side = torch.cuda.Stream(priority=prio)
        sh = torch.ctypes = None
        from ctypes import c_void_p
        sh = c_void_p(side.cuda_stream)
        sorted_ev = [torch.cuda.Event(), torch.cuda.Event()]
        free_ev = [torch.cuda.Event(), torch.cuda.Event()]
        for mode in ("serial", "overlap"):
            N = 300
            torch.cuda.synchronize()
            for rep in range(2):
                t0 = time.perf_counter()
                for k in range(N):
                    b = k & 1
                    if mode == "serial":
                        sort(b, mh)
                        query(b, mh)
                    else:
                        side.wait_event(free_ev[b])
                        sort(b, sh)
                        sorted_ev[b].record(side)
                        main_s.wait_event(sorted_ev[b])
                        query(b, mh)
                        free_ev[b].record(main_s)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
            print(f"prio {prio} {mode}: host {(t1 - t0) / N * 1e6:.1f} us, wall {(t2 - t0) / N * 1e6:.1f} us per batch",
                  flush=True)


if __name__ == "__main__":
    main()
