#!/usr/bin/env python3
"""Host-side cost of one query_sdf call (tiny batch: the GPU work is negligible), and of its parts."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd import query as Q  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402


def per_call(fn, reps=2000):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    nm, dec, pts = surface_map(300, buffer_size=1 << 22, query_backend="grid")
    for n in (1000, 70000):
        q = surface_queries(pts, n)
        print(f"n={n}: query_sdf {per_call(lambda: P.query_sdf(nm, dec, q, query_locally=False, want_certainty=False)):.1f} us/call")
    q = surface_queries(pts, 70000)
    print(f"_views {per_call(lambda: nm._views('global', False)):.1f} us")
    print(f"mlp_view {per_call(lambda: Q.mlp_view(dec)):.1f} us")
    print(f"backend {per_call(lambda: nm.backend()):.1f} us")
    print(f"grid_view {per_call(lambda: nm.grid_view('global', True)):.1f} us")
    gv = nm.grid_view('global', True)
    print(f"query_sort {per_call(lambda: Q.query_sort(gv, q)):.1f} us")
    print(f"torch.empty x5 {per_call(lambda: [torch.empty(70000, device='cuda') for _ in range(5)]):.1f} us")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def pieces():
    from pin_slam_amd import _lib
    nm, dec, pts = surface_map(300, buffer_size=1 << 22, query_backend="grid")
    q = surface_queries(pts, 70000)
    gv = nm.grid_view('global', True)
    dev = q.device
    print(f"current_stream() {per_call(lambda: torch.cuda.current_stream()):.2f} us")
    print(f"current_stream(dev) {per_call(lambda: torch.cuda.current_stream(dev)):.2f} us")
    print(f"_lib.stream() {per_call(lambda: _lib.stream()):.2f} us")
    print(f"_lib.ptr {per_call(lambda: _lib.ptr(q)):.2f} us")
    print(f"order_workspace {per_call(lambda: Q.order_workspace(70000, dev)):.2f} us")
    print(f"torch.empty q4 {per_call(lambda: torch.empty((70000, 4), dtype=torch.float32, device=dev)):.2f} us")
    ws = Q.order_workspace(70000, dev)
    q4 = torch.empty((70000, 4), dtype=torch.float32, device=dev)
    lib = _lib.load()
    s = _lib.stream()
    print(f"raw ctypes sort {per_call(lambda: lib.pin_query_sort(gv.ref(), _lib.ptr(q), 70000, _lib.ptr(q4), None, _lib.ptr(ws), s)):.2f} us")
    print(f"gv.ref() {per_call(lambda: gv.ref()):.2f} us")
    print(f"mlp_view {per_call(lambda: Q.mlp_view(dec)):.2f} us")
    print(f"tensor_key4 {per_call(lambda: Q.tensor_key((q, q, q, q))):.2f} us")
    print(f"occupancy {per_call(lambda: nm.occupancy()):.2f} us")
    print(f"compact {per_call(lambda: nm.compact_records('global', True)):.2f} us")


if __name__ == "__main__" and "--pieces" in sys.argv:
    pieces()


def stream_submit():
    nm, dec, pts = surface_map(1000, buffer_size=int(5e7), query_backend="grid")
    q = surface_queries(pts, 262144)
    pipe = P.SdfQueryStream(nm, dec, query_locally=False, want_grad=True, want_certainty=False)
    ev = torch.cuda.Event()
    ev.record()
    for _ in range(20):
        pipe.submit(q, ev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        pipe.submit(q, ev)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"submit host {(t1 - t0) / 200 * 1e6:.1f} us, wall {(t2 - t0) / 200 * 1e6:.1f} us per batch")
    t0 = time.perf_counter()
    for _ in range(200):
        P.query_sdf(nm, dec, q, query_locally=False, want_grad=True, want_certainty=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"query_sdf host {(t1 - t0) / 200 * 1e6:.1f} us, wall {(t2 - t0) / 200 * 1e6:.1f} us per batch")


if __name__ == "__main__" and "--stream" in sys.argv:
    stream_submit()
