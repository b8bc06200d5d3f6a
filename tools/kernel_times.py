#!/usr/bin/env python3
"""HIP-event times of the sorted SDF kernel alone for (weighted_first, gradient) variants on the
headline workload (262,144 queries, 1M-point map); PIN_LIB selects a variant library."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pin_slam_amd import _lib  # noqa: E402
from pin_slam_amd.query import mlp_view, query_sort  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402


def main():
    reps = 30
    sizes = [int(x) for x in os.environ.get("KT_SIZES", "262144").split(",")]
    wfs = [bool(int(x)) for x in os.environ.get("KT_WF", "1,0").split(",")]
    for wf, nq in [(w, s) for w in wfs for s in sizes]:
        nm, dec, pts = surface_map(1000, buffer_size=int(5e7), nn_k=8, weighted_first=wf, query_backend="grid")
        q = surface_queries(pts, nq)
        n = q.shape[0]
        gv = nm.grid_view("global", True)
        hv, pv = nm._views("global", False)
        mv = mlp_view(dec, packed=True)
        q4 = query_sort(gv, q)
        sdf = torch.empty(n, device=q.device)
        grad = torch.empty((n, 3), device=q.device)
        nn = torch.empty(n, dtype=torch.int32, device=q.device)
        std = torch.empty(n, device=q.device)
        for g in (True, False):
            def launch():
                _lib.call("pin_query_sdf_grid_sorted", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q4), n, 8, int(wf), 0,
                          _lib.ptr(sdf), _lib.ptr(grad) if g else None, _lib.ptr(nn), None,
                          None if wf else _lib.ptr(std), _lib.stream())
            for _ in range(3):
                launch()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for a, b in ev:
                a.record()
                launch()
                b.record()
            torch.cuda.synchronize()
            t = statistics.median(a.elapsed_time(b) for a, b in ev) * 1e3
            print(f"{os.path.basename(os.environ.get('PIN_LIB', 'default'))} n={n} wf={int(wf)} grad={int(g)} {t:.1f} us",
                  flush=True)


if __name__ == "__main__":
    main()
