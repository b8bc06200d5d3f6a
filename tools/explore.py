#!/usr/bin/env python3
"""Timing experiments for the fused query kernel (what limits it?).  GPU only."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def morton_order(q, res=0.3):
    g = torch.floor(q / res).long()
    g = g - g.min(0)[0]
    key = torch.zeros(q.shape[0], dtype=torch.long, device=q.device)
    for b in range(16):
        for a in range(3):
            key |= ((g[:, a] >> b) & 1) << (3 * b + a)
    return torch.argsort(key)


def main():
    N = 262144
    for B in (int(5e7),):
        for backend in ("hash", "grid"):
            nm, dec, pts = surface_map(1000, buffer_size=B, query_backend=backend)
            q = surface_queries(pts, N)
            if backend == "grid":
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                nm.occupancy()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                nm.compact_records("global", True)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                print(f"grid build: occupancy {1e3*(t1-t0):.2f} ms (incl. host sync), compact {1e3*(t2-t1):.2f} ms",
                      flush=True)
            perm = morton_order(q)
            qs = q[perm].contiguous()
            for name, qq in (("random", q), ("morton", qs)):
                for grad in (True, False):
                    ms = timeit(lambda: P.query_sdf(nm, dec, qq, query_locally=False, want_grad=grad,
                                                    want_certainty=False))
                    print(f"{backend:5s} {name:7s} grad={int(grad)} {ms*1e3:8.1f} us  {N/ms/1e3:8.1f} Mq/s",
                          flush=True)
            for wf in (False,):
                ms = timeit(lambda: P.query_sdf(nm, dec, q, query_locally=False, want_grad=True,
                                                want_certainty=False, weighted_first=wf, want_std=True))
                print(f"{backend:5s} nwf     grad=1 {ms*1e3:8.1f} us  {N/ms/1e3:8.1f} Mq/s", flush=True)
            qt = q.clone().requires_grad_(True)

            def dropin():
                f, _, w, _, _ = nm.query_feature(qt, training_mode=False, query_locally=False)
                s_ = dec.sdf(f)
                return torch.autograd.grad(s_, qt, torch.ones_like(s_))[0]
            ms = timeit(dropin)
            print(f"{backend:5s} drop-in query_feature+Decoder+autograd {ms*1e3:8.1f} us", flush=True)
            del nm
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
