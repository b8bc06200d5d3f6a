#!/usr/bin/env python3
"""Where a Tracker.registration_step's time goes (GPU only)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import surface_map, train_surface  # noqa: E402
from pin_slam_amd import tracker as T  # noqa: E402


def wall(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    nm, dec, pts = surface_map(1000)
    train_surface(nm, dec, pts, iters=300)
    src = pts[torch.randint(0, pts.shape[0], (200000,))].cuda() + 0.01
    cfg = nm.config
    tr = P.Tracker(cfg, nm, dec)
    z = torch.zeros(200000, device="cuda")
    r = {}
    r["query_sdf"] = wall(lambda: P.query_sdf(nm, dec, src, query_locally=True, want_grad=True, want_std=False,
                                              want_certainty=False))
    r["registration_step"] = wall(lambda: tr.registration_step(src, None, z, None, 0, 0.5, 2.0, 0.5, 0.2, 1e-4))
    sdf, grad, nn, _, _ = P.query_sdf(nm, dec, src, query_locally=True, want_grad=True, want_certainty=False)
    from pin_slam_amd import _lib
    prm = _lib.PinRegParams(min_nn_count=8, min_grad_norm=0.5, max_grad_norm=2.0, max_sdf_std=1.0, gm_dist=0.5,
                            gm_grad=0.2)
    valid = torch.empty(200000, dtype=torch.uint8, device="cuda")
    r["reg_accumulate(+sync)"] = wall(lambda: T._reg_accumulate(src, sdf, grad, nn, None, None, None, prm, valid))
    r["bool-mask index"] = wall(lambda: src[valid.bool()])
    cnt = int(valid.sum())
    r["nonzero_static index"] = wall(lambda: src[torch.nonzero_static(valid, size=cnt).squeeze(1)])
    print({k: round(v, 1) for k, v in r.items()})


if __name__ == "__main__":
    main()
