#!/usr/bin/env python3
"""Host/device attribution of one Tracker.registration_step on the bench's configs[2] setup:
wall time of the whole step and of its pieces (each piece synchronised on its own)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd import _lib, tracker as TR  # noqa: E402
from pin_slam_amd.query import query_sdf  # noqa: E402
from pin_slam_amd.synthetic import surface_map, train_surface  # noqa: E402


def wall(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    dev = "cuda"
    nm, dec, pts = surface_map(bench.N_SIDE, device=dev, buffer_size=int(5e7))
    g = torch.Generator(device="cpu").manual_seed(5)
    centre = pts.mean(0)
    near = pts[((pts[:, :2] - centre[:2]) ** 2).sum(1) < 60.0 ** 2]
    src = near[torch.randint(0, near.shape[0], (bench.TRACKER_SRC,), generator=g)].float().to(dev)
    train_surface(nm, dec, pts, iters=100)
    cfg = nm.config
    tr = P.Tracker(cfg, nm, dec)
    zeros = torch.zeros(bench.TRACKER_SRC, device=dev)

    def step():
        return tr.registration_step(src, None, zeros, None, 0, cfg.reg_min_grad_norm, cfg.reg_max_grad_norm,
                                    cfg.reg_GM_dist_m, cfg.reg_GM_grad, cfg.reg_lm_lambda)

    def q():
        return query_sdf(nm, dec, src, query_locally=True, want_grad=True, want_std=not cfg.weighted_first,
                         want_certainty=False)
    sdf, grad, nn, _, std = q()
    prm = _lib.PinRegParams(min_nn_count=8, min_grad_norm=float(cfg.reg_min_grad_norm),
                            max_grad_norm=float(cfg.reg_max_grad_norm), max_sdf_std=1.0,
                            gm_dist=float(cfg.reg_GM_dist_m), gm_grad=float(cfg.reg_GM_grad))
    valid = torch.empty(src.shape[0], dtype=torch.uint8, device=dev)

    def reg():
        return TR._reg_accumulate(src, sdf, grad, nn, None, zeros, None, prm, valid)
    acc = reg()

    def solve():
        return TR._solve(acc, cfg.reg_lm_lambda, False, False, dev)
    cnt = int(acc[3])

    def gather():
        return src[torch.nonzero_static(valid, size=cnt).squeeze(1)]
    res = {"step": wall(step), "query_sdf": wall(q), "reg_accumulate(+D2H)": wall(reg), "solve(+H2D)": wall(solve),
           "valid gather": wall(gather)}
    print(" ".join(f"{k} {v:.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
