#!/usr/bin/env python3
"""Query order vs kernel time (GPU only): random, Morton-sorted, brick-binned."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402
from explore import timeit, morton_order  # noqa: E402


def main():
    N = 262144
    nm, dec, pts = surface_map(1000)
    q = surface_queries(pts, N)
    orders = {"random": q, "morton": q[morton_order(q)].contiguous()}
    g = torch.floor(q / 0.3).long() // 8
    key = (g[:, 0] - g[:, 0].min()) * 100000 + (g[:, 1] - g[:, 1].min()) * 100 + (g[:, 2] - g[:, 2].min())
    orders["bin8"] = q[torch.argsort(key)].contiguous()
    # slab per XCD only: 8 x-slabs, random order inside each (block b runs on XCD b % 8 and the
    # kernel's xcd_block() hands each XCD a contiguous eighth of the blocks)
    gx = torch.floor(q[:, 0] / 0.3)
    slab = ((gx - gx.min()) * 8 / (gx.max() - gx.min() + 1)).long()
    orders["slab8"] = q[torch.argsort(slab, stable=True)].contiguous()
    slab64 = ((gx - gx.min()) * 64 / (gx.max() - gx.min() + 1)).long()
    orders["slab64"] = q[torch.argsort(slab64, stable=True)].contiguous()
    gy = torch.floor(q[:, 1] / 0.3)
    for t in (16, 32):
        tx = ((gx - gx.min()) * t / (gx.max() - gx.min() + 1)).long()
        ty = ((gy - gy.min()) * t / (gy.max() - gy.min() + 1)).long()
        orders[f"tile{t * t}"] = q[torch.argsort(ty * t + tx, stable=True)].contiguous()
    for name, qq in orders.items():
        for grad in (True, False):
            ms = timeit(lambda: P.query_sdf(nm, dec, qq, query_locally=False, want_grad=grad, want_certainty=False))
            print(f"{name:7s} grad={int(grad)} {ms*1e3:8.1f} us  {N/ms/1e3:8.1f} Mq/s", flush=True)


if __name__ == "__main__":
    main()
