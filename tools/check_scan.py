#!/usr/bin/env python3
"""Exposure check of the production brick-window scan (What's weak 1): with a library
built with -DPIN_CHECK_SCAN=1 (PIN_LIB=...), every grid query runs the window scan (wave-major
LDS candidate list, aliased with the decoder scratch) AND the LDS-free per-cell scan, and poisons
the query (NaN outputs) when their counts, payloads or distances differ.  Runs the configs[1]
batch weighted-first and per-neighbour, repeated and under random permutations (different wave
compositions), and reports the poisoned queries (GPU box)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from tests import helpers as H  # noqa: E402

total = 0
for wf in (True, False):
    nm, dec, pts = H.surface_map(1000, device="cuda", buffer_size=int(5e7), weighted_first=wf)
    q = H.surface_queries(pts, 262144, seed=7, device="cuda")
    for rep in range(6):
        x = q if rep < 2 else q[torch.randperm(q.shape[0], generator=torch.Generator().manual_seed(rep)).to("cuda")]
        for order in ("tile", "input"):
            out = P.query_sdf(nm, dec, x.contiguous(), query_locally=False, want_grad=True, want_certainty=False,
                              want_std=not wf, out_order=order)
            bad = int(torch.isnan(out[0]).sum())
            total += bad
            print(f"wf={int(wf)} rep {rep} {order}: {bad} queries where the window scan != the per-cell scan",
                  flush=True)
print("TOTAL mismatches", total)
