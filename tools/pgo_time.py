#!/usr/bin/env python3
"""Kernel time of the after-PGO SDF+grad query (model/neural_points.py:606-607: neighbour vectors
rotated by the points' quaternions) at the headline size, for each tools/exp_libs variant
(PIN_LIB) -- GPU box."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from tests import helpers as H  # noqa: E402

for wf in (True, False):
    nm, dec, pts = H.surface_map(1000, device="cuda", buffer_size=int(5e7), weighted_first=wf)
    g = torch.Generator(device="cpu").manual_seed(3)
    q = torch.randn(pts.shape[0], 4, generator=g) * torch.tensor([1.0, 0.05, 0.05, 0.05])
    nm.point_orientations = (q / q.norm(dim=1, keepdim=True)).to("cuda")
    nm.after_pgo = True
    x = H.surface_queries(pts, 262144, seed=7, device="cuda")

    def run():
        return P.query_sdf(nm, dec, x, query_locally=False, want_grad=True, want_certainty=False,
                           want_std=not wf, out_order="tile")
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(30):
        out = run()
    e.record()
    torch.cuda.synchronize()
    print(f"after_pgo wf={int(wf)}: {s.elapsed_time(e) / 30 * 1e3:.1f} us per 262144-query step (sort + query), "
          f"finite {bool(torch.isfinite(out[0]).all())}", flush=True)
