#!/usr/bin/env python3
"""Debug: the native double backward of query_feature (pin_query_feature_bwd2) against autograd over
the ATen restatement, output by output, for a loss on dL/dq only and on dL/dfeatures only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd.query as Q  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402

dev = "cuda"
for wf in (True, False):
    for which in ("q", "f", "both"):
        res = []
        for restated in (True, False):
            Q._QF_RESTATED = restated
            nm, dec, pts = surface_map(120, device=dev, weighted_first=wf, buffer_size=1 << 20, query_backend="grid")
            q = surface_queries(pts, 3000, seed=5, device=dev).requires_grad_(True)
            feats = nm.local_geo_features
            geo, _, wk, _, _ = nm.query_feature(q, None, training_mode=False)
            sdf = dec.sdf(geo)
            if not wf:
                sdf = torch.sum(sdf * wk, dim=1).squeeze(1)
            gq, gfe = torch.autograd.grad(sdf.sum(), (q, feats), create_graph=True)
            c1 = torch.linspace(-1.0, 1.0, gq.numel(), device=dev).view_as(gq)
            c2 = torch.linspace(0.5, -0.5, gfe.numel(), device=dev).view_as(gfe)
            loss = 0.0
            if which in ("q", "both"):
                loss = loss + (gq * c1).sum()
            if which in ("f", "both"):
                loss = loss + (gfe * c2).sum()
            outs = torch.autograd.grad(loss, [feats, q] + list(dec.parameters()), allow_unused=True)
            res.append([o if o is not None else torch.zeros(1, device=dev) for o in outs])
        names = ["feats", "q", "W1", "b1", "W2", "b2"]
        for nme, a, b in zip(names, *res):
            d = (a - b).abs().max().item()
            print(f"wf={wf} loss on {which:4s} {nme:5s} max|restated|={a.abs().max().item():.3e} max|diff|={d:.3e}")
