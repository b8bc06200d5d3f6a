#!/usr/bin/env python3
"""Debug: second-order gradients on an after-PGO map (random orientations), restated vs native."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd.query as Q  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402

dev = "cuda"
for restated in (True, False):
    Q._QF_RESTATED = restated
    nm, dec, pts = surface_map(120, device=dev, weighted_first=True, buffer_size=1 << 20, query_backend="grid")
    g = torch.Generator(device="cpu").manual_seed(13)
    quat = torch.randn(nm.neural_points.shape[0], 4, generator=g).to(dev)
    nm.point_orientations = quat / quat.norm(dim=1, keepdim=True)
    nm.local_point_orientations = nm.point_orientations.clone()
    nm.after_pgo = True
    q = surface_queries(pts, 3000, seed=5, device=dev).requires_grad_(True)
    feats = nm.local_geo_features
    print("restated", restated, "feats requires_grad", feats.requires_grad, type(feats))
    geo, _, wk, _, _ = nm.query_feature(q, None, training_mode=False)
    print("geo grad_fn", geo.grad_fn)
    sdf = dec.sdf(geo)
    gq, gfe = torch.autograd.grad(sdf.sum(), (q, feats), create_graph=True, allow_unused=True)
    print("gq", None if gq is None else gq.grad_fn, "gfe", None if gfe is None else gfe.grad_fn)
    loss = (gq * gq).sum()
    outs = torch.autograd.grad(loss, [feats, q], allow_unused=True)
    print([None if o is None else float(o.abs().max()) for o in outs])
