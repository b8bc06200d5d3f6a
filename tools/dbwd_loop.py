#!/usr/bin/env python3
"""Second-order training loop through the drop-in query_feature, for a kernel trace: the
reference's analytic-eikonal mapping step written with autograd (get_gradient with create_graph,
utils/tools.py:174-184; BCE + eikonal, utils/mapper.py:448-573), ITERS times after one warm-up.
Run under `rocprofv3 --kernel-trace --stats`; kernels launched once per iteration show Calls equal
to a multiple of ITERS (a prime, so setup kernels stand apart)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402

ITERS = 17


def main():
    dev = "cuda"
    for wf in (True, False):
        nm, dec, pts = surface_map(200, device=dev, weighted_first=wf, buffer_size=1 << 22,
                                   query_backend="grid")
        q0 = surface_queries(pts, 65536, seed=3, device=dev)
        label = torch.randn(q0.shape[0], device=dev) * 0.1
        feats = nm.local_geo_features
        bce = torch.nn.BCEWithLogitsLoss()

        def step():
            q = q0.clone().requires_grad_(True)
            geo, _, wk, _, _ = nm.query_feature(q, None, training_mode=False)
            sdf = dec.sdf(geo)
            if not wf:
                sdf = torch.sum(sdf * wk, dim=1).squeeze(1)
            g, = torch.autograd.grad(sdf, q, torch.ones_like(sdf), create_graph=True)
            loss = bce(sdf / 0.1, torch.sigmoid(label / 0.1)) + 0.1 * ((g.norm(2, dim=-1) - 1.0) ** 2).mean()
            feats.grad = None
            loss.backward()
            return loss

        step()
        torch.cuda.synchronize()
        for _ in range(ITERS):
            loss = step()
        torch.cuda.synchronize()
        print(f"weighted_first={wf}: {ITERS} second-order steps, loss {float(loss):.5f}", flush=True)


if __name__ == "__main__":
    main()
