#!/usr/bin/env python3
"""Valid-point census of the bench's tracker leg: nn counts, gradient norms and the kernel's
valid count, on a fresh fitted map and again after a global (query_locally=False) query."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.query import query_sdf  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries, train_surface  # noqa: E402


def census(tag, nm, dec, src, cfg):
    sdf, grad, nn, _, _ = query_sdf(nm, dec, src, query_locally=True, want_grad=True, want_certainty=False)
    gn = grad.norm(dim=1)
    tr = P.Tracker(cfg, nm, dec)
    zeros = torch.zeros(src.shape[0], device=src.device)
    out = tr.registration_step(src, None, zeros, None, 0, cfg.reg_min_grad_norm, cfg.reg_max_grad_norm,
                               cfg.reg_GM_dist_m, cfg.reg_GM_grad, cfg.reg_lm_lambda)
    print(f"{tag}: nn>=k {(nn >= cfg.query_nn_k).sum().item()} nn>0 {(nn > 0).sum().item()} "
          f"|g| min {gn.min().item():.3g} med {gn.median().item():.3g} max {gn.max().item():.3g} "
          f"in range {((gn > cfg.reg_min_grad_norm) & (gn < cfg.reg_max_grad_norm)).sum().item()} "
          f"sdf med {sdf.abs().median().item():.3g} valid {out[4].shape[0]} "
          f"grad range ({cfg.reg_min_grad_norm}, {cfg.reg_max_grad_norm})", flush=True)


def main():
    dev = "cuda"
    nm, dec, pts = surface_map(bench.N_SIDE, device=dev, buffer_size=int(5e7), nn_k=8, weighted_first=True)
    cfg = nm.config
    g = torch.Generator(device="cpu").manual_seed(5)
    centre = pts.mean(0)
    near = pts[((pts[:, :2] - centre[:2]) ** 2).sum(1) < 60.0 ** 2]
    src = near[torch.randint(0, near.shape[0], (bench.TRACKER_SRC,), generator=g)].float().to(dev)
    census("unfitted", nm, dec, src, cfg)
    q = surface_queries(pts, 262144, device=dev)
    query_sdf(nm, dec, q, query_locally=False, want_grad=True)
    census("after global query", nm, dec, src, cfg)
    f0 = nm.geo_features.detach().clone()
    w0 = [p.detach().clone() for p in dec.parameters()]
    loss = train_surface(nm, dec, pts, iters=300)
    print("fit loss", loss, flush=True)
    print("global features moved", (nm.geo_features - f0).abs().max().item(),
          "local == global", torch.equal(nm.local_geo_features.data[:-1], nm.geo_features[:-1]),
          "decoder moved", max((p - q).abs().max().item() for p, q in zip(dec.parameters(), w0)), flush=True)
    census("fitted", nm, dec, src, cfg)
    nm._cache = {}
    for k in ("_grid_view_cache", "_view_cache"):
        nm.__dict__.pop(k, None)
    census("fitted, caches cleared", nm, dec, src, cfg)
    # the fit's own training rows: sdf vs label
    from pin_slam_amd.synthetic import surface_pool
    coord, label, _ = surface_pool(pts, 4096, seed=3, device=dev)
    sdf, grad, nn, _, _ = query_sdf(nm, dec, coord, query_locally=True, want_grad=True, want_certainty=False)
    print("pool rows: corr(sdf, label)", torch.corrcoef(torch.stack([sdf, label]))[0, 1].item(),
          "sdf std", sdf.std().item(), "label std", label.std().item(), flush=True)


if __name__ == "__main__":
    main()
