"""Distinct feature rows per block of 256 processing slots in one mapping iteration (the bench
mapper leg's configuration): how much a per-block LDS pre-sum would cut the backward's atomics."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_pool  # noqa: E402

dev = "cuda"
WF = os.environ.get("WF", "1") != "0"
nm, dec, pts = surface_map(bench.MAPPER_SIDE, device=dev, buffer_size=int(5e7), nn_k=8, weighted_first=WF,
                           query_backend="grid", bs=bench.MAPPER_BS)
for p in dec.parameters():
    p.requires_grad_(False)
coord, label, ts = surface_pool(pts, bench.MAPPER_POOL, seed=11, device=dev)
mapper = P.Mapper(nm.config, None, nm, dec)
mapper.set_pool(coord, label, ts)
mapper.mapping(1)
ids = mapper._buf.ids
rows = ids.shape[0]
for blk in (64, 128, 256, 1024):
    nb = rows // blk
    x = ids[: nb * blk].reshape(nb, blk * ids.shape[1]).long()
    valid = (x >= 0).sum().item()
    xs, _ = torch.sort(torch.where(x >= 0, x, torch.full_like(x, -1)), dim=1)
    distinct = ((xs[:, 1:] != xs[:, :-1]) & (xs[:, 1:] >= 0)).sum().item() + (xs[:, 0] >= 0).sum().item()
    print(f"block {blk}: pairs {valid}  distinct per block summed {distinct}  factor {valid / distinct:.2f}")
