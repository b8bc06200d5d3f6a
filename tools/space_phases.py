#!/usr/bin/env python3
"""Phase times of one shard="space" Mapper.mapping call on the bench's configs[3] map, N ranks on
one GPU over gloo (launch with torch.distributed.run): partition build, per-iteration train_step /
halo exchanges / Adam, and the end-of-call reconciliation and all-gather of the owned rows."""
import collections
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import pin_slam_amd as P  # noqa: E402
import pin_slam_amd.sharding as SH  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_pool  # noqa: E402

T = collections.defaultdict(float)


def timed(obj, name, label):
    f = getattr(obj, name)

    def w(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = f(*a, **k)
        torch.cuda.synchronize()
        T[label] += time.perf_counter() - t0
        return r
    setattr(obj, name, w)


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = "cuda"
    nm, dec, pts = surface_map(bench.MAPPER_SIDE, device=dev, buffer_size=int(5e7), nn_k=8, weighted_first=True,
                               query_backend="grid", bs=bench.MAPPER_BS)
    for p in dec.parameters():
        p.requires_grad_(False)
    coord, label, ts = surface_pool(pts, bench.MAPPER_POOL, seed=11 + rank, device=dev)
    mapper = P.Mapper(nm.config, None, nm, dec, group=dist.group.WORLD, shard="space")
    mapper.set_pool(coord, label, ts)
    for n in ("exchange_gradients", "exchange_features", "reconcile_side_effects", "gather_owned"):
        timed(SH.SlabPartition, n, n)
    for n in ("_slab_partition", "train_step", "_adam", "_batch_index"):
        timed(mapper, n, n)
    mapper.mapping(1)
    T.clear()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    mapper.mapping(3)
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    print(f"rank {rank}/{world}: mapping(3) {total:.3f} s; " + ", ".join(f"{k} {v:.3f}" for k, v in T.items()),
          flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
