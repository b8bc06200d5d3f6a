#!/usr/bin/env python3
"""Does gloo take device tensors for reduce_scatter_tensor / all_gather_into_tensor (in place)
with async_op?  Two ranks on cuda:0 (the 1-GPU multirank tests run sharding.OwnerAdam this way)."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def w(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    x = torch.arange(8, dtype=torch.float32, device="cuda") + rank * 100
    out = torch.empty(4, device="cuda")
    try:
        dist.reduce_scatter_tensor(out, x, async_op=True).wait()
        print(rank, "reduce_scatter_tensor cuda ok", out.cpu().tolist(), flush=True)
    except Exception as e:
        print(rank, "reduce_scatter_tensor cuda FAIL", repr(e)[:200], flush=True)
    buf = torch.zeros(8, device="cuda")
    buf[rank * 4:(rank + 1) * 4] = rank + 1
    try:
        dist.all_gather_into_tensor(buf, buf[rank * 4:(rank + 1) * 4], async_op=True).wait()
        print(rank, "all_gather_into_tensor cuda ok", buf.cpu().tolist(), flush=True)
    except Exception as e:
        print(rank, "all_gather_into_tensor cuda FAIL", repr(e)[:200], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(w, args=(2, int(sys.argv[1]) if len(sys.argv) > 1 else 29655), nprocs=2)
