"""Data-parallel mapping logic on CPU with gloo, world_size 2.

Each rank takes half of a reference mapper batch, computes its gradients with the oracle
scaled by 1/world (what pin_train_backward's grad_scale does on the GPU), and runs the
package's own collectives (pin_slam_amd.mapper.allreduce_gradients / sync_side_effects).
The result must equal the single-process gradient and side effects of the whole batch:
the mean loss over the union of equal halves is the mean of the halves' means, and with a
half size divisible by gradient_decimation the ranks' stencil rows partition the full
batch's.  Also covers bench.py's max-over-ranks timing reduction."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import pin_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _grads(case, rows=None):
    z = np.load(os.path.join(GOLDEN, f"{case}.npz"))
    st = O.map_from_fixture(z)
    mlp = O.mlp_from_fixture(z)
    dx = O.neighbor_offsets(int(z["num_nei_cells"]), float(z["search_alpha"]))
    coord, label, ts = z["it0_coord"], z["it0_label"], z["it0_ts"]
    if rows is not None:
        coord, label, ts = coord[rows], label[rows], ts[rows]
    cert0 = st.local_certainties.copy()
    out = O.mapper_forward_backward(st, mlp, coord, label, ts, int(z["nn_k"]), dx, float(z["map_max_valid_dist2"]),
                                    bool(z["weighted_first"]), float(z["sigma"]), float(z["weight_e"]),
                                    int(z["gradient_decimation"]), float(z["num_grad_eps"]))
    flat = np.concatenate([out["mlp_grads"][k].reshape(-1) for k in ("W1", "b1", "W2", "b2")])
    return out["feat_grad"].astype(np.float64), flat.astype(np.float64), cert0, st.local_certainties, \
        st.local_ts_update, out["loss"]


def _worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pin_slam_amd.mapper import allreduce_gradients, sync_side_effects
        n = 2000
        half = n // world
        fg, mg, cert0, cert, ts, loss = _grads(case, np.arange(rank * half, (rank + 1) * half))
        fg_t = torch.from_numpy(fg / world)
        mg_t = torch.from_numpy(mg / world)
        allreduce_gradients([fg_t, mg_t, None])
        # gradients in the mapper's 64-B accumulator rows (lanes 0..7; lane 8 = certainty delta)
        acc = torch.zeros((fg.shape[0], 16), dtype=torch.float64)
        acc[:, :8] = torch.from_numpy(fg / world)
        acc[:-1, 8] = torch.from_numpy((cert - cert0).astype(np.float64))
        allreduce_gradients([acc])
        assert torch.equal(acc[:, :8], fg_t), "packed lanes must reduce like the plain gradient"
        cert_delta = acc[:-1, 8].contiguous()
        ts_t = torch.from_numpy(ts.astype(np.int64))
        sync_side_effects(cert_delta, ts_t)
        cert_t = torch.from_numpy(cert0.astype(np.float64)) + cert_delta
        lt = torch.tensor([loss / world], dtype=torch.float64)
        dist.all_reduce(lt)
        tm = torch.tensor([1.0 + rank], dtype=torch.float64)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put((fg_t.numpy(), mg_t.numpy(), cert_t.numpy(), ts_t.numpy(), float(lt), float(tm)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["mapper_wf", "mapper_nwf"])
def test_data_parallel_mapping_equals_single_process(case):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        fg, mg, cert, ts, loss, tmax = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    fg1, mg1, _, cert1, ts1, loss1 = _grads(case)
    np.testing.assert_allclose(fg, fg1, rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(mg, mg1, rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(cert, cert1, rtol=1e-6, atol=1e-5)
    np.testing.assert_array_equal(ts, ts1)
    assert loss == pytest.approx(loss1, rel=1e-9)
    assert tmax == 2.0
