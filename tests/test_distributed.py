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


# ------------------------------------------------------------------ spatially sharded mapping
def _shard_setup(nx=120, ny=40):
    """A small all-local oracle map (surface grid nx x ny at 0.3 m), the mapper fixture's decoder
    and two seeded batches: surface points + N(0, 0.25^2) along z, label = -offset."""
    z = np.load(os.path.join(GOLDEN, "mapper_wf.npz"))
    mlp = O.mlp_from_fixture(z)
    res = 0.3
    xs, ys = np.meshgrid((np.arange(nx) + 0.5) * res, (np.arange(ny) + 0.5) * res, indexing="ij")
    pts = np.stack([xs.ravel(), ys.ravel(), 0.5 * np.sin(xs.ravel() / 7) * np.cos(ys.ravel() / 5) + 0.15], -1)
    st = O.empty_map(res, 1 << 20, np.zeros(1, np.float32), 1e9)
    O.map_update(st, pts.astype(np.float32), 0)
    O.reset_local_map(st, np.array([nx * res / 2, ny * res / 2, 0.0]), 0, 1e6)
    rng = np.random.default_rng(3)
    st.local_features[:-1] = rng.normal(0, 0.05, st.local_features[:-1].shape).astype(np.float32)
    batches = []
    for it in range(2):
        idx = rng.integers(0, st.points.shape[0], 1600)
        off = rng.normal(0, 0.25, 1600).astype(np.float32)
        coord = st.points[idx].copy()
        coord[:, 2] += off
        batches.append((coord, -off, np.zeros(1600, np.int64)))
    cfg = dict(nn_k=8, neighbor_dx=O.neighbor_offsets(2, 0.2), maxd2=float(3 * (3 * res) ** 2),
               weighted_first=True, sigma=float(z["sigma"]), weight_e=0.5, decimation=10, eps=0.06, lr=0.01)
    return st, mlp, batches, cfg


def _rank_grad(st, mlp, batch, mask, cfg, n_total):
    """Oracle forward/backward of one rank's rows (st mutated: its side effects), scaled so that the
    ranks' gradients add up to the gradient of the sum of their means weighted by rows."""
    coord, label, ts = batch
    out = O.mapper_forward_backward(st, mlp, coord[mask], label[mask], ts[mask], cfg["nn_k"], cfg["neighbor_dx"],
                                    cfg["maxd2"], cfg["weighted_first"], cfg["sigma"], cfg["weight_e"],
                                    cfg["decimation"], cfg["eps"])
    return out["feat_grad"].astype(np.float32) * np.float32(mask.sum() / n_total)


def _shard_worker(rank, world, port, q, grid, layout):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pin_slam_amd.sharding import SlabPartition
        st, mlp, batches, cfg = _shard_setup(*grid)
        reach = float(np.sqrt(cfg["maxd2"])) * 1.001 + cfg["eps"] + 1e-3
        part = SlabPartition(torch.from_numpy(st.local_points), reach, layout=layout)
        feats = torch.from_numpy(st.local_features)        # shares memory with the oracle state
        m, v = torch.zeros_like(feats), torch.zeros_like(feats)
        cert_before = torch.from_numpy(st.local_certainties.copy())
        owned = part.adam_rows.numpy()        # owned rows + the shared row (Adam by every rank)
        masks = []
        for it, batch in enumerate(batches):
            mask = part.sample_mask(torch.from_numpy(batch[0])).numpy()
            masks.append(mask)
            g = torch.from_numpy(_rank_grad(st, mlp, batch, mask, cfg, batch[0].shape[0]))
            part.exchange_gradients(g)
            p_o, g_o, m_o, v_o = (t.numpy()[owned].copy() for t in (feats, g, m, v))
            O.adam_step(p_o, g_o, m_o, v_o, it + 1, cfg["lr"])
            for t, val in ((feats, p_o), (m, m_o), (v, v_o)):
                t.numpy()[owned] = val
            part.exchange_features(feats)
        cert = torch.from_numpy(st.local_certainties)
        ts = torch.from_numpy(st.local_ts_update)
        part.reconcile_side_effects(cert_before, cert, ts)
        part.gather_owned(feats, cert, ts)
        q.put((rank, feats.numpy().copy(), cert.numpy().copy(), ts.numpy().copy(), masks,
               int(part.owned.numel()), int(part.halo.numel()), part.shape))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,grid,layout,shape", [(2, (120, 40), "auto", (2, 1)),
                                                    (4, (60, 60), "auto", (2, 2)),
                                                    (4, (60, 60), "1d", (4, 1)),
                                                    (8, (100, 80), "auto", (4, 2))])
def test_slab_sharded_mapping_equals_dense_data_parallel(world, grid, layout, shape):
    """shard='space' (pin_slam_amd.sharding): halo gradients to owners, Adam on owned rows (and
    the shared row), halo features refreshed, side effects reconciled, owned rows all-gathered --
    equals the dense data-parallel step on the same per-rank batches (sum of the ranks'
    gradients, Adam on every row, summed certainty deltas, max ts) on every replica, over two
    iterations.  1-D slabs on a corridor, 2 x 2 cells on a square map (layout auto) and 4 strips
    on the same square map (layout 1d)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q, grid, layout)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    st, mlp, batches, cfg = _shard_setup(*grid)
    L = st.local_points.shape[0]
    assert all(r[7] == shape for r in res)
    assert sum(r[5] for r in res) == L and all(0 < r[6] < L // 2 for r in res)   # owners partition; small halos
    assert all(abs(r[5] - L / world) < 0.05 * L / world for r in res)            # equal-count cells
    m, v = np.zeros_like(st.local_features), np.zeros_like(st.local_features)
    cert0 = st.local_certainties.copy()
    cert_delta = np.zeros_like(cert0)
    ts = st.local_ts_update.copy()
    for it, batch in enumerate(batches):
        g = np.zeros_like(st.local_features)
        for r in range(world):
            sr = st.copy()
            sr.local_certainties[:] = 0
            g += _rank_grad(sr, mlp, batch, res[r][4][it], cfg, batch[0].shape[0])
            cert_delta += sr.local_certainties
            ts = np.maximum(ts, sr.local_ts_update)
        O.adam_step(st.local_features, g, m, v, it + 1, cfg["lr"])
    for r in range(world):
        np.testing.assert_allclose(res[r][1], st.local_features, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(res[r][2], cert0 + cert_delta, rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(res[r][3], ts)


def _plan_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pin_slam_amd.sharding import SlabPartition, slab_batch_plan
        st, _, _, cfg = _shard_setup(100, 80)
        reach = float(np.sqrt(cfg["maxd2"])) * 1.001 + cfg["eps"] + 1e-3
        part = SlabPartition(torch.from_numpy(st.local_points), reach)
        rng = np.random.default_rng(5)
        pool = torch.from_numpy(st.points[rng.integers(0, st.points.shape[0], 20000)])
        new_idx = torch.arange(15000, 20000)
        out = {"shape": part.shape}
        plan = slab_batch_plan(part, pool, new_idx, bs=4096, bs_new_sample=1024, new_mode=True)
        rows, new, scales = plan
        # this rank's draw: as many history / new rows as its share (any positive counts would do)
        bh = max(1, int(round(3072 * rows.numel() / 20000)))
        bn = max(1, int(round(1024 * new.numel() / 5000)))
        sh, sn = scales(bh, bn)
        out["full"] = (int(rows.numel()), int(new.numel()), bh * sh, bn * sn,
                       bool(part.sample_mask(pool[rows]).all()))
        # pool samples only left of the map's middle: the right-hand cells hold none
        left = pool[pool[:, 0] < float(st.points[:, 0].mean())]
        out["empty"] = slab_batch_plan(part, left, None, bs=4096, bs_new_sample=0, new_mode=False)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_slab_batch_plan_world8_and_dense_fallback():
    """slab_batch_plan (Mapper._slab_partition) on 8 ranks with the 4 x 2 cells of bench.py's 8-GPU
    mapper leg: the slabs' pool rows partition the pool, the scaled history / new rows of the
    ranks add up to one reference batch (3,072 + 1,024 rows); and when one cell holds no pool
    samples EVERY rank returns None (the call falls back to the dense all-reduce together)."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [r[1] for r in sorted(q.get(timeout=240) for _ in range(world))]
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(r["shape"] == (4, 2) for r in res)
    assert sum(r["full"][0] for r in res) == 20000 and sum(r["full"][1] for r in res) == 5000
    assert all(r["full"][0] > 0 and r["full"][4] for r in res)
    assert sum(r["full"][2] for r in res) == pytest.approx(3072, rel=1e-12)
    assert sum(r["full"][3] for r in res) == pytest.approx(1024, rel=1e-12)
    assert all(r["empty"] is None for r in res)


def _world_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import types
        from pin_slam_amd.mapper import Mapper
        from pin_slam_amd.tracker import Tracker
        q.put((rank, Mapper._world(types.SimpleNamespace()), Mapper._world(types.SimpleNamespace(group=None)),
               Mapper._world(types.SimpleNamespace(group=dist.group.WORLD)),
               Tracker._shard_range(types.SimpleNamespace(), 10), Tracker._shard_range(
                   types.SimpleNamespace(group=dist.group.WORLD), 10)))
    finally:
        dist.destroy_process_group()


def test_data_parallel_only_with_an_explicit_group():
    """An initialised default process group alone does not make a Mapper / Tracker data-parallel
    (bench.py's whole-frame leg runs one independent SLAM per rank: its mappers must not exchange
    gradients of differently sized maps); an explicit group does."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=120) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, w_none, w_none2, w_group, sh_none, sh_group in res:
        assert (w_none, w_none2, w_group) == (1, 1, 2)
        assert sh_none == (0, 10, 1)
        assert sh_group == ((0, 5, 2) if rank == 0 else (5, 10, 2))


# ------------------------------------------------------------------ dense step: owner Adam
def _adam_ref(p, g, m, v, t, first, lr=0.01, b1=0.9, b2=0.99, eps=1e-15):
    """torch.optim.Adam's update (utils/tools.py:89-116) on one contiguous piece, in place; the
    gradient is consumed (zeroed) as pin_adam_step's zero_grad does."""
    if first:
        m.zero_()
        v.zero_()
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    denom = (v.sqrt() / np.sqrt(1 - b2 ** t)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / (1 - b1 ** t))
    g.zero_()


def _rank_grads(n, extra, world, it):
    gens = [torch.Generator().manual_seed(1000 * it + r) for r in range(world)]
    return [torch.randn(n + extra, generator=gg, dtype=torch.float64) / world for gg in gens]


def _owner_worker(rank, world, port, n, extra, iters, buckets, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pin_slam_amd.sharding import OwnerAdam
        oa = OwnerAdam(n, None, buckets)
        params = torch.linspace(-1, 1, n, dtype=torch.float64)
        dec = torch.zeros(extra, dtype=torch.float64)
        grads = torch.zeros(n + extra, dtype=torch.float64)
        m = torch.empty(oa.moments_size(), dtype=torch.float64)
        v = torch.empty_like(m)
        dm, dv = torch.empty(extra, dtype=torch.float64), torch.empty(extra, dtype=torch.float64)
        for it in range(1, iters + 1):
            grads += _rank_grads(n, extra, world, it)[rank]     # this rank's backward (scaled 1/W)
            oa.step(params, grads, m, v, lambda p, g, mm, vv: _adam_ref(p, g, mm, vv, it, it == 1),
                    lambda: _adam_ref(dec, grads[n:], dm, dv, it, it == 1) if extra else None)
            assert not grads.any(), "the gradient buffer must be consumed"
        q.put((rank, params.numpy(), dec.numpy(), oa.buckets, oa.rest))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("n,extra,buckets", [(8 * 40001, 833, 4), (8 * 4096, 0, 3), (8 * 7, 5, 4)])
def test_owner_adam_equals_single_process_adam(world, n, extra, buckets):
    """Mapper's data-parallel dense step (mapper._owner_adam, sharding.OwnerAdam): reduce-scatter
    in buckets, Adam on the owned pieces, all-gather (plus the all-reduced rest and decoder tail),
    three iterations with fresh-moment first step, equals one process summing the ranks'
    gradients and stepping every element -- and leaves every replica bit-identical.  Sizes: a map
    whose rows do not fill the buckets evenly (rest + decoder tail), an exact split without a
    tail, and a map too small to split (everything in the all-reduced rest)."""
    iters = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_owner_worker, args=(r, world, port, n, extra, iters, buckets, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict((r, (a, b, nb, rest)) for r, a, b, nb, rest in (q.get(timeout=240) for _ in range(world)))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in range(1, world):
        np.testing.assert_array_equal(res[0][0], res[r][0])
        np.testing.assert_array_equal(res[0][1], res[r][1])
    params = torch.linspace(-1, 1, n, dtype=torch.float64)
    dec = torch.zeros(extra, dtype=torch.float64)
    m, v = torch.empty(n + extra, dtype=torch.float64), torch.empty(n + extra, dtype=torch.float64)
    for it in range(1, iters + 1):
        g = torch.stack(_rank_grads(n, extra, world, it)).sum(0)
        _adam_ref(params, g[:n], m[:n], v[:n], it, it == 1)
        _adam_ref(dec, g[n:], m[n:], v[n:], it, it == 1)
    np.testing.assert_allclose(res[0][0], params.numpy(), rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(res[0][1], dec.numpy(), rtol=1e-9, atol=1e-12)
    nb, rest = res[0][2], res[0][3]
    if n == 8 * 7:
        assert nb == 0 and rest == n
    else:
        assert nb == buckets and rest < buckets * world * 64
