"""Multi-rank Mapper.mapping on the GPU: two ranks share cuda:0 over gloo (as
tools/rehearse_multi.sh does; the scaling run uses one rank per GPU over RCCL) and run the
whole fused mapping() call end to end with shard="dense" (the feature gradient reduce-scattered,
Adam on each rank's rows, the rows all-gathered -- sharding.OwnerAdam; the decoder's gradients
all-reduced) and shard="space" (slab ownership, halo exchange, shared row, Adam on owned
rows, all-gather of the owned rows).

Oracle: one process on the union of the same batches.  Every train_step of each rank is
recorded (pool rows drawn, row scales); the single process replays, per iteration, both ranks'
calls into one gradient accumulator with those scales and takes one Adam step over every row --
the data-parallel step the collectives must implement.  The replicas must end bit-identical to
each other; against the single process the features differ only by the float-atomic summation
order amplified by fresh Adam (a near-zero gradient moves an element by +-lr on its sign):
more than 1e-4 on at most 0.5 % of the elements and ||diff|| <= 3e-3 ||features moved|| (the
tolerances of tests/test_gpu_mapper.py's whole-call test), decoder 1e-4 relative, certainties
rel 1e-5 of their max, ts exact."""
import os
import socket
import warnings

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

ITERS = 4
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _state(nm, dec):
    return dict(feats=nm.local_geo_features.data.cpu().numpy().copy(),
                cert=nm.local_point_certainties.cpu().numpy().copy(),
                ts=nm.local_point_ts_update.cpu().numpy().copy(),
                dec=[p.detach().cpu().numpy().copy() for p in dec.parameters()])


def _worker(rank, world, port, case, shard, q, layout="auto"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from tests.replay import ReplayDraws
        from tests.test_gpu_mapper import _mapping_call_setup
        z = dict(np.load(os.path.join(GOLDEN, f"{case}.npz")))
        nm, dec, mapper, _ = _mapping_call_setup(z, "cuda", "grid")
        mapper.group = dist.group.WORLD
        mapper.shard = shard
        mapper.slab_layout = layout
        draws = ReplayDraws(7000 + 31 * rank)
        mapper._randint = lambda high, k: torch.from_numpy(draws.randint(high, k)).to("cuda")
        calls = []
        step, step_index = mapper.train_step, mapper._step_index

        # every iteration's batch passes _step_index (the dense loop calls it directly, train_step --
        # the slab path -- from inside, with the rank's scales, recorded after it)
        def recorded_index(coord, index, index_new, packed):
            full = index
            if index_new is not None:      # a batch split into history rows + new_idx[draw]
                new_sel, draw = index_new
                full = torch.cat((index, new_sel[draw]), dim=0)
            calls.append(dict(index=full.cpu().numpy(), scale=None, n_tail=0, scale_tail=0.0, world=world))
            return step_index(coord, index, index_new, packed)

        def recorded(*a, **kw):
            out = step(*a, **kw)
            calls[-1].update(scale=kw.get("scale"), n_tail=int(kw.get("n_tail", 0)),
                             scale_tail=float(kw.get("scale_tail", 0.0)), world=int(a[5]))
            return out
        mapper._step_index = recorded_index
        mapper.train_step = recorded
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            mapper.mapping(ITERS)
        torch.cuda.synchronize()
        part = getattr(mapper, "_partition", None)
        out = _state(nm, dec)
        out.update(calls=calls, warnings=[str(w.message) for w in caught],
                   part=None if part is None else dict(shape=part.shape, owned=int(part.owned.numel()),
                                                       halo=int(part.halo.numel()),
                                                       shared=part.shared.cpu().tolist()))
        q.put((rank, out))    # numpy only: tensors travel as shared-memory handles that die with this process
    except BaseException as e:           # report instead of leaving the parent waiting on the queue
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _single_process(case, calls, dev, world=WORLD):
    """The union of the ranks' batches in one process: per iteration every rank's train_step into
    one accumulator (reduce=False, the rank's scales), then one Adam step over all rows."""
    from tests.test_gpu_mapper import _mapping_call_setup
    from pin_slam_amd import _lib
    z = dict(np.load(os.path.join(GOLDEN, f"{case}.npz")))
    nm, dec, mapper, _ = _mapping_call_setup(z, dev, "grid")
    fdata = nm.local_geo_features.data
    feats0 = fdata.cpu().numpy().copy()
    f_grad, f_m, f_v = (torch.zeros_like(fdata) for _ in range(3))
    mlp_params = [p for p in dec.parameters() if p.requires_grad]
    m_grad = m_m = m_v = None
    if mlp_params:
        m_grad = torch.zeros((_lib.MLP_GRAD_SIZE,), dtype=torch.float32, device=dev)
        m_m, m_v = torch.zeros_like(m_grad), torch.zeros_like(m_grad)
    mapper._adam_t = 0
    for it in range(ITERS):
        for r in range(world):
            c = calls[r][it]
            scale = c["scale"] if c["scale"] is not None else 1.0 / c["world"]
            mapper.train_step(mapper.global_coord_pool, mapper.sdf_label_pool, mapper.time_pool, f_grad, m_grad, 1,
                              index=torch.from_numpy(c["index"]).to(dev), reduce=False, scale=scale, n_tail=c["n_tail"],
                              scale_tail=c["scale_tail"], weight=mapper.weight_pool)
        mapper._adam(fdata, f_grad, f_m, f_v, mlp_params, m_grad, m_m, m_v)
    torch.cuda.synchronize()
    return _state(nm, dec), feats0, mapper


def _run(case, shard, world=WORLD, layout="auto"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, shard, q, layout)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert isinstance(res[r], dict), f"rank {r}: {res[r]}"
    assert all(p.exitcode == 0 for p in procs)
    return res


def _norm(a):
    return float(np.linalg.norm(np.asarray(a, dtype=np.float64).ravel()))


@pytest.mark.parametrize("case,shard,world,layout", [("mapping_wf", "dense", 2, "auto"), ("mapping_wf", "dense", 4, "auto"),
                                                     ("mapping_nwf_weighted", "dense", 2, "auto"),
                                                     ("mapping_wf", "space", 2, "auto"),
                                                     ("mapping_wf_frozen", "space", 2, "auto"),
                                                     ("mapping_nwf_weighted", "space", 2, "auto"),
                                                     ("mapping_wf", "space", 4, (2, 2)),
                                                     ("mapping_wf_frozen", "space", 4, (2, 2))])
def test_multirank_mapping_equals_union_of_batches(case, shard, world, layout):
    """world 4 runs the 2-D cell path (2 x 2 cells, the bench's 8-GPU layout is 4 x 2): halo rows
    exchanged with up to three neighbours, the shared quirk row summed over four ranks."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    res = _run(case, shard, world, layout)
    r0 = res[0]
    calls = [res[r]["calls"] for r in range(world)]
    assert all(len(c) == ITERS for c in calls)
    if shard == "space":
        for r in range(world):
            assert res[r]["part"] is not None and not any("dense" in w for w in res[r]["warnings"]), res[r]["warnings"]
            assert res[r]["part"]["shared"] == [1]
            if world == 4:
                assert tuple(res[r]["part"]["shape"]) == (2, 2)
        assert sum(res[r]["part"]["owned"] for r in range(world)) == r0["feats"].shape[0] - 1
    else:
        assert r0["part"] is None
    # replicas agree bit for bit
    for r in range(1, world):
        for key in ("feats", "cert", "ts"):
            np.testing.assert_array_equal(r0[key], res[r][key], err_msg=key)
        for a, b in zip(r0["dec"], res[r]["dec"]):
            np.testing.assert_array_equal(a, b)
    ref, feats0, mapper = _single_process(case, calls, "cuda", world)
    if shard == "space":
        # the slab scales keep the union an unbiased estimate of one batch: sum_r scale_h,r bs_hist,r / bs_hist = 1
        c = mapper.config
        n_new = int(mapper.new_idx.numel())
        bs_hist = int(c.bs) - min(n_new, int(c.bs_new_sample))
        tot = sum(calls[r][0]["scale"] * (calls[r][0]["index"].size - calls[r][0]["n_tail"]) for r in range(world))
        assert tot / bs_hist == pytest.approx(1.0, rel=1e-9)
    moved = _norm(ref["feats"] - feats0)
    d = r0["feats"] - ref["feats"]
    frac = float((np.abs(d) > 1e-4).mean())
    assert frac <= 5e-3, frac
    assert _norm(d) <= 3e-3 * moved, (_norm(d), moved)
    for a, b in zip(r0["dec"], ref["dec"]):
        assert _norm(a - b) <= 1e-4 * max(_norm(b), 1e-12)
    np.testing.assert_allclose(r0["cert"], ref["cert"], rtol=1e-5, atol=1e-5 * float(np.abs(ref["cert"]).max()))
    np.testing.assert_array_equal(r0["ts"], ref["ts"])


# ------------------------------------------------------------------ point-sharded registration
def _reg_worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        out = _registration(case, "cuda", dist.group.WORLD)
        q.put((rank, out))
    except BaseException as e:
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _registration(case, dev, group):
    """One registration_step and a whole tracking loop on the tracker fixture (group: shard the
    source points over the group's ranks)."""
    from tests import helpers as H
    from pin_slam_amd.tracker import Tracker
    z = dict(np.load(os.path.join(GOLDEN, f"{case}.npz")))
    nm = H.neural_points_from_fixture(z, dev)
    nm.local_geo_features = torch.nn.Parameter(torch.as_tensor(z["local_features"], device=dev))
    dec = H.decoder_from_fixture(z, nm.config)
    cfg = nm.config
    cfg.surface_sample_range_m = float(z["surface_sample_range_m"])
    cfg.max_sdf_std_ratio = float(z["max_sdf_std_ratio"])
    cfg.reg_iter_n = int(z["reg_iter_n"])
    tr = Tracker(cfg, nm, dec, group=group)
    src = torch.as_tensor(z["source"], device=dev)
    T, _, _, _, valid, resid, _ = tr.registration_step(
        src, None, torch.zeros(src.shape[0], device=dev), None, 9, float(z["reg_min_grad_norm"]),
        float(z["reg_max_grad_norm"]), float(z["reg_GM_dist_m"]), float(z["reg_GM_grad"]), float(z["reg_lm_lambda"]))
    Tt, _, _, ok = tr.tracking(src, torch.eye(4, dtype=torch.float64, device=dev), cur_ts=9)
    return dict(T=T.cpu().numpy(), valid=valid.cpu().numpy(), resid=float(resid), Tt=Tt.cpu().numpy(), ok=bool(ok))


@pytest.mark.parametrize("case", ["tracker_wf", "tracker_nwf"])
def test_point_sharded_registration_equals_single_process(case):
    """Tracker(group=...) (the tracker's one exchange step): two ranks on cuda:0
    (gloo) each query half of the source points and SUM all-reduce the 31 normal-equation
    accumulators; the step's increment, residual and valid points, and the whole tracking loop's
    pose, equal the single-process ones (f64 sums in another order: 1e-9)."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reg_worker, args=(r, WORLD, port, case, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in range(WORLD))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(WORLD):
        assert isinstance(res[r], dict), f"rank {r}: {res[r]}"
    ref = _registration(case, "cuda", None)
    for r in range(WORLD):
        np.testing.assert_allclose(res[r]["T"], ref["T"], rtol=0, atol=1e-9)
        assert np.array_equal(res[r]["valid"], ref["valid"])
        assert res[r]["resid"] == pytest.approx(ref["resid"], rel=1e-9)
        np.testing.assert_allclose(res[r]["Tt"], ref["Tt"], rtol=0, atol=1e-7)
        assert res[r]["ok"] == ref["ok"]
