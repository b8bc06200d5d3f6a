"""The deterministic training mode (Mapper(deterministic=True)).

Float atomics make the feature-gradient scatter and the certainty side effect of the reference's
scatter_add_ / index backward (model/neural_points.py:634-652, utils/mapper.py:571-573) depend on
the order the atomics arrive in, so two runs of the same mapping() call differ in the last bits
and, through Adam's sign-sized first steps, in whole elements.  The deterministic mode sums those
terms as 64-bit fixed-point integers (PinTrainState.grad_fixed / cert_fixed) and tile-sorts the
rows stably (pin_query_sort_stable): a mapping() call is then a function of its inputs and draws.

  * two whole mapping(15) calls of the reference fixtures in the mode are bitwise identical
    (features, certainties, ts, decoder, loss), and still meet the fixtures' tolerances;
  * a tiled training batch (stable sort + the decoder-gradient partials) likewise;
  * pin_fixed_accumulate and pin_query_sort_stable against host restatements (exact).
"""
import ctypes

import numpy as np
import pytest
import torch

import pin_slam_amd as P
from pin_slam_amd import _lib
from tests.test_gpu_mapper import MLP_KEYS, _mapping_call_setup, _norm, _np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


def _state(nm, dec, mapper):
    return ([nm.geo_features.detach().clone(), nm.point_certainties.clone(), nm.point_ts_update.clone()]
            + [p.detach().clone() for p in dec.parameters()] + [mapper.last_loss.clone()])


@pytest.mark.parametrize("case", ["mapping_wf", "mapping_wf_frozen", "mapping_nwf_weighted", "mapping_eik_wf",
                                  "mapping_eik_livox"])
def test_deterministic_mapping_call_bitwise(golden, dev, case):
    """Two whole Mapper.mapping(15) calls of a reference fixture in the deterministic mode, from
    the same map and the same replayed draws: every output bitwise equal.  The mode is the same
    computation (fixed-point sums instead of float atomics), so the fixture's tolerances hold:
    the whole-call test's for the numerical eikonal cases, the analytic-eikonal test's otherwise."""
    z = golden(case)
    runs = []
    for _ in range(2):
        nm, dec, mapper, replay = _mapping_call_setup(z, dev, "grid")
        mapper.deterministic = True
        before = nm.geo_features.detach().cpu().numpy().copy()
        mapper.mapping(int(z["iters"]))
        assert replay.calls == 2 * int(z["iters"])
        runs.append(_state(nm, dec, mapper))
    for k, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), f"output {k} differs between two deterministic calls"
    got, want = _np(runs[0][0]), z["global_features_after"]
    if "eik" in case:
        tol = 1e-3 * _norm(want - before) + 3 * float(z["spread_norm_global_features_after"])
        assert _norm(got - want) <= tol, (_norm(got - want), tol)
        return
    off = np.abs(got - want) > 1e-4
    assert off.mean() <= 5e-3, f"{off.sum()} of {off.size} feature elements off by > 1e-4"
    assert _norm(got - want) <= 3e-3 * _norm(want - before), (_norm(got - want), _norm(want - before))
    np.testing.assert_allclose(_np(runs[0][1]), z["global_cert_after"], rtol=1e-5, atol=1e-4)
    np.testing.assert_array_equal(_np(runs[0][2]), z["global_ts_update_after"])
    if not bool(z["frozen"]):
        for key, p in zip(MLP_KEYS, runs[0][3:7]):
            w = z[f"after_{key}"]
            assert _norm(_np(p) - w) <= 1e-4 * _norm(w), (key, _norm(_np(p) - w), _norm(w))


def test_deterministic_tiled_training_call_bitwise(dev):
    """A batch large enough to be tile-sorted (70K rows + stencil) with the decoder training: the
    stable sort fixes the rows' processing order, hence the per-block decoder-gradient partials
    and the per-wave loss partials -- two calls bitwise equal; the default (float-atomic) mode on
    the same draws stays within float noise of it."""
    from pin_slam_amd.synthetic import surface_map, surface_pool
    outs = []
    for det in (True, True, False):
        nm, dec, pts = surface_map(300, device=dev, buffer_size=1 << 22, query_backend="grid", bs=70000)
        torch.manual_seed(11)
        for p in dec.parameters():
            p.requires_grad_(True)
        coord, label, ts = surface_pool(pts, 200000, seed=5, device=dev)
        ts = torch.randint(0, 4, ts.shape, device=dev)
        mapper = P.Mapper(nm.config, None, nm, dec, deterministic=det)
        mapper.set_pool(coord, label, ts)
        torch.manual_seed(77)
        mapper.mapping(3)
        outs.append(_state(nm, dec, mapper))
    for k, (a, b) in enumerate(zip(outs[0], outs[1])):
        assert torch.equal(a, b), f"output {k} differs between two deterministic calls"
    f0, f2 = outs[0][0], outs[2][0]
    off = ~torch.isclose(f0, f2, rtol=1e-4, atol=1e-5)
    assert float(off.float().mean()) <= 2e-3
    torch.testing.assert_close(outs[0][1], outs[2][1], rtol=1e-5, atol=1e-5)
    assert torch.equal(outs[0][2], outs[2][2])
    for a, b in zip(outs[0][3:7], outs[2][3:7]):
        assert _norm(_np(a) - _np(b)) <= 1e-4 * _norm(_np(b))


def test_deterministic_mode_keeps_tiny_gradients(dev):
    """A query that sits ON a neural point gives that point u = 1 / (0 + 1e-15) and its other
    neighbours IDW weights of ~1e-15, so they train on gradients of ~1e-18 -- and Adam with eps
    1e-15 (utils/tools.py:89-116) turns those into steps of ~1e-3 lr.  The reference's float sums
    keep them (its frame-0 mapping of the configs[0] replay moves such elements by ~1e-5 on the
    first step); the deterministic mode's fixed point must too (its fine part, fixed_add): one
    mapping step from the same state in both modes, every element's step equal to float noise."""
    from pin_slam_amd.synthetic import surface_map, surface_pool
    steps = []
    for det in (False, True):
        nm, dec, pts = surface_map(200, device=dev, buffer_size=1 << 22, query_backend="grid", bs=20000)
        for p in dec.parameters():
            p.requires_grad_(False)
        coord, label, ts = surface_pool(pts, 60000, seed=5, sigma=0.0, device=dev)   # rows ON neural points
        label = torch.randn(label.shape, generator=torch.Generator().manual_seed(3)).to(dev) * 0.1
        mapper = P.Mapper(nm.config, None, nm, dec, deterministic=det)
        mapper.set_pool(coord, label, ts)
        before = nm.geo_features.detach().clone()
        torch.manual_seed(77)
        mapper.mapping(1)
        steps.append((nm.geo_features.detach() - before).double().cpu().numpy())
    lr = float(nm.config.lr)
    f, d = steps
    frac = (np.abs(f) > 0) & (np.abs(f) < 0.5 * lr)   # steps of a gradient within ~eps: the tiny ones
    assert int(frac.sum()) > 100, "the batch should train elements on eps-sized gradients"
    np.testing.assert_allclose(d[frac], f[frac], rtol=1e-4, atol=1e-3 * lr * 1e-3)
    off = np.abs(d - f) > 1e-4 * lr
    assert off.mean() <= 1e-3, f"{off.sum()} of {off.size} steps differ"


def test_fixed_accumulate_exact(dev):
    """pin_fixed_accumulate: out += float32(float64(integer sum of the replicas) * 2^-shift), the
    replicas zeroed -- against numpy on the same integers."""
    g = np.random.default_rng(3)
    n, R, shift = 10007, 3, 50
    acc = g.integers(-(1 << 55), 1 << 55, size=(R, n), dtype=np.int64)
    out = g.standard_normal(n).astype(np.float32)
    a, o = torch.from_numpy(acc.copy()).to(dev), torch.from_numpy(out.copy()).to(dev)
    _lib.call("pin_fixed_accumulate", _lib.ptr(a), R, n, shift, 1, _lib.ptr(o), _lib.stream())
    torch.cuda.synchronize()
    want = out + (acc.sum(0).astype(np.float64) * 2.0 ** -shift).astype(np.float32)
    np.testing.assert_array_equal(_np(o), want)
    assert int(a.abs().max()) == 0
    # two parts (PinTrainState.grad_fixed): coarse at 2^-shift, fine at 2^-(shift + 40)
    acc2 = g.integers(-(1 << 55), 1 << 55, size=(2, R, n), dtype=np.int64)
    a2, o2 = torch.from_numpy(acc2.copy()).to(dev), torch.from_numpy(out.copy()).to(dev)
    _lib.call("pin_fixed_accumulate", _lib.ptr(a2), R, n, shift, 2, _lib.ptr(o2), _lib.stream())
    torch.cuda.synchronize()
    inv = 2.0 ** -shift
    want2 = out + (acc2[0].sum(0).astype(np.float64) * inv + acc2[1].sum(0).astype(np.float64) * (inv / 2.0 ** 40)
                   ).astype(np.float32)
    np.testing.assert_array_equal(_np(o2), want2)
    assert int(a2.abs().max()) == 0


def _host_tiles(gv, q, large):
    """tile_of (pin_query.hip) on the host: the tile map of the grid box, f32 arithmetic."""
    g = gv.struct
    d = g.dims
    maxt = 16384 if large else 4096
    ex, ey, ez = 4 * d.nbx, 4 * d.nby, 4 * d.nbz
    sh = 3
    while True:
        nx, ny, nz = ((e + (1 << sh) - 1) >> sh for e in (ex, ey, ez))
        if nx * ny * nz <= maxt:
            break
        sh += 1
    inv = np.float32(1.0) / np.float32(g.resolution)
    c = [np.floor(q[:, a].astype(np.float32) * inv).astype(np.int64) - o for a, o in enumerate((d.ox, d.oy, d.oz))]
    ax = [np.clip(ci >> sh, 0, nt - 1) for ci, nt in zip(c, (nx, ny, nz))]
    return (ax[2] * ny + ax[1]) * nx + ax[0]


@pytest.mark.parametrize("n", [100_000, 1_200_000])
def test_stable_tile_sort(dev, n):
    """pin_query_sort_stable: the queries by tile (pin_query_sort's tile map), input order kept
    inside a tile -- exactly numpy's stable argsort of the host-computed tiles; the counting sort
    lists the same tiles in the same order (only its order inside a tile differs)."""
    from pin_slam_amd.query import query_sort
    from pin_slam_amd.synthetic import surface_map, surface_queries
    nm, dec, pts = surface_map(400, device=dev, buffer_size=1 << 22, query_backend="grid")
    q = surface_queries(pts, n, device=dev)
    gv = nm.grid_view("local", False)
    s4 = query_sort(gv, q, stable=True)
    f4 = query_sort(gv, q)
    torch.cuda.synchronize()
    tiles = _host_tiles(gv, q.cpu().numpy(), n >= (1 << 20))
    want = np.argsort(tiles, kind="stable")
    got = s4[:, 3].contiguous().view(torch.int32).cpu().numpy()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(s4[:, :3].cpu().numpy(), q.cpu().numpy()[want])
    fast = f4[:, 3].contiguous().view(torch.int32).cpu().numpy()
    np.testing.assert_array_equal(tiles[fast], tiles[want])
