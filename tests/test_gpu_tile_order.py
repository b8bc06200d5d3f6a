"""Tile-order outputs (PIN_QUERY_OUT_TILE): the fused SDF query may leave its outputs in the order
the tile sort processed the queries, with the sorted rows q4 {x, y, z, bits(index)} saying which
query each output row belongs to, and the tracker's normal equations consume them in that order
(PinRegParams.q4_points).  Same kernel, same per-query arithmetic: the outputs must be the
input-order outputs permuted, bit for bit; the registration step must agree with the input-order
step to the f64 summation order (its sums run over the points in another order)."""
import numpy as np
import pytest
import torch

import pin_slam_amd as P
from pin_slam_amd import query as Q
from tests import helpers as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


@pytest.mark.parametrize("wf", [True, False])
def test_tile_order_outputs_are_the_input_order_outputs_permuted(dev, wf):
    from pin_slam_amd.synthetic import surface_map, surface_queries
    nm, dec, pts = surface_map(300, device=dev, buffer_size=1 << 22, weighted_first=wf)
    assert nm.backend() == "grid"
    q = surface_queries(pts, 100_000, device=dev)
    assert q.shape[0] >= Q._TILE_MIN
    kw = dict(query_locally=False, want_grad=True, want_certainty=True, want_std=not wf)
    ref = P.query_sdf(nm, dec, q, **kw)
    out = P.query_sdf(nm, dec, q, out_order="tile", **kw)
    q4 = out[5]
    assert q4 is not None
    idx = q4[:, 3].contiguous().view(torch.int32).long()
    assert torch.equal(torch.sort(idx).values, torch.arange(q.shape[0], device=dev))   # a permutation
    assert torch.equal(q4[:, :3], q[idx])
    for k, name in enumerate(("sdf", "grad", "nn_count", "certainty", "sdf_std")):
        if ref[k] is None:
            assert out[k] is None
            continue
        assert torch.equal(out[k], ref[k][idx]), name
    # below the tiling threshold the outputs stay in input order and no q4 is returned
    small = P.query_sdf(nm, dec, q[:1000], out_order="tile", **kw)
    assert small[5] is None and torch.equal(small[0], ref[0][:1000])


@pytest.mark.parametrize("case", ["tracker_wf", "tracker_nwf"])
def test_registration_on_tile_order_outputs(golden, dev, case, monkeypatch):
    """registration_step with the query tiled (threshold lowered to the fixture's size) and its
    outputs consumed in tile order == the input-order step: the same valid points (in source
    order), residual and increment to the f64 summation order."""
    from pin_slam_amd.tracker import Tracker
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev, backend="grid")
    nm.local_geo_features = torch.nn.Parameter(torch.as_tensor(z["local_features"], device=dev))
    dec = H.decoder_from_fixture(z, nm.config)
    cfg = nm.config
    cfg.surface_sample_range_m = float(z["surface_sample_range_m"])
    cfg.max_sdf_std_ratio = float(z["max_sdf_std_ratio"])
    tr = Tracker(cfg, nm, dec)
    src = torch.as_tensor(z["source"], device=dev)
    labels = torch.linspace(-0.01, 0.01, src.shape[0], device=dev)   # labels are read by source index

    def step():
        return tr.registration_step(src, None, labels, None, 9, float(z["reg_min_grad_norm"]),
                                    float(z["reg_max_grad_norm"]), float(z["reg_GM_dist_m"]), float(z["reg_GM_grad"]),
                                    float(z["reg_lm_lambda"]))
    monkeypatch.setattr(Q, "_TILE_QUERIES", False)
    T0, _, _, _, v0, r0, _ = step()
    monkeypatch.setattr(Q, "_TILE_QUERIES", True)
    monkeypatch.setattr(Q, "_TILE_MIN", 1)
    T1, _, _, _, v1, r1, _ = step()
    assert torch.equal(v0, v1)
    assert r1 == pytest.approx(r0, rel=1e-9)
    np.testing.assert_allclose(T1.cpu().numpy(), T0.cpu().numpy(), rtol=0, atol=1e-9)


def _tiles_of(nm, pts):
    """Host restatement of the sort's tile key (pin_query.hip tile_map / tile_of) for a check that
    the lean sort's output is grouped by tile in ascending tile order."""
    occ = nm.occupancy()
    dims = occ[1]
    res = np.float32(nm.resolution)
    ex, ey, ez = 4 * dims.nbx, 4 * dims.nby, 4 * dims.nbz
    sh = 3
    while True:
        nt = [(e + (1 << sh) - 1) >> sh for e in (ex, ey, ez)]
        if nt[0] * nt[1] * nt[2] <= 4096:
            break
        sh += 1
    inv = np.float32(1.0) / res
    p = pts.cpu().numpy()
    ax = []
    for a, o in enumerate((dims.ox, dims.oy, dims.oz)):
        c = (np.floor(p[:, a] * inv).astype(np.int64) - o) >> sh
        ax.append(np.clip(c, 0, nt[a] - 1))
    return (ax[2] * nt[1] + ax[1]) * nt[0] + ax[0]


def test_lean_sort_groups_by_tile(dev):
    """pin_query_sort_ex(PIN_SORT_LEAN): a permutation of the batch with the coordinates carried,
    grouped by tile in ascending tile order (the standard sort's contract; order inside a tile is
    arbitrary); the workspace state is left zero (a second call on it sorts again)."""
    from pin_slam_amd import _lib
    from pin_slam_amd.synthetic import surface_map, surface_queries
    nm, dec, pts = surface_map(300, device=dev, buffer_size=1 << 22)
    q = surface_queries(pts, 100_003, device=dev)
    gv = nm.grid_view("global", True)
    ws = Q.order_workspace(q.shape[0], q.device)
    for _ in range(2):
        q4 = torch.empty((q.shape[0], 4), device=dev)
        order = torch.empty(q.shape[0], dtype=torch.int32, device=dev)
        _lib.call("pin_query_sort_ex", gv.ref(), _lib.ptr(q), q.shape[0], _lib.ptr(q4), _lib.ptr(order), _lib.ptr(ws),
                  Q.SORT_LEAN, _lib.stream())
        idx = q4[:, 3].contiguous().view(torch.int32).long()
        assert torch.equal(torch.sort(idx).values, torch.arange(q.shape[0], device=dev))
        assert torch.equal(order.long(), idx)
        assert torch.equal(q4[:, :3], q[idx])
        tiles = _tiles_of(nm, q[idx])
        assert np.all(np.diff(tiles) >= 0)
    assert int(ws[:Q.ORDER_STATE_BYTES].view(torch.int32)[:4096].abs().sum()) == 0


def test_query_pipeline_matches_query_sdf(dev):
    """QueryPipeline (lean sort of batch k+1 on a second stream beside the query of batch k): for
    four different batches, every output row equals query_sdf's output of the query it names."""
    from pin_slam_amd.synthetic import surface_map, surface_queries
    nm, dec, pts = surface_map(300, device=dev, buffer_size=1 << 22)
    n = 80_000
    batches = [surface_queries(pts, n, seed=11 + k, device=dev) for k in range(4)]
    pipe = P.QueryPipeline(nm, dec, n)
    pipe.sort(batches[0])
    got = []
    for k in range(4):
        if k + 1 < 4:
            pipe.sort(batches[k + 1])
        sdf, grad, nn, q4 = pipe.query()
        got.append((sdf.clone(), grad.clone(), nn.clone(), q4.clone()))
    for k, (sdf, grad, nn, q4) in enumerate(got):
        ref = P.query_sdf(nm, dec, batches[k], query_locally=False, want_grad=True, want_certainty=False)
        idx = q4[:, 3].contiguous().view(torch.int32).long()
        assert torch.equal(torch.sort(idx).values, torch.arange(n, device=dev))
        assert torch.equal(sdf, ref[0][idx]) and torch.equal(grad, ref[1][idx]) and torch.equal(nn, ref[2][idx])
    with pytest.raises(RuntimeError):
        pipe.query()
