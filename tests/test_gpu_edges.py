"""Edge cases of the HIP path (needs an MI355X): empty and ragged batches, queries with no
neighbours, an empty map, the smallest mapper batch, too few valid points for registration.
Expected values follow the reference's behaviour (file:line in each test)."""
import numpy as np
import pytest
import torch

import pin_slam_amd as P
from oracle import pin_oracle as O
from pin_slam_amd.synthetic import points_map
from tests import helpers as H

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


@pytest.fixture(scope="module")
def small_map(dev):
    return H.surface_map(80, device=dev, buffer_size=1 << 20)


@pytest.mark.parametrize("backend", ["hash", "grid"])
@pytest.mark.parametrize("n", [0, 1, 63, 65, 257])
def test_ragged_batches_match_oracle(small_map, dev, backend, n):
    """Batch sizes that are not multiples of the wave / block (partial last wave)."""
    nm, dec, pts = small_map
    nm.config.query_backend = backend
    q = H.surface_queries(pts, n, seed=n + 1, device=dev)
    sdf, grad, nn, cert, _ = P.query_sdf(nm, dec, q, query_locally=True, want_grad=True)
    assert sdf.shape == (n,) and grad.shape == (n, 3) and nn.shape == (n,)
    if n:
        st, mlp = H.oracle_state(nm), H.oracle_mlp(dec)
        osdf, ograd, _, oq = O.sdf_and_grad(st, mlp, _np(q), 8, O.neighbor_offsets(2, 0.2), nm.max_valid_dist2,
                                            True, True)
        np.testing.assert_array_equal(_np(nn), oq.nn_counts)
        np.testing.assert_allclose(_np(sdf), osdf, atol=1e-5)
    nm.config.query_backend = "auto"


@pytest.mark.parametrize("backend", ["hash", "grid"])
def test_queries_without_neighbours(small_map, dev, backend):
    """Far from the map: nn_count 0, zero weights, sdf = Decoder.sdf(0) (query_feature's zero
    feature, neural_points.py:618-632) or 0 with zero_empty (mesher.py:100-105), zero gradient
    (the weights do not depend on q), certainty 0."""
    nm, dec, pts = small_map
    nm.config.query_backend = backend
    q = torch.tensor([[1e4, 1e4, 1e4], [-5e3, 2e3, 0.0], [0.0, 0.0, 500.0]], device=dev)
    sdf, grad, nn, cert, _ = P.query_sdf(nm, dec, q, query_locally=False, want_grad=True)
    assert int(nn.max()) == 0 and float(cert.abs().max()) == 0.0 and float(grad.abs().max()) == 0.0
    zero = dec.sdf(torch.zeros((1, 11), device=dev)).reshape(-1)[0]
    np.testing.assert_allclose(_np(sdf), float(zero.detach()), atol=1e-7)
    sdf0, _, _, _, _ = P.query_sdf(nm, dec, q, query_locally=False, want_grad=False, zero_empty=True)
    assert float(sdf0.abs().max()) == 0.0
    d2, idx = nm.radius_neighborhood_search(q)
    assert int(idx.max()) == -1
    nm.config.query_backend = "auto"


def test_empty_map(dev):
    """A map with no points (before the first update): every query has no neighbours (the
    reference raises IndexError on this input; the drop-in answers with empty neighbourhoods)."""
    cfg = P.Config(device=dev, buffer_size=1 << 16)
    nm = P.NeuralPoints(cfg)
    dec = P.Decoder(cfg, 64, 1, 1)
    assert nm.is_empty() and nm.backend() == "hash"
    q = torch.randn(100, 3, device=dev)
    sdf, grad, nn, cert, _ = P.query_sdf(nm, dec, q, query_locally=False, want_grad=True)
    assert int(nn.max()) == 0 and float(grad.abs().max()) == 0.0
    feat, _, w, nnc, c = nm.query_feature(q, training_mode=False, query_locally=False)
    assert int(nnc.max()) == 0 and float(w.abs().max()) == 0.0


def test_update_then_query_incremental(dev):
    """Two frames through NeuralPoints.update + reset_local_map (model/neural_points.py:205-313)
    and a query against the oracle restatement of the same map."""
    cfg = P.Config(device=dev, buffer_size=1 << 20, weighted_first=True)
    nm = P.NeuralPoints(cfg)
    nm.travel_dist = torch.arange(10, dtype=torch.float32, device=dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    for frame in range(2):
        xy = torch.rand(20000, 2, generator=g) * 30.0 + frame * 5.0
        z = 0.3 * torch.sin(xy[:, :1] / 3.0)
        pts = torch.cat([xy, z], 1).to(dev)
        nm.update(pts, torch.zeros(3, device=dev), torch.eye(3, device=dev), frame)
        nm.reset_local_map(torch.zeros(3, device=dev), torch.eye(3, device=dev), frame)
    nm.geo_features = torch.randn(nm.geo_features.shape, generator=g).to(dev) * 0.05
    nm.geo_features[-1] = 0
    nm.reset_local_map(torch.zeros(3, device=dev), torch.eye(3, device=dev), 1)
    dec = P.Decoder(cfg, 64, 1, 1)
    q = nm.neural_points[:5000] + 0.1 * torch.randn(5000, 3, generator=g).to(dev)
    sdf, grad, nn, _, _ = P.query_sdf(nm, dec, q, query_locally=True, want_grad=True)
    st, mlp = H.oracle_state(nm), H.oracle_mlp(dec)
    osdf, ograd, _, oq = O.sdf_and_grad(st, mlp, _np(q), cfg.query_nn_k, O.neighbor_offsets(2, 0.2),
                                        nm.max_valid_dist2, True, True)
    np.testing.assert_array_equal(_np(nn), oq.nn_counts)
    np.testing.assert_allclose(_np(sdf), osdf, atol=1e-5)


def test_smallest_mapper_batch(small_map, dev):
    """A batch smaller than gradient_decimation still has one stencil row group
    (coord[::10] of 3 rows = 1 row, mapper.py:482-485)."""
    nm, dec, pts = small_map
    mapper = P.Mapper(nm.config, None, nm, dec)
    q = pts[:3].to(dev) + torch.tensor([0.0, 0.0, 0.05], device=dev)
    fg = torch.zeros_like(nm.local_geo_features.data)
    loss = mapper.train_step(q, torch.full((3,), -0.05, device=dev), torch.zeros(3, dtype=torch.int64, device=dev), fg)
    st = H.oracle_state(nm)
    c = nm.config
    out = O.mapper_forward_backward(st, H.oracle_mlp(dec), _np(q), np.full(3, -0.05, np.float32), np.zeros(3, np.int64),
                                    8, O.neighbor_offsets(2, 0.2), nm.max_valid_dist2, True,
                                    float(np.float32(mapper.sdf_scale)), c.weight_e, 10,
                                    c.voxel_size_m * c.num_grad_step_ratio)
    assert float(loss) == pytest.approx(out["loss"], rel=1e-5)


def test_registration_with_too_few_points(small_map, dev):
    """Fewer than 10 valid points: identity increment (utils/tracker.py:382-386 early exit)."""
    nm, dec, pts = small_map
    tr = P.Tracker(nm.config, nm, dec)
    src = torch.tensor([[1e4, 1e4, 1e4]] * 5, device=dev)
    T, cov, eig, _, valid, resid, _ = tr.registration_step(src, None, torch.zeros(5, device=dev), None, 0, 0.5, 2.0,
                                                           0.5, 0.2, 1e-4)
    assert torch.equal(T, torch.eye(4, dtype=torch.float64, device=dev)) and valid.shape[0] == 0


def _lattice_map(dev, nn_k, seed):
    """One point per cell centre of a 24 x 24 lattice, 2 layers deep at x < 12 cells and 6 layers
    deep beyond; half of the points moved by up to 2e-6 m per axis (a few f32 ulps), so that the
    queries below see exactly equal and nearly equal candidate distances."""
    res = 0.3
    rng = np.random.default_rng(seed)
    i, j, k = np.meshgrid(np.arange(24), np.arange(24), np.arange(6), indexing="ij")
    keep = (k < 2) | (i >= 12)
    pts = (np.stack([i[keep], j[keep], k[keep]], 1) + 0.5) * res
    moved = rng.random(pts.shape[0]) < 0.5
    pts[moved] += rng.uniform(-2e-6, 2e-6, (int(moved.sum()), 3))
    nm, dec, _ = points_map(pts.astype(np.float32), res=res, seed=seed, device=dev,
                                        buffer_size=1 << 22, nn_k=nn_k)
    return nm, dec, res


@pytest.mark.parametrize("nn_k", [8, 6])
def test_equal_and_near_equal_distances_match_oracle(dev, nn_k):
    """Candidates at exactly equal distances (a query on a lattice node is equidistant from 8
    cell centres) and at distances a few ulps apart.  The reference keeps the k nearest after
    torch's unstable sort (model/neural_points.py:561-565; ties in the order std::sort leaves them,
    restated by the oracle and by the kernels' resolve_ties); the grid kernel's packed-key
    selection truncates d2 to 18 mantissa bits and must fall back to the exact order where that
    matters.  Two layers (<= 32 occupied cells per query: packed keys) and six (33 > 32:
    the segmented scan).  A different neighbour set would move the SDF by ~1e-2."""
    nm, dec, res = _lattice_map(dev, nn_k, 3 + nn_k)
    assert nm.backend() == "grid"
    rng = np.random.default_rng(11)
    a, b = np.meshgrid(np.arange(2, 23), np.arange(2, 23), indexing="ij")
    nodes = np.stack([a.ravel(), b.ravel()], 1).astype(np.float64)
    qs = []
    for z in (1.0, 0.5, 3.0):                     # lattice nodes, cell centres in z, deep layers
        qs.append(np.concatenate([nodes, np.full((nodes.shape[0], 1), z)], 1) * res)
        qs.append(np.concatenate([nodes + [0.5, 0.0], np.full((nodes.shape[0], 1), z)], 1) * res)
    q = np.concatenate(qs, 0)
    q = np.concatenate([q, q + rng.uniform(-3e-7, 3e-7, q.shape)], 0).astype(np.float32)
    qt = torch.from_numpy(q).to(dev)
    sdf, grad, nn, _, _ = P.query_sdf(nm, dec, qt, query_locally=False, want_grad=True)
    st, mlp = H.oracle_state(nm), H.oracle_mlp(dec)
    osdf, ograd, _, oq = O.sdf_and_grad(st, mlp, q, nn_k, O.neighbor_offsets(2, 0.2), nm.max_valid_dist2,
                                        True, False)
    np.testing.assert_array_equal(_np(nn), oq.nn_counts)
    assert int(oq.nn_counts.max()) > 32 and float((oq.nn_counts > nn_k).mean()) > 0.5
    np.testing.assert_allclose(_np(sdf), osdf, atol=1e-5)
    gerr = np.abs(_np(grad) - ograd).max(-1) / np.maximum(np.abs(ograd).max(-1), 1e-3)
    assert float(gerr.max()) < 1e-3


def test_dynamic_filter_both_strategies_match_oracle(dev):
    """Mapper.dynamic_filter (utils/mapper.py:79-108): strategy 1 (certain free space: certainty
    and SDF thresholds) and strategy 2 (type_2_on: also a flat analytic gradient at a certain
    point, |grad| <= 0.3 and certainty >= 0.5) against the oracle's SDF, gradient and queried
    certainty.  The thresholds are set (config) or scaled into (decoder output weights, which the
    gradient is linear in) the middle of this map's values so both outcomes occur; decisions
    within the parity tolerance of a threshold are not compared."""
    nm, dec, pts = H.surface_map(80, device=dev, buffer_size=1 << 20)
    q = H.surface_queries(pts, 4096, seed=5, device=dev)
    qn = _np(q)
    off = O.neighbor_offsets(2, 0.2)

    def oracle():
        return O.sdf_and_grad(H.oracle_state(nm), H.oracle_mlp(dec), qn, 8, off, nm.max_valid_dist2, True, True)
    _, ograd, _, _ = oracle()
    with torch.no_grad():   # median gradient norm -> 0.3
        dec.lout.weight.mul_(0.3 / float(np.median(np.linalg.norm(ograd, axis=-1))))
    osdf, ograd, _, oq = oracle()
    c = nm.config
    c.dynamic_certainty_thre = float(np.median(oq.certainty))
    c.dynamic_sdf_ratio_thre = float(np.median(osdf)) / c.voxel_size_m
    thr_s = np.float32(c.dynamic_sdf_ratio_thre * c.voxel_size_m)
    cert, gn = oq.certainty, np.linalg.norm(ograd.astype(np.float64), axis=-1)
    s1 = (cert < c.dynamic_certainty_thre) | (osdf < thr_s)
    s2 = s1 & ((gn > 0.3) | (cert < 0.5))
    near = ((np.abs(osdf - thr_s) <= 1e-5) | (np.abs(gn - 0.3) <= 1e-4) |
            (np.abs(cert - c.dynamic_certainty_thre) <= 1e-5) | (np.abs(cert - 0.5) <= 1e-5))
    assert near.mean() < 0.01
    mapper = P.Mapper(c, None, nm, dec)
    for type_2, ref in ((False, s1), (True, s2)):
        got = _np(mapper.dynamic_filter(q, type_2))
        assert got.dtype == np.bool_ and got.shape == (qn.shape[0],)
        np.testing.assert_array_equal(got[~near], ref[~near])
        assert 0.05 < float(ref.mean()) < 0.95


@pytest.mark.parametrize("n", [2, 16, 17, 33, 57, 81, 93, 125, 128])
def test_wave_ref_sort_is_torch_cpu_sort(dev, n):
    """The kernels' tie order (resolve_ties: the row held by the wave, std::sort restated with
    parallel partitions, the heap-sort fallback entry by entry, a stable final rank) through its
    test hook pin_ref_sort_rows: the whole permutation equals torch's CPU sort(stable=False) --
    the sort the reference's k-NN calls -- on tie-heavy rows, sorted / reversed rows, and
    adversarial rows (McIlroy) that drive the introsort into its heap sort, with and without ties."""
    from pin_slam_amd import _lib
    from tests.test_oracle_golden import ref_sort_test_rows
    rows = np.stack(ref_sort_test_rows(n, np.random.default_rng(100 + n)))
    keys = torch.from_numpy(rows).to(dev)
    order = torch.full(rows.shape, -1, dtype=torch.int32, device=dev)
    _lib.call("pin_ref_sort_rows", _lib.ptr(keys), n, rows.shape[0], _lib.ptr(order), _lib.stream())
    torch.cuda.synchronize()
    _, want = torch.sort(torch.from_numpy(rows), dim=1)
    np.testing.assert_array_equal(_np(order).astype(np.int64), want.numpy())
