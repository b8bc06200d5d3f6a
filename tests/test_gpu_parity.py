"""HIP path vs the reference's golden vectors and vs the oracle (needs an MI355X).

Tolerances (fp32): SDF abs <= 1e-5 (north-star bar; observed ~1e-7), neighbour sets and
nn_counts bit-exact, IDW weights rel 2e-6, gradients rel 1e-4 / abs 2e-5 with at most a
handful of rows allowed off where an MLP pre-activation sits within rounding of the ReLU
kink (counted, never more than 0.1% of rows).
"""
import numpy as np
import pytest
import torch

from oracle import pin_oracle as O
from tests import helpers as H

pytestmark = pytest.mark.gpu

QUERY_CASES = ["query_wf", "query_nwf", "query_kitti", "query_ties"]
BACKENDS = ["hash", "grid"]
SDF_ATOL = 1e-5


def _np(t):
    return t.detach().cpu().numpy()


def assert_grad_close(got, want, rtol=1e-4, atol=2e-5, max_bad_frac=1e-3):
    bad = ~np.isclose(got, want, rtol=rtol, atol=atol).all(-1)
    assert bad.mean() <= max_bad_frac, f"{bad.sum()} / {bad.shape[0]} gradient rows off; worst " \
        f"{np.abs(got - want).max(-1)[bad][:5]}"


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


@pytest.mark.parametrize("case", QUERY_CASES)
@pytest.mark.parametrize("tf", [0, 1])
def test_radius_search_exact(golden, dev, case, tf):
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev)
    d2, idx = nm.radius_neighborhood_search(torch.as_tensor(z["queries"], device=dev), time_filtering=bool(tf))
    np.testing.assert_array_equal(_np(idx), z[f"rns{tf}_idx"])
    np.testing.assert_array_equal(_np(d2), z[f"rns{tf}_dist2"])


@pytest.mark.parametrize("case", QUERY_CASES)
@pytest.mark.parametrize("ql", [0, 1])
@pytest.mark.parametrize("backend", BACKENDS)
def test_query_feature_dropin(golden, dev, backend, case, ql):
    """NeuralPoints.query_feature + Decoder.sdf + autograd (the reference's own call
    sequence, utils/tracker.py:230-252) through the HIP forward/backward kernels."""
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev, backend=backend)
    dec = H.decoder_from_fixture(z, nm.config)
    q = torch.as_tensor(z["queries"], device=dev).requires_grad_(True)
    feat, _, w, nn_counts, cert = nm.query_feature(q, training_mode=False, query_locally=bool(ql))
    p = f"q{ql}_"
    np.testing.assert_array_equal(_np(nn_counts), z[p + "nn_counts"])
    np.testing.assert_allclose(_np(w)[..., 0], z[p + "weights"], rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(_np(feat), z[p + "feat"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(_np(cert), z[p + "certainty"], rtol=1e-5, atol=1e-5)
    sdf = dec.sdf(feat)
    if not nm.config.weighted_first:
        sdf = torch.sum(sdf * w, dim=1).squeeze(1)
    g = torch.autograd.grad(sdf, q, torch.ones_like(sdf), create_graph=True)[0]
    np.testing.assert_allclose(_np(sdf), z[p + "sdf"], rtol=0, atol=SDF_ATOL)
    assert_grad_close(_np(g), z[p + "grad"])


@pytest.mark.parametrize("case", QUERY_CASES)
@pytest.mark.parametrize("ql", [0, 1])
@pytest.mark.parametrize("backend", BACKENDS)
def test_query_sdf_fused(golden, dev, backend, case, ql):
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev, backend=backend)
    dec = H.decoder_from_fixture(z, nm.config)
    import pin_slam_amd as P
    sdf, grad, nn, cert, std = P.query_sdf(nm, dec, torch.as_tensor(z["queries"], device=dev),
                                           query_locally=bool(ql), want_grad=True, want_std=True)
    p = f"q{ql}_"
    np.testing.assert_array_equal(_np(nn), z[p + "nn_counts"])
    np.testing.assert_allclose(_np(sdf), z[p + "sdf"], rtol=0, atol=SDF_ATOL)
    np.testing.assert_allclose(_np(cert), z[p + "certainty"], rtol=1e-5, atol=1e-5)
    assert_grad_close(_np(grad), z[p + "grad"])
    if not nm.config.weighted_first:
        np.testing.assert_allclose(_np(std), z[p + "sdf_std"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("case", QUERY_CASES)
@pytest.mark.parametrize("backend", BACKENDS)
def test_after_pgo(golden, dev, backend, case):
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev, orientations=z["pgo_point_orientations"], after_pgo=True,
                                      backend=backend)
    dec = H.decoder_from_fixture(z, nm.config)
    import pin_slam_amd as P
    sdf, grad, nn, cert, std = P.query_sdf(nm, dec, torch.as_tensor(z["queries"], device=dev),
                                           query_locally=True, want_grad=True, want_std=True)
    np.testing.assert_allclose(_np(sdf), z["qpgo_sdf"], rtol=0, atol=SDF_ATOL)
    assert_grad_close(_np(grad), z["qpgo_grad"])
    q = torch.as_tensor(z["queries"], device=dev).requires_grad_(True)
    feat, _, w, _, _ = nm.query_feature(q, training_mode=False, query_locally=True)
    np.testing.assert_allclose(_np(feat), z["qpgo_feat"], rtol=1e-5, atol=5e-6)
    s = dec.sdf(feat)
    if not nm.config.weighted_first:
        s = torch.sum(s * w, dim=1).squeeze(1)
    g = torch.autograd.grad(s, q, torch.ones_like(s))[0]
    assert_grad_close(_np(g), z["qpgo_grad"])


@pytest.mark.parametrize("case", QUERY_CASES)
@pytest.mark.parametrize("backend", BACKENDS)
def test_training_side_effects(golden, dev, backend, case):
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev, backend=backend)
    np.testing.assert_array_equal(_np(nm.local_point_certainties), z["train_cert_before"])
    q = torch.as_tensor(z["queries"], device=dev)
    ts = torch.as_tensor(z["train_query_ts"], device=dev)
    nm.query_feature(q, ts, training_mode=True, query_locally=True)
    np.testing.assert_allclose(_np(nm.local_point_certainties), z["train_cert_after"], rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(_np(nm.local_point_ts_update), z["train_ts_after"])


@pytest.mark.parametrize("case", QUERY_CASES)
def test_query_certainty(golden, dev, case):
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev)
    nm.set_search_neighborhood(num_nei_cells=1, search_alpha=0.0)
    c = nm.query_certainty(torch.as_tensor(z["queries"], device=dev))
    np.testing.assert_array_equal(_np(c), z["qc_certainty"])


@pytest.mark.parametrize("backend", BACKENDS)
def test_mesher_fixture(golden, dev, backend):
    z = golden("mesher_wf")
    nm = H.neural_points_from_fixture(z, dev, backend=backend)
    dec = H.decoder_from_fixture(z, nm.config)
    import pin_slam_amd as P
    sdf, _, nn, _, _ = P.query_sdf(nm, dec, torch.as_tensor(z["coord"], device=dev), query_locally=False,
                                   want_grad=False, zero_empty=True)
    np.testing.assert_array_equal(_np(nn) >= int(z["mesh_min_nn"]), z["mc_mask"])
    np.testing.assert_allclose(_np(sdf), z["sdf"], rtol=0, atol=SDF_ATOL)


@pytest.mark.parametrize("host", [True, False])
@pytest.mark.parametrize("out_torch", [False, True])
def test_mesher_query_points_dropin(golden, dev, host, out_torch):
    """Mesher.query_points (utils/mesher.py:41-136): batched, host or device coordinates,
    reference output types (float64 numpy / CPU float32 tensors, mask as 0/1)."""
    z = golden("mesher_wf")
    nm = H.neural_points_from_fixture(z, dev)
    dec = H.decoder_from_fixture(z, nm.config)
    import pin_slam_amd as P
    mesher = P.Mesher(nm.config, nm, dec)
    coord = torch.as_tensor(z["coord"])
    if not host:
        coord = coord.to(dev)
    sdf, sem, color, mask = mesher.query_points(coord, 7777, True, False, False, True, query_locally=False,
                                                mask_min_nn_count=int(z["mesh_min_nn"]), out_torch=out_torch)
    assert sem is None and color is None
    if out_torch:
        assert sdf.dtype == torch.float32 and mask.dtype == torch.float32 and not sdf.is_cuda
        sdf, mask = sdf.numpy(), mask.numpy()
    else:
        assert sdf.dtype == np.float64 and mask.dtype == np.float64
    np.testing.assert_array_equal(mask, z["mc_mask"].astype(np.float64))
    np.testing.assert_allclose(sdf, z["sdf"], rtol=0, atol=SDF_ATOL)


@pytest.mark.parametrize("case", ["tracker_wf", "tracker_nwf"])
@pytest.mark.parametrize("backend", BACKENDS)
def test_tracker_fixture_queries(golden, dev, backend, case):
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev, backend=backend)
    nm.local_geo_features = torch.nn.Parameter(torch.as_tensor(z["local_features"], device=dev))
    dec = H.decoder_from_fixture(z, nm.config)
    import pin_slam_amd as P
    sdf, grad, nn, cert, std = P.query_sdf(nm, dec, torch.as_tensor(z["source"], device=dev), query_locally=True,
                                           want_grad=True, want_std=True)
    np.testing.assert_allclose(_np(sdf), z["sdf"], rtol=0, atol=SDF_ATOL)
    assert_grad_close(_np(grad), z["grad"])
    np.testing.assert_array_equal(_np(nn) >= int(z["nn_k"]), z["mask"])
    np.testing.assert_allclose(_np(cert), z["certainty"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(_np(std), z["sdf_std"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("case", ["mapper_wf", "mapper_nwf"])
@pytest.mark.parametrize("backend", BACKENDS)
def test_mapper_dropin_backward(golden, dev, backend, case):
    """One reference mapping iteration through the drop-in classes (query_feature in
    training mode, numerical gradient, BCE + eikonal, backward): feature and MLP grads."""
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev, backend=backend)
    dec = H.decoder_from_fixture(z, nm.config)
    cfg = nm.config
    coord = torch.as_tensor(z["it0_coord"], device=dev)
    label = torch.as_tensor(z["it0_label"], device=dev)
    ts = torch.as_tensor(z["it0_ts"], device=dev)

    def sdf_of(x, ts_=None):
        f, _, w, _, _ = nm.query_feature(x, ts_)
        s = dec.sdf(f)
        if not cfg.weighted_first:
            s = torch.sum(s * w, dim=1).squeeze(1)
        return s

    sdf = sdf_of(coord, ts)
    xd = coord[::10]
    eps = float(z["num_grad_eps"])
    stencil = torch.cat([xd + torch.tensor(e, device=dev) for e in
                         ([eps, 0, 0], [-eps, 0, 0], [0, eps, 0], [0, -eps, 0], [0, 0, eps], [0, 0, -eps])])
    s = sdf_of(stencil).view(6, -1)
    g = torch.stack([(s[0] - s[1]), (s[2] - s[3]), (s[4] - s[5])], 1) / (2 * eps)
    sigma = float(z["sigma"])
    loss = torch.nn.functional.binary_cross_entropy_with_logits(sdf / sigma, torch.sigmoid(label / sigma)) + \
        float(z["weight_e"]) * ((g.norm(2, dim=-1) - 1.0) ** 2).mean()
    loss.backward()
    assert float(loss.detach()) == pytest.approx(float(z["it0_loss"]), rel=1e-5)
    np.testing.assert_allclose(_np(sdf), z["it0_sdf"], atol=SDF_ATOL)
    np.testing.assert_allclose(_np(nm.local_geo_features.grad), z["it0_feat_grad"], rtol=1e-4, atol=1e-8)
    for key, prm in zip(["W1", "b1", "W2", "b2"], dec.parameters()):
        np.testing.assert_allclose(_np(prm.grad), z[f"it0_grad_{key}"], rtol=1e-3, atol=1e-7)
    np.testing.assert_allclose(_np(nm.local_point_certainties), z["it0_cert_after"], rtol=1e-5, atol=1e-4)
    np.testing.assert_array_equal(_np(nm.local_point_ts_update), z["it0_ts_after"])


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("wf", [True, False])
def test_random_map_vs_oracle(dev, wf, backend):
    """Larger seeded map (250K points, 20K queries) against the oracle: exact neighbour
    counts and k-NN ids, SDF within 1e-5, gradients within tolerance."""
    nm, dec, pts = H.surface_map(500, device=dev, weighted_first=wf, buffer_size=1 << 22, query_backend=backend)
    assert nm.backend() == backend
    q = H.surface_queries(pts, 20000, device=dev)
    import pin_slam_amd as P
    sdf, grad, nn, cert, std = P.query_sdf(nm, dec, q, query_locally=True, want_grad=True, want_std=True)
    st = H.oracle_state(nm)
    mlp = H.oracle_mlp(dec)
    dx = O.neighbor_offsets(2, 0.2)
    osdf, ograd, ostd, oq = O.sdf_and_grad(st, mlp, _np(q), 8, dx, nm.max_valid_dist2, wf, True)
    np.testing.assert_array_equal(_np(nn), oq.nn_counts)
    np.testing.assert_allclose(_np(sdf), osdf, rtol=0, atol=SDF_ATOL)
    assert_grad_close(_np(grad), ograd)
    feat, _, w, nnc, _ = nm.query_feature(q, training_mode=False)
    np.testing.assert_allclose(_np(w)[..., 0], oq.weights, rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("wf", [True, False])
@pytest.mark.parametrize("feature_std,wscale", [(1e-4, 1.0), (0.05, 1.0), (20.0, 1.0), (0.05, 30.0)])
def test_matrix_core_decoder_matches_f32(dev, wf, feature_std, wscale):
    """The f16-split MFMA decoder (pin_mlp_pack) against the f32 VALU decoder on the same
    queries, across input and weight magnitudes (the per-row / per-query power-of-two scaling
    keeps both f16 terms in range): SDF within 2e-6 relative to the SDF scale of the batch,
    gradients within the parity tolerance."""
    from pin_slam_amd import _lib
    from pin_slam_amd.query import mlp_view
    nm, dec, pts = H.surface_map(200, device=dev, weighted_first=wf, buffer_size=1 << 22, query_backend="grid",
                                 feature_std=feature_std)
    with torch.no_grad():
        dec.layers[0].weight.mul_(wscale)
    q = H.surface_queries(pts, 30001, device=dev)
    gv = nm.grid_view("global", True)
    _, pv = nm._views("global", False)
    n = q.shape[0]
    res = []
    for packed in (False, True):
        mv = mlp_view(dec, packed=packed)
        assert bool(mv.struct.packed) == packed
        sdf = torch.empty(n, device=dev)
        grad = torch.empty((n, 3), device=dev)
        nn = torch.empty(n, dtype=torch.int32, device=dev)
        std = torch.empty(n, device=dev)
        _lib.call("pin_query_sdf_grid", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q), n, 8, int(wf), 0, _lib.ptr(sdf),
                  _lib.ptr(grad), _lib.ptr(nn), None, _lib.ptr(std), None, _lib.stream())
        res.append((_np(sdf), _np(grad), _np(nn), _np(std)))
    (s0, g0, n0, d0), (s1, g1, n1, d1) = res
    np.testing.assert_array_equal(n1, n0)
    scale = max(1.0, float(np.abs(s0).max()))
    np.testing.assert_allclose(s1, s0, rtol=0, atol=2e-6 * scale)
    assert_grad_close(g1, g0, atol=2e-5 * max(1.0, float(np.abs(g0).max())))
    if not wf:
        np.testing.assert_allclose(d1, d0, rtol=0, atol=2e-6 * scale)


@pytest.mark.parametrize("wf", [True, False])
def test_query_order_is_a_permutation_and_invisible(dev, wf):
    """pin_query_order / pin_query_sort group a random batch by spatial tile (a counting sort whose
    workspace state is left zero by every call, so repeated calls stay valid); the SDF kernel's
    outputs are bitwise identical in input order, in `order` and over the sorted float4 rows
    (the order only changes which lane runs a query)."""
    from pin_slam_amd import _lib
    from pin_slam_amd.query import mlp_view, query_order, query_sort
    nm, dec, pts = H.surface_map(300, device=dev, weighted_first=wf, buffer_size=1 << 22, query_backend="grid")
    q = H.surface_queries(pts, 70001, device=dev)
    gv = nm.grid_view("global", True)
    for _ in range(3):
        order = query_order(gv, q)
        assert torch.equal(torch.sort(order.long())[0], torch.arange(q.shape[0], device=dev))
    q4 = query_sort(gv, q)
    idx = q4[:, 3].contiguous().view(torch.int32).long()
    assert torch.equal(torch.sort(idx)[0], torch.arange(q.shape[0], device=dev))
    assert torch.equal(q4[:, :3], q[idx])
    # tile grouping: the tile id along the sorted rows never returns to an earlier tile
    d = gv.struct.dims
    inv = 1.0 / torch.tensor(np.float32(nm.resolution), dtype=torch.float32, device=dev)   # the kernel's rule
    cell = torch.floor(q4[:, :3] * inv).long() - torch.tensor([d.ox, d.oy, d.oz], device=dev)
    ext = torch.tensor([4 * d.nbx, 4 * d.nby, 4 * d.nbz], device=dev)
    sh = 3
    while int(torch.prod((ext + (1 << sh) - 1) >> sh)) > 4096:
        sh += 1
    nt = (ext + (1 << sh) - 1) >> sh
    tc = torch.minimum(torch.clamp(cell >> sh, min=0), nt - 1)
    tile = (tc[:, 2] * nt[1] + tc[:, 1]) * nt[0] + tc[:, 0]
    starts = torch.nonzero(tile[1:] != tile[:-1]).numel() + 1
    assert starts == torch.unique(tile).numel()
    hv, pv = nm._views("global", False)
    for packed in (False, True):   # f32 VALU decoder and f16 matrix-core decoder
        _check_order_invisible(gv, pv, mlp_view(dec, packed=packed), q, q4, order, wf)


def _check_order_invisible(gv, pv, mv, q, q4, order, wf):
    from pin_slam_amd import _lib
    dev = q.device
    outs = []
    for o in (None, order, "sorted"):
        sdf = torch.empty(q.shape[0], device=dev)
        grad = torch.empty((q.shape[0], 3), device=dev)
        nn = torch.empty(q.shape[0], dtype=torch.int32, device=dev)
        std = torch.empty(q.shape[0], device=dev)
        if isinstance(o, str):
            _lib.call("pin_query_sdf_grid_sorted", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q4), q.shape[0], 8, int(wf),
                      0, _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn), None, _lib.ptr(std), _lib.stream())
        else:
            _lib.call("pin_query_sdf_grid", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q), q.shape[0], 8, int(wf), 0,
                      _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn), None, _lib.ptr(std), _lib.ptr(o), _lib.stream())
        outs.append((sdf, grad, nn, std))
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


def test_backend_selection(golden, dev):
    """The grid is used only when it is exact: after adjust_map (points moved, table not
    rebuilt) the table holds entries off their own voxel and the hash path must be taken."""
    z = golden("query_wf")
    nm = H.neural_points_from_fixture(z, dev)
    assert nm.backend() == "grid"
    with torch.no_grad():
        nm.neural_points += 0.37
    assert nm.backend() == "hash"


@pytest.mark.parametrize("case", ["tracker_wf", "tracker_nwf"])
@pytest.mark.parametrize("backend", BACKENDS)
def test_registration_step_fixture(golden, dev, backend, case):
    """Tracker.registration_step (utils/tracker.py:277-452) vs the reference's own step."""
    from pin_slam_amd.tracker import Tracker
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev, backend=backend)
    nm.local_geo_features = torch.nn.Parameter(torch.as_tensor(z["local_features"], device=dev))
    dec = H.decoder_from_fixture(z, nm.config)
    cfg = nm.config
    cfg.surface_sample_range_m = float(z["surface_sample_range_m"])
    cfg.max_sdf_std_ratio = float(z["max_sdf_std_ratio"])
    tr = Tracker(cfg, nm, dec)
    src = torch.as_tensor(z["source"], device=dev)
    T, cov, eig, _, valid_points, resid_cm, _ = tr.registration_step(
        src, None, torch.zeros(src.shape[0], device=dev), None, 9, float(z["reg_min_grad_norm"]),
        float(z["reg_max_grad_norm"]), float(z["reg_GM_dist_m"]), float(z["reg_GM_grad"]), float(z["reg_lm_lambda"]))
    assert abs(valid_points.shape[0] - int(z["valid_count"])) <= 2
    assert resid_cm == pytest.approx(float(z["resid_cm"]), rel=1e-3)
    np.testing.assert_allclose(_np(T), z["delta_T"], atol=5e-6)
    # reg_dist_div_grad_norm (utils/tracker.py:335-336): residual sdf / |g| - label
    cfg.reg_dist_div_grad_norm = True
    T, _, _, _, _, resid_cm, _ = tr.registration_step(
        src, None, torch.zeros(src.shape[0], device=dev), None, 9, float(z["reg_min_grad_norm"]),
        float(z["reg_max_grad_norm"]), float(z["reg_GM_dist_m"]), float(z["reg_GM_grad"]), float(z["reg_lm_lambda"]))
    cfg.reg_dist_div_grad_norm = False
    assert resid_cm == pytest.approx(float(z["divnorm_resid_cm"]), rel=1e-3)
    np.testing.assert_allclose(_np(T), z["divnorm_delta_T"], atol=5e-6)


@pytest.mark.parametrize("case,mode", [("tracker_wf", "loop"), ("tracker_nwf", "loop"), ("tracker_wf", "sorted"),
                                       ("tracker_wf", "stepwise")])
def test_tracking_loop_fixture(golden, dev, case, mode, monkeypatch):
    """The whole Tracker.tracking loop (utils/tracker.py:39-174: iterations, convergence,
    validity checks, fall-back) from the identity guess vs the reference's own run on a
    well-conditioned room scene: same number of iterations, per-iteration increments within
    5e-5 (f32 reductions in a different order feed the next iteration), residuals within
    1e-3 relative, valid-point counts within 3 (points at the gradient-norm thresholds), the
    final pose within 1e-4 and the same validity verdict.  Modes: "loop" = the pipelined
    loop (_RegLoop: one iteration enqueued ahead of the host's read); "sorted" = the same with the
    cloud tile-sorted once and re-posed in tile order on later iterations (forced on for this
    small cloud); "stepwise" = one _register call per iteration (the sharded path's form)."""
    from pin_slam_amd import tracker as trk
    from pin_slam_amd.tracker import Tracker
    if mode == "sorted":
        monkeypatch.setattr(trk, "_LOOP_SORT_MIN", 0)
    if mode == "stepwise":
        monkeypatch.setattr(trk, "_PIPELINE", False)
    z = golden(case)
    nm = H.neural_points_from_fixture(z, dev)
    nm.local_geo_features = torch.nn.Parameter(torch.as_tensor(z["local_features"], device=dev))
    dec = H.decoder_from_fixture(z, nm.config)
    cfg = nm.config
    cfg.surface_sample_range_m = float(z["surface_sample_range_m"])
    cfg.max_sdf_std_ratio = float(z["max_sdf_std_ratio"])
    cfg.reg_iter_n = int(z["reg_iter_n"])
    tr = Tracker(cfg, nm, dec)
    hist = []

    def recording_step(i, delta, st):   # every registration iteration the loop ran
        solved = st[4] > 0
        d = delta if isinstance(delta, np.ndarray) else _np(delta)
        hist.append((d if solved else np.eye(4), float(st[1]) if solved else 0.0, int(st[0])))

    tr._iteration_done = recording_step
    src = torch.as_tensor(z["source"], device=dev)
    if mode == "sorted":
        assert nm.backend() == "grid"
    T, cov, _, valid = tr.tracking(src, torch.eye(4, dtype=torch.float64, device=dev), cur_ts=9)
    assert tr.last_iterations == len(hist)
    assert len(hist) == z["tracking_delta_T"].shape[0]
    for i, (dT, res, cnt) in enumerate(hist):
        np.testing.assert_allclose(dT, z["tracking_delta_T"][i], atol=5e-5, err_msg=f"iteration {i}")
        assert res == pytest.approx(float(z["tracking_resid_cm"][i]), rel=1e-3)
        assert abs(cnt - int(z["tracking_valid_count"][i])) <= 3
    assert bool(valid) == bool(z["tracking_valid"])
    np.testing.assert_allclose(_np(T), z["tracking_T"], atol=1e-4)

