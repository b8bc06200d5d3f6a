"""Fused mapping iteration (pin_train_forward / pin_train_backward / pin_adam_step) against
the reference's mapper fixtures (utils/mapper.py:443-575 run by tests/golden/gen_golden.py).

Tolerances (fp32; the reference's CPU autograd and our float atomics sum in different
orders): loss rel 1e-5, sdf abs 1e-5, feature grads rel 1e-4 / abs 1e-8, decoder grads
rel 1e-3 / abs 1e-7, certainties rel 1e-5 / abs 1e-4, ts_update exact; Adam fed the
reference's own gradients matches its post-step parameters to rel 1e-6 / abs 1e-7.
"""
import numpy as np
import pytest
import torch

import pin_slam_amd as P
from pin_slam_amd import _lib
from pin_slam_amd.query import tensor_key
from tests import helpers as H

pytestmark = pytest.mark.gpu

BACKENDS = ["hash", "grid"]
CASES = ["mapper_wf", "mapper_nwf"]
MLP_KEYS = ["W1", "b1", "W2", "b2"]


def _np(t):
    return t.detach().cpu().numpy()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


def _setup(z, dev, backend):
    nm = H.neural_points_from_fixture(z, dev, backend=backend)
    assert nm.backend() == backend
    dec = H.decoder_from_fixture(z, nm.config)
    dec.to(dev)
    cfg = nm.config
    assert abs(cfg.voxel_size_m * cfg.num_grad_step_ratio - float(z["num_grad_eps"])) < 1e-12
    assert cfg.gradient_decimation == int(z["gradient_decimation"]) and cfg.weight_e == float(z["weight_e"])
    assert cfg.lr == float(z["lr"]) and cfg.adam_eps == float(z["adam_eps"])
    mapper = P.Mapper(cfg, None, nm, dec)
    assert abs(mapper.sdf_scale - float(z["sigma"])) < 1e-12
    np.testing.assert_array_equal(_np(nm.local_geo_features), z["local_features_before"])
    np.testing.assert_array_equal(_np(nm.local_point_certainties), z["local_cert_before"])
    return nm, dec, mapper


def _split(flat):
    out, off = {}, 0
    for key, n in zip(MLP_KEYS, (64 * 11, 64, 64, 1)):
        out[key] = flat[off:off + n]
        off += n
    return out


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("backend", BACKENDS)
def test_train_step_fixture(golden, dev, backend, case):
    """Each iteration: loss, sdf, feature and decoder gradients and the side effects of the
    fused forward/backward; then Adam on the reference's gradients (isolates the optimiser)."""
    z = golden(case)
    nm, dec, mapper = _setup(z, dev, backend)
    feats = nm.local_geo_features.data
    f_grad = torch.zeros_like(feats)
    f_m, f_v = torch.zeros_like(feats), torch.zeros_like(feats)
    m_grad = torch.zeros((_lib.MLP_GRAD_SIZE,), dtype=torch.float32, device=dev)
    m_m, m_v = torch.zeros_like(m_grad), torch.zeros_like(m_grad)
    params = list(dec.parameters())
    for it in range(int(z["iters"])):
        coord = torch.as_tensor(z[f"it{it}_coord"], device=dev)
        label = torch.as_tensor(z[f"it{it}_label"], device=dev)
        ts = torch.as_tensor(z[f"it{it}_ts"], device=dev)
        loss = mapper.train_step(coord, label, ts, f_grad, m_grad)
        assert float(loss) == pytest.approx(float(z[f"it{it}_loss"]), rel=1e-5)
        np.testing.assert_allclose(_np(mapper.last_sdf), z[f"it{it}_sdf"], atol=1e-5)
        np.testing.assert_allclose(_np(f_grad), z[f"it{it}_feat_grad"], rtol=1e-4, atol=1e-8)
        got = _split(_np(m_grad))
        for key in MLP_KEYS:
            want = z[f"it{it}_grad_{key}"].reshape(-1)
            np.testing.assert_allclose(got[key], want, rtol=1e-3, atol=1e-7, err_msg=key)
        np.testing.assert_allclose(_np(nm.local_point_certainties), z[f"it{it}_cert_after"], rtol=1e-5, atol=1e-4)
        np.testing.assert_array_equal(_np(nm.local_point_ts_update), z[f"it{it}_ts_after"])
        # Adam on the reference's own gradients; zero_grad clears our buffers for the next step
        f_grad.copy_(torch.as_tensor(z[f"it{it}_feat_grad"], device=dev))
        m_grad.copy_(torch.as_tensor(np.concatenate([z[f"it{it}_grad_{k}"].reshape(-1) for k in MLP_KEYS]),
                                     device=dev))
        mapper._adam(feats, f_grad, f_m, f_v, params, m_grad, m_m, m_v, step=it + 1)
        assert float(f_grad.abs().max()) == 0.0 and float(m_grad.abs().max()) == 0.0
        np.testing.assert_allclose(_np(feats), z[f"it{it}_features_after"], rtol=1e-6, atol=1e-7)
        for key, p in zip(MLP_KEYS, params):
            np.testing.assert_allclose(_np(p), z[f"it{it}_{key}_after"], rtol=1e-6, atol=1e-7, err_msg=key)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("backend", BACKENDS)
def test_mapping_call_fixture(golden, dev, backend, case, monkeypatch):
    """Mapper.mapping(iters) end to end on the fixture's batches: global features, certainty
    and ts after assign_local_to_global.  Adam's first step moves every touched feature by
    +-lr whatever the gradient's size, so elements whose reference gradient is within float
    noise of 0 may legitimately take the other sign: at most 0.1% of elements may differ."""
    z = golden(case)
    nm, dec, mapper = _setup(z, dev, backend)
    batches = iter(range(int(z["iters"])))

    def get_batch(global_coord=False):
        it = next(batches)
        coord = torch.as_tensor(z[f"it{it}_coord"], device=dev)
        label = torch.as_tensor(z[f"it{it}_label"], device=dev)
        ts = torch.as_tensor(z[f"it{it}_ts"], device=dev)
        return coord, label, ts, None, None, None, torch.ones_like(label)

    monkeypatch.setattr(mapper, "get_batch", get_batch)
    mapper.mapping(int(z["iters"]))
    got = _np(nm.geo_features)
    want = z["global_features_after"]
    off = ~np.isclose(got, want, rtol=1e-5, atol=1e-6)
    assert off.mean() <= 1e-3, f"{off.sum()} of {off.size} feature elements off"
    np.testing.assert_allclose(_np(nm.point_certainties), z["global_cert_after"], rtol=1e-5, atol=1e-4)
    np.testing.assert_array_equal(_np(nm.point_ts_update), z["global_ts_update_after"])
    for key, p in zip(MLP_KEYS, dec.parameters()):
        np.testing.assert_allclose(_np(p), z[f"it{int(z['iters']) - 1}_{key}_after"], rtol=1e-4, atol=1e-5,
                                   err_msg=key)


@pytest.mark.parametrize("frozen", [True, False])
def test_pair_forward_equals_one_lane_per_row(dev, frozen, monkeypatch):
    """PIN_TRAIN_PAIR (two lanes per row, the candidate list split and merged in reference order):
    the forward's saved state -- neighbour ids, weights, sdf, x -- bitwise that of one lane per
    row, on a batch with many equal-distance candidates (grid-aligned queries); frozen decoder
    (PIN_TRAIN_DX) and training decoder (matrix-core sdf, x saved)."""
    import pin_slam_amd.mapper as M
    from pin_slam_amd.synthetic import surface_map, surface_pool
    res = []
    for pair in (False, True):
        monkeypatch.setattr(M, "_PAIR_ROWS", 1 << 30 if pair else 0)
        nm, dec, pts = surface_map(300, device=dev, weighted_first=True, buffer_size=1 << 22, query_backend="grid")
        if frozen:
            for p in dec.parameters():
                p.requires_grad_(False)
        coord, label, ts = surface_pool(pts, 20000, device=dev)
        # a quarter of the rows on voxel corners: equidistant neighbours (ties in the top-k)
        r = float(nm.resolution)
        coord[::4] = torch.round(coord[::4] / r) * r
        mapper = P.Mapper(nm.config, None, nm, dec)
        fg = torch.zeros_like(nm.local_geo_features.data)
        mg = None if frozen else torch.zeros((_lib.MLP_GRAD_SIZE,), dtype=torch.float32, device=dev)
        loss = float(mapper.train_step(coord, label, ts, fg, mg))
        b = mapper._buf
        rows = b.sdf.shape[0]
        used = b.x.view(-1)[: rows * (8 if frozen else 11)]   # PIN_TRAIN_DX: [rows, 8] in the [rows, 11] buffer
        res.append((loss, b.ids.clone(), b.weights.clone(), b.sdf.clone(), used.clone(), fg))
    (l0, i0, w0, s0, x0, f0), (l1, i1, w1, s1, x1, f1) = res
    assert torch.equal(i0, i1) and torch.equal(w0, w1) and torch.equal(s0, s1) and torch.equal(x0, x1)
    assert l1 == pytest.approx(l0, rel=1e-9)
    np.testing.assert_allclose(_np(f1), _np(f0), rtol=1e-4, atol=1e-9)


@pytest.mark.parametrize("wf", [True, False])
def test_train_step_tile_order_invisible(dev, wf, monkeypatch):
    """Large batches are processed in tile order (pin_train_rows + pin_query_sort): per-row sdf
    and ts are bitwise those of input order, gradients / certainties / loss agree to float-atomic
    reordering."""
    import pin_slam_amd.mapper as M
    from pin_slam_amd.synthetic import surface_map, surface_pool
    res = []
    for tiles in (False, True):
        monkeypatch.setattr(M, "_TILE_QUERIES", tiles)
        nm, dec, pts = surface_map(400, device=dev, weighted_first=wf, buffer_size=1 << 22, query_backend="grid")
        coord, label, ts = surface_pool(pts, 70000, device=dev)
        ts = torch.randint(0, 5, ts.shape, device=dev)
        mapper = P.Mapper(nm.config, None, nm, dec)
        fg = torch.zeros_like(nm.local_geo_features.data)
        mg = torch.zeros((_lib.MLP_GRAD_SIZE,), dtype=torch.float32, device=dev)
        loss = float(mapper.train_step(coord, label, ts, fg, mg))
        assert (mapper._order is not None) == tiles
        res.append((loss, mapper.last_sdf.clone(), fg, mg, nm.local_point_certainties.clone(),
                    nm.local_point_ts_update.clone()))
    (l0, s0, f0, m0, c0, t0), (l1, s1, f1, m1, c1, t1) = res
    assert torch.equal(s0, s1) and torch.equal(t0, t1)
    assert l1 == pytest.approx(l0, rel=1e-9)
    np.testing.assert_allclose(_np(f1), _np(f0), rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(_np(m1), _np(m0), rtol=1e-4, atol=1e-8)
    np.testing.assert_allclose(_np(c1), _np(c0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("wf", [True, False])
@pytest.mark.parametrize("backend", BACKENDS)
def test_matrix_core_train_step_matches_f32(dev, backend, wf, monkeypatch):
    """Frozen decoder on the matrix cores -- weighted_first: the forward saves s dsdf/dx for the
    backward (PIN_TRAIN_DX); per-neighbour: the backward's per-neighbour input gradients --
    feature gradients, loss, sdf, certainties and ts against the f32 VALU path."""
    import pin_slam_amd.mapper as M
    from pin_slam_amd.synthetic import surface_map, surface_pool
    res = []
    for dx in (False, True):
        monkeypatch.setattr(M, "_MLP_PACK", dx)
        nm, dec, pts = surface_map(300, device=dev, weighted_first=wf, buffer_size=1 << 22, query_backend=backend)
        coord, label, ts = surface_pool(pts, 70001, device=dev)
        ts = torch.randint(0, 5, ts.shape, device=dev)
        mapper = P.Mapper(nm.config, None, nm, dec)
        fg = torch.zeros_like(nm.local_geo_features.data)
        loss = float(mapper.train_step(coord, label, ts, fg, None))
        res.append((loss, mapper.last_sdf.clone(), fg, nm.local_point_certainties.clone(),
                    nm.local_point_ts_update.clone()))
    (l0, s0, f0, c0, t0), (l1, s1, f1, c1, t1) = res
    assert torch.equal(t0, t1)
    np.testing.assert_allclose(_np(s1), _np(s0), rtol=0, atol=1e-6)
    assert l1 == pytest.approx(l0, rel=1e-6)
    scale = float(f0.abs().max())
    # per-term error ~1e-6 relative; sums of terms of both signs: absolute slack at 1e-4 of the
    # largest; a hidden unit whose pre-activation sits at 0 can take the other ReLU branch in one
    # of the two decoders (a gradient step of w2 W1): a few elements in 10^5 allowed off
    off = ~np.isclose(_np(f1), _np(f0), rtol=1e-4, atol=1e-4 * scale)
    assert off.mean() <= 1e-4, (off.sum(), off.size)
    np.testing.assert_allclose(_np(c1), _np(c0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("backend", BACKENDS)
def test_nwf_mask_backward_matches_redecode(dev, backend, monkeypatch):
    """Per-neighbour decoding, frozen decoder: the forward's f32 decode saves each neighbour's
    ReLU masks and the backward's input gradients are the matrix-core GEMM2 over them
    (PIN_TRAIN_DX), against the backward re-decoding every neighbour on the matrix cores: the
    same sdf / loss / certainties / ts bitwise (the forward is unchanged), feature gradients within
    the split-f16 rounding (a neighbour at a ReLU kink may take the other branch in one of the two
    decoders: a few elements in 10^5)."""
    import pin_slam_amd.mapper as M
    from pin_slam_amd.synthetic import surface_map, surface_pool
    res = []
    for mask in (False, True):
        monkeypatch.setattr(M, "_NWF_MASK", mask)
        nm, dec, pts = surface_map(300, device=dev, weighted_first=False, buffer_size=1 << 22, query_backend=backend)
        for p in dec.parameters():
            p.requires_grad_(False)
        coord, label, ts = surface_pool(pts, 70001, device=dev)
        ts = torch.randint(0, 5, ts.shape, device=dev)
        mapper = P.Mapper(nm.config, None, nm, dec)
        fg = torch.zeros_like(nm.local_geo_features.data)
        loss = float(mapper.train_step(coord, label, ts, fg, None))
        res.append((loss, mapper.last_sdf.clone(), fg, nm.local_point_certainties.clone(),
                    nm.local_point_ts_update.clone()))
    (l0, s0, f0, c0, t0), (l1, s1, f1, c1, t1) = res
    assert torch.equal(s0, s1) and torch.equal(t0, t1)
    assert l1 == pytest.approx(l0, rel=1e-9)
    scale = float(f0.abs().max())
    off = ~np.isclose(_np(f1), _np(f0), rtol=1e-5, atol=1e-5 * scale)
    assert off.mean() <= 1e-4, (off.sum(), off.size)
    np.testing.assert_allclose(_np(c1), _np(c0), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("det", [False, True])
def test_nwf_sorted_backward_matches_wave_scatter(dev, det, monkeypatch):
    """Per-neighbour decoding, frozen decoder, a batch that scatters straight into the gradient
    (no replicas): k_train_backward_nwf_sorted -- the block's pairs sorted by feature row, each
    pair's term evaluated in sorted order and the runs pre-summed before the atomics, side effects
    on the runs -- against the per-wave unsorted scatter of the same forward (the replica path,
    summed): the same loss / sdf / ts bitwise, feature gradients and certainties to float-sum
    reordering.  det: the fixed-point mode -- two sorted calls bitwise equal."""
    import pin_slam_amd.mapper as M
    from pin_slam_amd.synthetic import surface_map, surface_pool
    res = []
    for sorted_ in (False, True, True):
        # replicas (small-batch path, unsorted scatter) or none (the sorted kernel)
        monkeypatch.setattr(M, "_REPLICA_ROWS", 0 if sorted_ else 1 << 30)
        nm, dec, pts = surface_map(300, device=dev, weighted_first=False, buffer_size=1 << 22, query_backend="grid")
        for p in dec.parameters():
            p.requires_grad_(False)
        coord, label, ts = surface_pool(pts, 70001, device=dev)
        ts = torch.randint(0, 5, ts.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
        mapper = P.Mapper(nm.config, None, nm, dec, deterministic=det)
        fg = torch.zeros_like(nm.local_geo_features.data)
        loss = float(mapper.train_step(coord, label, ts, fg, None))
        res.append((loss, mapper.last_sdf.clone(), fg, nm.local_point_certainties.clone(),
                    nm.local_point_ts_update.clone()))
    (l0, s0, f0, c0, t0), (l1, s1, f1, c1, t1), (l2, s2, f2, c2, t2) = res
    assert torch.equal(s0, s1) and torch.equal(t0, t1)
    assert l1 == pytest.approx(l0, rel=1e-9)
    scale = float(f0.abs().max())
    np.testing.assert_allclose(_np(f1), _np(f0), rtol=1e-5, atol=1e-6 * scale)
    np.testing.assert_allclose(_np(c1), _np(c0), rtol=1e-5, atol=1e-5)
    if det:
        assert torch.equal(f1, f2) and torch.equal(c1, c2) and torch.equal(t1, t2)


def test_frozen_decoder_trains_features_only(golden, dev):
    """Decoder frozen (freeze_model, utils/tools.py:186-191, after freeze_after_frame): the
    decoder parameters stay bit-identical and the features still move."""
    z = golden("mapper_wf")
    nm, dec, mapper = _setup(z, dev, "grid")
    for p in dec.parameters():
        p.requires_grad_(False)
    before = [p.detach().clone() for p in dec.parameters()]
    f0 = nm.local_geo_features.detach().clone()
    coord = torch.as_tensor(z["it0_coord"], device=dev)
    label = torch.as_tensor(z["it0_label"], device=dev)
    ts = torch.as_tensor(z["it0_ts"], device=dev)
    mapper.get_batch = lambda global_coord=False: (coord, label, ts, None, None, None, torch.ones_like(label))
    mapper.mapping(1)
    for b, p in zip(before, dec.parameters()):
        assert torch.equal(b, p.detach())
    moved = (nm.geo_features[nm.local_mask] != f0).any(-1)
    assert int(moved.sum()) > 100


def test_adam_matches_torch(dev):
    """pin_adam_step against torch.optim.Adam on the same device, three steps."""
    g = torch.Generator(device="cpu").manual_seed(0)
    p0 = torch.randn(10007, generator=g)
    grads = [torch.randn(10007, generator=g) * 10 ** (-k) for k in range(3)]
    ref = torch.nn.Parameter(p0.clone().to(dev))
    opt = torch.optim.Adam([ref], lr=0.01, betas=(0.9, 0.99), eps=1e-15, foreach=False)
    mine = p0.clone().to(dev)
    m, v = torch.zeros_like(mine), torch.zeros_like(mine)
    from pin_slam_amd.mapper import adam_scalars
    import ctypes
    for t, gr in enumerate(grads, 1):
        ref.grad = gr.to(dev)
        opt.step()
        gbuf = gr.to(dev).contiguous()
        _lib.call("pin_adam_step", _lib.ptr(mine), _lib.ptr(gbuf), _lib.ptr(m), _lib.ptr(v), mine.numel(),
                  ctypes.byref(adam_scalars(0.01, t, 1e-15)), _lib.stream())
        np.testing.assert_allclose(_np(mine), _np(ref), rtol=1e-6, atol=1e-7)


def test_fused_adam_equals_separate_launches(dev):
    """pin_adam_step_segments (features + the decoder's segments in one launch, the mapper's
    training iteration) against pin_adam_step + pin_adam_segments on copies: bitwise equal."""
    import ctypes
    from pin_slam_amd.mapper import adam_scalars
    g = torch.Generator(device="cpu").manual_seed(1)
    n = 8 * 1237
    sizes = [704, 64, 64, 1]
    fa = [torch.randn(n, generator=g).to(dev) for _ in range(4)]          # param, grad, m, v
    fa[3] = fa[3].abs()
    seg = [torch.randn(k, generator=g).to(dev) for k in sizes]
    sg, sm, sv = (torch.randn(sum(sizes), generator=g).to(dev) for _ in range(3))
    sv = sv.abs()
    fb, segb = [t.clone() for t in fa], [t.clone() for t in seg]
    sgb, smb, svb = sg.clone(), sm.clone(), sv.clone()
    st = adam_scalars(0.01, 3, 1e-15)
    ptrs = (ctypes.c_void_p * 4)(*[t.data_ptr() for t in seg])
    szs = (ctypes.c_int64 * 4)(*sizes)
    _lib.call("pin_adam_step_segments", *[_lib.ptr(t) for t in fa], n, ptrs, szs, 4, _lib.ptr(sg), _lib.ptr(sm),
              _lib.ptr(sv), ctypes.byref(st), _lib.stream())
    _lib.call("pin_adam_step", *[_lib.ptr(t) for t in fb], n, ctypes.byref(st), _lib.stream())
    ptrs_b = (ctypes.c_void_p * 4)(*[t.data_ptr() for t in segb])
    _lib.call("pin_adam_segments", ptrs_b, szs, 4, _lib.ptr(sgb), _lib.ptr(smb), _lib.ptr(svb), ctypes.byref(st),
              _lib.stream())
    torch.cuda.synchronize()
    for a, b in zip(fa + seg + [sg, sm, sv], fb + segb + [sgb, smb, svb]):
        assert torch.equal(a, b)
    assert float(fa[1].abs().max()) == 0.0 and float(sg.abs().max()) == 0.0   # gradients zeroed


def test_train_adam_equals_replica_sum_segments_and_pack(dev):
    """pin_adam_step_train (the dense mapping loop's one optimiser launch) against the separate
    launches on copies: the replicas added into the gradient (k_replica_reduce's order), then
    pin_adam_step_segments, then pin_mlp_pack of the stepped decoder -- bitwise equal parameters,
    moments, zeroed gradients and replicas, and the same operand image."""
    import ctypes
    from pin_slam_amd.mapper import adam_scalars
    from pin_slam_amd.query import mlp_view
    cfg = P.Config(device=dev)
    torch.manual_seed(3)
    decs = [P.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1).to(dev) for _ in range(2)]
    decs[1].load_state_dict(decs[0].state_dict())
    g = torch.Generator(device="cpu").manual_seed(4)
    n, R = 8 * 1237, 8
    fa = [torch.randn(n, generator=g).to(dev) for _ in range(4)]          # param, grad, m, v
    fa[3] = fa[3].abs()
    rep = torch.randn(R * n, generator=g).to(dev)
    sizes = [p.numel() for p in decs[0].parameters()]
    sg, sm, sv = (torch.randn(sum(sizes), generator=g).to(dev) for _ in range(3))
    sv = sv.abs()
    fb, repb = [t.clone() for t in fa], rep.clone()
    sgb, smb, svb = sg.clone(), sm.clone(), sv.clone()
    st = adam_scalars(0.01, 3, 1e-15)
    szs = (ctypes.c_int64 * 4)(*sizes)
    views = [mlp_view(d, packed=True) for d in decs]
    packs = [torch.zeros(_lib.MLP_PACK_BYTES, dtype=torch.uint8, device=dev) for _ in range(2)]
    ptrs = [(ctypes.c_void_p * 4)(*[p.data.data_ptr() for p in d.parameters()]) for d in decs]
    _lib.call("pin_adam_step_train", *[_lib.ptr(t) for t in fa], n, _lib.ptr(rep), R, None, 0, ptrs[0], szs, 4,
              _lib.ptr(sg), _lib.ptr(sm), _lib.ptr(sv), views[0].ref(), _lib.ptr(packs[0]), ctypes.byref(st),
              _lib.stream())
    acc = torch.zeros(n, device=dev)
    for k in range(R):
        acc += repb[k * n:(k + 1) * n]
    fb[1] += acc
    _lib.call("pin_adam_step_segments", *[_lib.ptr(t) for t in fb], n, ptrs[1], szs, 4, _lib.ptr(sgb), _lib.ptr(smb),
              _lib.ptr(svb), ctypes.byref(st), _lib.stream())
    _lib.call("pin_mlp_pack", views[1].ref(), _lib.ptr(packs[1]), _lib.stream())
    torch.cuda.synchronize()
    for a, b in zip(fa + [sg, sm, sv], fb + [sgb, smb, svb]):
        assert torch.equal(a, b)
    for pa, pb in zip(decs[0].parameters(), decs[1].parameters()):
        assert torch.equal(pa, pb)
    assert float(rep.abs().max()) == 0.0 and float(fa[1].abs().max()) == 0.0
    assert torch.equal(packs[0], packs[1])


def test_fresh_moments_flag_equals_zero_moments(dev):
    """PinAdamStep.zero_grad bit 1 (the first step of a fresh optimiser): moments holding garbage
    are taken as zero -- bitwise the step on zeroed moments; features and decoder segments.  Bit 0
    alone zeroes the gradient: zero_grad = 2 (fresh moments, gradient kept) leaves it as it was."""
    import ctypes
    from pin_slam_amd.mapper import adam_scalars
    g = torch.Generator(device="cpu").manual_seed(5)
    n, sizes = 8 * 999, [704, 64, 64, 1]
    p0, gr = torch.randn(n, generator=g).to(dev), torch.randn(n, generator=g).to(dev)
    seg0 = [torch.randn(k, generator=g).to(dev) for k in sizes]
    sgr = torch.randn(sum(sizes), generator=g).to(dev)
    out, grads = [], []
    for zg in (1, 3, 2):
        fresh = bool(zg & 2)
        p, gg = p0.clone(), gr.clone()
        m = torch.full_like(p, float("nan")) if fresh else torch.zeros_like(p)
        v = torch.full_like(p, float("nan")) if fresh else torch.zeros_like(p)
        seg = [t.clone() for t in seg0]
        sg = sgr.clone()
        sm = torch.full_like(sg, float("nan")) if fresh else torch.zeros_like(sg)
        sv = torch.full_like(sg, float("nan")) if fresh else torch.zeros_like(sg)
        ptrs = (ctypes.c_void_p * 4)(*[t.data_ptr() for t in seg])
        szs = (ctypes.c_int64 * 4)(*sizes)
        st = adam_scalars(0.01, 1, 1e-15, zero_grad=zg)
        _lib.call("pin_adam_step_train", _lib.ptr(p), _lib.ptr(gg), _lib.ptr(m), _lib.ptr(v), n, None, 0, None, 0,
                  ptrs, szs, 4, _lib.ptr(sg), _lib.ptr(sm), _lib.ptr(sv), None, None, ctypes.byref(st),
                  _lib.stream())
        torch.cuda.synchronize()
        out.append([p, m, v, sm, sv] + seg)
        grads.append((gg, sg))
    for k in (1, 2):
        for a, b in zip(out[0], out[k]):
            assert torch.equal(a, b)
    assert float(grads[1][0].abs().max()) == 0.0 and float(grads[1][1].abs().max()) == 0.0
    assert torch.equal(grads[2][0], gr) and torch.equal(grads[2][1], sgr)


def test_split_gather_equals_concatenated_index(dev):
    """pin_train_gather_packed_split (get_batch's history draw + new_idx[draw], utils/mapper.py:
    335-340) against pin_train_gather_packed over the torch.cat of the same rows: bitwise equal
    rows (batch + stencil), labels, ts, weights; a draw outside new_idx is clamped and reported."""
    import ctypes
    g = torch.Generator(device="cpu").manual_seed(2)
    N, n_hist, n_new, n_sel = 5000, 700, 324, 300
    coord = torch.randn(N, 3, generator=g).to(dev)
    label = torch.randn(N, generator=g).to(dev)
    ts = torch.randint(0, 1 << 40, (N,), generator=g).to(dev)
    weight = torch.randn(N, generator=g).to(dev)
    packed = P.Mapper._pack(coord, label, ts, weight)
    index = torch.randint(0, N, (n_hist,), generator=g).to(dev)
    new_sel = torch.randint(0, N, (n_sel,), generator=g).to(dev)
    draw = torch.randint(0, n_sel, (n_new,), generator=g).to(dev)
    n = n_hist + n_new
    cfg = _lib.PinTrainCfg(n_main=n, n_stencil=(n + 9) // 10, decimation=10, nn_k=8, weighted_first=1, eps=0.06,
                           sigma=0.1, weight_e=0.1, grad_scale=1.0, flags=0, n_tail=0, grad_scale_tail=0.0)
    rows = n + 6 * cfg.n_stencil

    def outs():
        return (torch.empty(rows * 3, device=dev), torch.empty(n, device=dev),
                torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, device=dev),
                torch.zeros(1, dtype=torch.int32, device=dev))
    a, b = outs(), outs()
    full = torch.cat((index, new_sel[draw]))
    _lib.call("pin_train_gather_packed", _lib.ptr(packed), N, _lib.ptr(full), ctypes.byref(cfg),
              *[_lib.ptr(t) for t in a], _lib.stream())
    _lib.call("pin_train_gather_packed_split", _lib.ptr(packed), N, _lib.ptr(index), n_hist, _lib.ptr(new_sel), n_sel,
              _lib.ptr(draw), ctypes.byref(cfg), *[_lib.ptr(t) for t in b], _lib.stream())
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert int(b[4].item()) == 0
    bad = draw.clone()
    bad[5] = n_sel
    c = outs()
    _lib.call("pin_train_gather_packed_split", _lib.ptr(packed), N, _lib.ptr(index), n_hist, _lib.ptr(new_sel), n_sel,
              _lib.ptr(bad), ctypes.byref(cfg), *[_lib.ptr(t) for t in c], _lib.stream())
    torch.cuda.synchronize()
    assert int(c[4].item()) == 1


def _mix64(z):
    m = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def test_device_batch_draws(dev):
    """pin_train_gather_packed_draw (get_batch's two torch.randint draws replaced by a counter-based
    generator in the gather): the gathered rows are exactly the pool rows of the host restatement
    of the draws (history rows uniform over the pool, new rows new_idx[uniform]); the same
    (seed, counter) repeats the batch, another counter gives another one; the history draws are
    uniform (chi-square over 64 bins)."""
    import ctypes
    g = torch.Generator(device="cpu").manual_seed(9)
    N, n_hist, n_new, n_sel = 50000, 7000, 1200, 900
    coord = torch.randn(N, 3, generator=g).to(dev)
    label = torch.randn(N, generator=g).to(dev)
    ts = torch.randint(0, 1 << 40, (N,), generator=g).to(dev)
    weight = torch.randn(N, generator=g).to(dev)
    packed = P.Mapper._pack(coord, label, ts, weight)
    new_sel = torch.randint(0, N, (n_sel,), generator=g).to(dev)
    n = n_hist + n_new
    cfg = _lib.PinTrainCfg(n_main=n, n_stencil=(n + 9) // 10, decimation=10, nn_k=8, weighted_first=1, eps=0.06,
                           sigma=0.1, weight_e=0.1, grad_scale=1.0, flags=0, n_tail=0, grad_scale_tail=0.0)
    rows = n + 6 * cfg.n_stencil

    def run(seed, ctr):
        o = (torch.empty(rows * 3, device=dev), torch.empty(n, device=dev), torch.empty(n, dtype=torch.int64, device=dev),
             torch.empty(n, device=dev), torch.zeros(1, dtype=torch.int32, device=dev))
        _lib.call("pin_train_gather_packed_draw", _lib.ptr(packed), N, n_hist, _lib.ptr(new_sel), n_sel, seed, ctr,
                  ctypes.byref(cfg), *[_lib.ptr(t) for t in o], _lib.stream())
        torch.cuda.synchronize()
        return o
    seed, ctr = 0x1234_5678_9ABC_DEF0, 7
    a, b, c = run(seed, ctr), run(seed, ctr), run(seed, ctr + 1)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert not torch.equal(a[1], c[1])
    key = _mix64(seed ^ _mix64(ctr))
    m = (1 << 64) - 1
    idx = []
    for r in range(n):
        u = _mix64((key + r * 0x9E3779B97F4A7C15) & m)
        idx.append((u * (N if r < n_hist else n_sel)) >> 64)
    idx = np.array(idx)
    pool_rows = np.concatenate([idx[:n_hist], _np(new_sel)[idx[n_hist:]]])
    np.testing.assert_array_equal(_np(a[0])[: 3 * n].reshape(n, 3), _np(coord)[pool_rows])
    np.testing.assert_array_equal(_np(a[1]), _np(label)[pool_rows])
    np.testing.assert_array_equal(_np(a[2]), _np(ts)[pool_rows])
    np.testing.assert_array_equal(_np(a[3]), np.abs(_np(weight)[pool_rows]))
    assert int(a[4].item()) == 0
    counts = np.bincount(idx[:n_hist] * 64 // N, minlength=64)
    chi2 = float(((counts - n_hist / 64) ** 2 / (n_hist / 64)).sum())
    assert chi2 < 120, chi2    # 63 degrees of freedom: p ~ 1e-5 at 120
    # the new-sample rows: positions in new_idx, uniform over [0, n_sel)
    assert idx[n_hist:].min() >= 0 and idx[n_hist:].max() < n_sel and idx[:n_hist].max() < N
    counts = np.bincount(idx[n_hist:] * 16 // n_sel, minlength=16)
    chi2 = float(((counts - n_new / 16) ** 2 / (n_new / 16)).sum())
    assert chi2 < 45, chi2     # 15 degrees of freedom: p ~ 1e-4 at 45


def test_device_draws_leave_the_cpu_generator_alone(dev):
    """mapping()'s device draws take their seed from the device's torch generator (seed + Philox
    offset, advanced per call) -- the CPU generator's stream is untouched, torch.manual_seed fixes
    the run (two calls from the same seed draw the same batches) and consecutive calls differ."""
    from pin_slam_amd.synthetic import surface_map, surface_pool

    def call(reseed):
        nm, dec, pts = surface_map(120, device=dev, buffer_size=1 << 20, query_backend="grid", bs=4096)
        coord, label, ts = surface_pool(pts, 30000, seed=5, device=dev)
        mapper = P.Mapper(nm.config, None, nm, dec)
        mapper.set_pool(coord, label, ts)
        if reseed:
            torch.manual_seed(123)
        cpu = torch.get_rng_state()
        mapper.mapping(2)
        assert torch.equal(cpu, torch.get_rng_state()), "mapping() advanced the CPU generator"
        return nm.geo_features.detach().clone()
    a, b = call(True), call(True)
    c = call(False)   # the device generator moved on: another batch
    # the same batches: equal up to float-atomic noise (Adam's sign-sized steps on noise gradients)
    assert float((~torch.isclose(a, b, rtol=1e-4, atol=1e-6)).float().mean()) <= 2e-3
    assert float((~torch.isclose(a, c, rtol=1e-4, atol=1e-6)).float().mean()) >= 0.05


def test_fat_cache_sees_training_writes(dev):
    """Local inference queries read cached copies of the local features and certainties (fat
    compact records).  mapping() writes those through raw pointers (Adam, certainty / ts side
    effects); the cache must be rebuilt, so a query after mapping() equals one on a fresh cache."""
    from pin_slam_amd.synthetic import surface_map, surface_pool
    nm, dec, pts = surface_map(200, device=dev, buffer_size=1 << 22, query_backend="grid")
    for p in dec.parameters():
        p.requires_grad_(False)
    q = surface_pool(pts, 5000, seed=3, device=dev)[0]
    coord, label, ts = surface_pool(pts, 20000, seed=4, device=dev)
    before = P.query_sdf(nm, dec, q, query_locally=True, want_grad=True, want_certainty=True)
    mapper = P.Mapper(nm.config, None, nm, dec)
    mapper.set_pool(coord, label, ts)
    mapper.mapping(2)
    after = P.query_sdf(nm, dec, q, query_locally=True, want_grad=True, want_certainty=True)
    nm._cache = {}
    fresh = P.query_sdf(nm, dec, q, query_locally=True, want_grad=True, want_certainty=True)
    assert not torch.equal(before[0], fresh[0])          # training moved the SDF
    for a, b in zip(after, fresh):
        if a is not None:
            assert torch.equal(a, b)


def test_decoder_image_sees_training_writes(dev):
    """With the decoder training, Adam updates its parameters through raw pointers; the gradient
    queries decode on the matrix cores from an operand image cached per parameter version, so a
    query after mapping() must equal one through a fresh copy of the trained decoder."""
    from pin_slam_amd.synthetic import surface_map, surface_pool
    nm, dec, pts = surface_map(200, device=dev, buffer_size=1 << 22, query_backend="grid")
    for p in dec.parameters():
        p.requires_grad_(True)
    q = surface_pool(pts, 5000, seed=3, device=dev)[0]
    coord, label, ts = surface_pool(pts, 20000, seed=4, device=dev)
    before = P.query_sdf(nm, dec, q, query_locally=True, want_grad=True)
    w0 = [p.detach().clone() for p in dec.parameters()]
    mapper = P.Mapper(nm.config, None, nm, dec)
    mapper.set_pool(coord, label, ts)
    mapper.mapping(3)
    assert max((p - w).abs().max().item() for p, w in zip(dec.parameters(), w0)) > 0   # the decoder moved
    # the loop's last Adam launch re-packed the image: mapping() caches it under the new parameter
    # versions (mlp_view_repacked), so this query does not pack again
    hit = dec.__dict__.get("_pin_mlp_view")
    assert hit is not None and hit[1].struct.packed == dec.__dict__["_pin_mlp_pack_buf"].data_ptr()
    assert hit[0] == (tensor_key((dec.layers[0].weight, dec.layers[0].bias, dec.lout.weight, dec.lout.bias)),
                      float(dec.sdf_scale))
    after = P.query_sdf(nm, dec, q, query_locally=True, want_grad=True)
    copy = P.Decoder(nm.config, 64, 1, 1)
    copy.load_state_dict(dec.state_dict())
    fresh = P.query_sdf(nm, copy, q, query_locally=True, want_grad=True)
    # the cached image is byte for byte the fresh decoder's pin_mlp_pack image
    assert torch.equal(dec.__dict__["_pin_mlp_pack_buf"], copy.__dict__["_pin_mlp_pack_buf"])
    assert not torch.equal(before[0], after[0])
    torch.testing.assert_close(after[0], fresh[0], rtol=0, atol=0)
    torch.testing.assert_close(after[1], fresh[1], rtol=0, atol=0)


def test_fused_gather_path_matches_get_batch(dev):
    """mapping() with get_batch's gathers fused into pin_train_gather gives the same features,
    certainties and ts as mapping() through get_batch (same draws: the batch index is drawn by
    the same code), up to float-atomic reordering of the gradient sums."""
    from pin_slam_amd.synthetic import surface_map, surface_pool
    outs = []
    for fused in (True, False):
        nm, dec, pts = surface_map(300, device=dev, buffer_size=1 << 22, query_backend="grid", bs=70000)
        for p in dec.parameters():
            p.requires_grad_(False)
        coord, label, ts = surface_pool(pts, 200000, seed=5, device=dev)
        ts = torch.randint(0, 4, ts.shape, device=dev)
        mapper = P.Mapper(nm.config, None, nm, dec)
        mapper.set_pool(coord, label, ts)
        mapper.device_draws = False    # both paths draw with torch.randint (the same draws)
        if not fused:
            mapper.get_batch = lambda global_coord=False, m=mapper: P.Mapper.get_batch(m, global_coord)
        torch.manual_seed(77)
        mapper.mapping(3)
        outs.append((nm.geo_features.clone(), nm.point_certainties.clone(), nm.point_ts_update.clone(),
                     float(mapper.last_loss)))
    (f0, c0, t0, l0), (f1, c1, t1, l1) = outs
    assert torch.equal(t0, t1)
    assert l0 == pytest.approx(l1, rel=1e-6)
    off = ~torch.isclose(f0, f1, rtol=1e-5, atol=1e-6)
    assert float(off.float().mean()) <= 1e-3
    np.testing.assert_allclose(_np(c0), _np(c1), rtol=1e-5, atol=1e-5)


def test_adam_rows_matches_dense_adam_on_those_rows(dev):
    """pin_adam_rows (the owned rows of a slab-sharded mapper) equals pin_adam_step on those rows
    and leaves every other row, its moments and its gradient untouched."""
    import ctypes
    from pin_slam_amd.mapper import adam_scalars
    g = torch.Generator(device="cpu").manual_seed(1)
    L = 5001
    p0 = torch.randn((L, 8), generator=g).to(dev)
    rows = torch.randperm(L, generator=g)[:1700].sort()[0].to(dev)
    pa, pb = p0.clone(), p0.clone()
    ma, va, mb, vb = (torch.zeros_like(p0) for _ in range(4))
    for t in range(1, 4):
        grad = torch.randn((L, 8), generator=g).to(dev)
        ga, gb = grad.clone(), grad.clone()
        st = adam_scalars(0.01, t, 1e-15)
        _lib.call("pin_adam_rows", _lib.ptr(pa), _lib.ptr(ga), _lib.ptr(ma), _lib.ptr(va), _lib.ptr(rows), rows.numel(),
                  ctypes.byref(st), _lib.stream())
        _lib.call("pin_adam_step", _lib.ptr(pb), _lib.ptr(gb), _lib.ptr(mb), _lib.ptr(vb), pb.numel(),
                  ctypes.byref(st), _lib.stream())
        assert torch.equal(pa[rows], pb[rows]) and torch.equal(ma[rows], mb[rows]) and torch.equal(va[rows], vb[rows])
        other = torch.ones(L, dtype=torch.bool, device=dev)
        other[rows] = False
        assert torch.equal(pa[other], p0[other]) and torch.equal(ga[other], grad[other])
        assert float(ga[rows].abs().max()) == 0.0
        pb[other] = p0[other]
        mb[other] = 0
        vb[other] = 0


# ---------------------------------------------------------------- whole mapping() calls
def _mapping_call_setup(z, dev, backend):
    import json
    import types
    from tests.replay import ReplayDraws, mapping_pool
    nm = H.neural_points_from_fixture(z, dev, backend=backend)
    cfg = nm.config
    for k, v in json.loads(str(z["config_json"])).items():
        setattr(cfg, k, v)
    dec = H.decoder_from_fixture(z, cfg)
    dec.to(dev)
    if bool(z["frozen"]):
        for p in dec.parameters():
            p.requires_grad_(False)
    P_local = nm.local_neural_points.detach().cpu().numpy()
    coord, label, ts, weight = mapping_pool(P_local, int(z["pool_n"]), int(z["pool_seed"]))
    t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    mapper = P.Mapper(cfg, types.SimpleNamespace(stop_status=False), nm, dec)
    mapper.set_pool(t(coord), t(label), t(ts), t(weight))
    n = int(z["pool_n"])
    mapper.new_idx = torch.arange(n - n // 10, n, device=dev)
    replay = ReplayDraws(int(z["replay_seed"]))
    mapper._randint = lambda high, k: torch.from_numpy(replay.randint(high, k)).to(dev)
    return nm, dec, mapper, replay


def _norm(a):
    return float(np.linalg.norm(np.asarray(a, dtype=np.float64).ravel()))


def _first_step_check(z, dev, backend, rel=1e-5):
    """The call's first iteration (same draws): the feature gradient and, while the decoder
    trains, the decoder gradients before Adam's first step against the reference's (it0_*),
    within `rel` of their norm; no element of non-negligible size changes sign."""
    nm, dec, mapper, _ = _mapping_call_setup(z, dev, backend)
    fg = torch.zeros_like(nm.local_geo_features.data)
    mg = None if bool(z["frozen"]) else torch.zeros((_lib.MLP_GRAD_SIZE,), dtype=torch.float32, device=dev)
    mapper.train_step(mapper.global_coord_pool, mapper.sdf_label_pool, mapper.time_pool, fg, mg, 1,
                      index=mapper._batch_index(), weight=mapper.weight_pool)
    g, w = _np(fg), z["it0_feat_grad"]
    assert _norm(g - w) <= rel * _norm(w), ("feature gradient", _norm(g - w) / _norm(w))
    big = np.abs(w) > 1e-4 * np.abs(w).max()
    assert not (np.sign(g) != np.sign(w))[big].any()
    if mg is not None:
        for key, part in _split(_np(mg)).items():
            ref = z[f"it0_grad_{key}"].reshape(-1)
            assert _norm(part - ref) <= rel * _norm(ref), (key, _norm(part - ref) / _norm(ref))


@pytest.mark.parametrize("case", ["mapping_wf", "mapping_wf_frozen", "mapping_nwf_weighted"])
@pytest.mark.parametrize("backend", BACKENDS)
def test_whole_mapping_call_fixture(golden, dev, backend, case):
    """One whole Mapper.mapping(15) call of the reference (tests/golden/gen_golden.py
    gen_mapping_call: fresh Adam, 15 x get_batch with history + new samples, BCE + numerical
    eikonal, backward, step; the draws replayed) -- trainable decoder, frozen decoder (the
    matrix-core PIN_TRAIN_DX path) and per-neighbour decoding with the weighted BCE
    (loss_weight_on).  Tolerances: the first iteration's feature and decoder gradients within 1e-5 of
    their norm (measured ~4e-6; the reference's own 1- vs 8-thread spread is ~1e-6); after the 15
    iterations the features differ by more than 1e-4 on at most 0.5 % of the elements (fresh Adam
    moves an element by +-lr on the sign of its gradient, so float noise at a near-zero gradient
    is amplified -- measured 0.18 % per-neighbour, 0 weighted_first) and by ||.|| <= 3e-3
    ||features moved|| (measured 1.2e-3 per-neighbour); the trained decoder within 1e-4 relative."""
    z = golden(case)
    _first_step_check(z, dev, backend)
    nm, dec, mapper, replay = _mapping_call_setup(z, dev, backend)
    before = nm.geo_features.detach().cpu().numpy().copy()
    mapper.mapping(int(z["iters"]))
    assert replay.calls == 2 * int(z["iters"])
    got = _np(nm.geo_features)
    want = z["global_features_after"]
    off = np.abs(got - want) > 1e-4
    assert off.mean() <= 5e-3, f"{off.sum()} of {off.size} feature elements off by > 1e-4"
    assert _norm(got - want) <= 3e-3 * _norm(want - before), (_norm(got - want), _norm(want - before))
    np.testing.assert_allclose(_np(nm.point_certainties), z["global_cert_after"], rtol=1e-5, atol=1e-4)
    np.testing.assert_array_equal(_np(nm.point_ts_update), z["global_ts_update_after"])
    if not bool(z["frozen"]):
        for key, p in zip(MLP_KEYS, dec.parameters()):
            w = z[f"after_{key}"]
            assert _norm(_np(p) - w) <= 1e-4 * _norm(w), (key, _norm(_np(p) - w), _norm(w))


@pytest.mark.parametrize("case", ["mapping_eik_wf", "mapping_eik_livox"])
@pytest.mark.parametrize("backend", BACKENDS)
def test_analytic_eikonal_mapping_call(golden, dev, backend, case):
    """numerical_grad off: the eikonal term on autograd's dsdf/dq with create_graph=True, a double
    backward (utils/mapper.py:50-54, :481-482, utils/tools.py:174-184), here in closed form
    (PIN_TRAIN_EIK).  Cases: weighted_first, and the run_livox.yaml neural-point settings
    (voxel 0.15, alpha 0.5 -> Kc 81, k 8, per-neighbour decoding, weighted BCE, sigma 0.08).

    The reference's own double backward is ill-conditioned on the per-neighbour case: with 1
    instead of 8 threads its first-step feature gradient moves by 18 % of its norm (queries a few
    mm from a neural point make du/dq ~ 1/d^3, and the terms cancel).  Tolerances: first-step
    gradients within 1e-4 of their norm + 3 x the reference's own spread (fixture spread_norm_*);
    after the 15 iterations the features within 1e-3 ||moved|| + 3 x the reference's spread."""
    z = golden(case)
    nm, dec, mapper, replay = _mapping_call_setup(z, dev, backend)
    assert not bool(nm.config.numerical_grad) and bool(z["require_gradient"])
    fg = torch.zeros_like(nm.local_geo_features.data)
    mg = torch.zeros((_lib.MLP_GRAD_SIZE,), dtype=torch.float32, device=dev)
    mapper.train_step(mapper.global_coord_pool, mapper.sdf_label_pool, mapper.time_pool, fg, mg, 1,
                      index=mapper._batch_index(), weight=mapper.weight_pool)
    g, w = _np(fg), z["it0_feat_grad"]
    tol = 1e-4 * _norm(w) + 3 * float(z["spread_norm_it0_feat_grad"])
    print(f"{case}: first-step feature gradient |ours - ref| {_norm(g - w):.3e}, |ref| {_norm(w):.3e}, "
          f"reference spread {float(z['spread_norm_it0_feat_grad']):.3e}")
    assert _norm(g - w) <= tol, (_norm(g - w), tol)
    for key, part in _split(_np(mg)).items():
        ref = z[f"it0_grad_{key}"].reshape(-1)
        tol = 1e-4 * _norm(ref) + 3 * float(z[f"spread_norm_it0_grad_{key}"])
        print(f"   {key}: |ours - ref| {_norm(part - ref):.3e}, |ref| {_norm(ref):.3e}")
        assert _norm(part - ref) <= tol, (key, _norm(part - ref), tol)
    nm, dec, mapper, replay = _mapping_call_setup(z, dev, backend)
    before = nm.geo_features.detach().cpu().numpy().copy()
    mapper.mapping(int(z["iters"]))
    got, want = _np(nm.geo_features), z["global_features_after"]
    tol = 1e-3 * _norm(want - before) + 3 * float(z["spread_norm_global_features_after"])
    print(f"   after {int(z['iters'])} iterations: |ours - ref| {_norm(got - want):.3e}, moved {_norm(want - before):.3e}")
    assert _norm(got - want) <= tol, (_norm(got - want), tol)


@pytest.mark.parametrize("case", ["mapping_eik_wf", "mapping_eik_livox"])
@pytest.mark.parametrize("backend", BACKENDS)
def test_query_feature_double_backward_matches_reference(golden, dev, backend, case):
    """The reference's own first mapping iteration with numerical_grad off, written with its
    autograd calls on the DROP-IN query_feature (utils/mapper.py:448-573): get_gradient(coord, sdf)
    with create_graph=True (utils/tools.py:174-184), BCE + weight_e * mean((|g| - 1)^2), backward --
    a double backward through QueryFeatureFn.  The feature and decoder gradients must match the
    reference's first-step gradients (it0_*) with the analytic-eikonal test's tolerances (1e-4 of
    their norm + 3 x the reference's own 1- vs 8-thread spread)."""
    import torch.nn as nn
    z = golden(case)
    nm, dec, mapper, _ = _mapping_call_setup(z, dev, backend)
    cfg = nm.config
    assert not bool(cfg.numerical_grad)
    index = mapper._batch_index()                       # the first iteration's draws
    coord = mapper.global_coord_pool[index].clone().requires_grad_(True)
    label = mapper.sdf_label_pool[index]
    ts = mapper.time_pool[index]
    weight = torch.abs(mapper.weight_pool[index]).detach()
    feats = nm.local_geo_features
    feats.grad = None
    for p in dec.parameters():
        p.grad = None
    geo, _, wk, _, _ = nm.query_feature(coord, ts)
    sdf = dec.sdf(geo)
    if not cfg.weighted_first:
        sdf = torch.sum(sdf * wk, dim=1).squeeze(1)
    g = torch.autograd.grad(sdf, coord, torch.ones_like(sdf), create_graph=True, retain_graph=True,
                            only_inputs=True)[0]
    sigma = mapper.sdf_scale
    bce = (nn.BCEWithLogitsLoss(weight=weight) if cfg.loss_weight_on else nn.BCEWithLogitsLoss())(
        sdf / sigma, torch.sigmoid(label / sigma))
    loss = bce + cfg.weight_e * ((g.norm(2, dim=-1) - 1.0) ** 2).mean()
    loss.backward()
    got, want = _np(feats.grad), z["it0_feat_grad"]
    tol = 1e-4 * _norm(want) + 3 * float(z["spread_norm_it0_feat_grad"])
    print(f"{case}: drop-in double backward, feature gradient |ours - ref| {_norm(got - want):.3e} (tol {tol:.3e})")
    assert _norm(got - want) <= tol, (_norm(got - want), tol)
    for key, p in zip(MLP_KEYS, dec.parameters()):
        ref = z[f"it0_grad_{key}"]
        tol = 1e-4 * _norm(ref) + 3 * float(z[f"spread_norm_it0_grad_{key}"])
        assert _norm(_np(p.grad) - ref) <= tol, (key, _norm(_np(p.grad) - ref), tol)


def test_query_feature_backward_first_order_unchanged(golden, dev):
    """Without create_graph the backward stays the native kernel; with it, the differentiable
    restatement gives the same first-order gradients (it is only needed for the second order)."""
    z = golden("mapping_eik_wf")
    nm, dec, mapper, _ = _mapping_call_setup(z, dev, "grid")
    index = mapper._batch_index()
    outs = []
    for create in (False, True):
        coord = mapper.global_coord_pool[index].clone().requires_grad_(True)
        nm.local_geo_features.grad = None
        geo, _, wk, _, _ = nm.query_feature(coord, None, training_mode=False)
        sdf = dec.sdf(geo)
        gq, = torch.autograd.grad(sdf.sum(), coord, create_graph=create, retain_graph=True)
        gf, = torch.autograd.grad(sdf.sum(), nm.local_geo_features, create_graph=create)
        outs.append((gq.detach(), gf.detach()))
    # the parity tolerance for gradients (rel 1e-4 / abs 2e-5): the two
    # evaluate the same terms in another order (measured: 1 of 49,152 elements off by 3e-6)
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-4, atol=2e-5)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("wf", [True, False])
@pytest.mark.parametrize("pgo", [False, True])
def test_native_double_backward_matches_restated(dev, wf, pgo, monkeypatch):
    """The closed-form double backward of query_feature (pin_query_feature_bwd2, behind
    QueryFeatureBwdFn) against autograd over the ATen restatement on the same neighbour sets: a
    second-order loss on both first-order gradients (dL/dq and dL/dfeatures) differentiated w.r.t.
    the features, the decoder and the query points; weighted_first and per-neighbour, with and
    without the after-PGO rotation of the neighbour vectors."""
    import pin_slam_amd.query as Q
    from pin_slam_amd.synthetic import surface_map, surface_queries
    res = []
    for restated in (True, False):
        monkeypatch.setattr(Q, "_QF_RESTATED", restated)
        nm, dec, pts = surface_map(120, device=dev, weighted_first=wf, buffer_size=1 << 20, query_backend="grid")
        if pgo:
            g = torch.Generator(device="cpu").manual_seed(13)
            quat = torch.randn(nm.neural_points.shape[0], 4, generator=g).to(dev)
            nm.point_orientations = quat / quat.norm(dim=1, keepdim=True)
            assert nm.local_count() == nm.count()    # the whole map is local, in the same order
            nm.local_point_orientations = nm.point_orientations.clone()
            nm.after_pgo = True
        q = surface_queries(pts, 3000, seed=5, device=dev).requires_grad_(True)
        feats = nm.local_geo_features
        geo, _, wk, _, _ = nm.query_feature(q, None, training_mode=False)
        sdf = dec.sdf(geo)
        if not wf:
            sdf = torch.sum(sdf * wk, dim=1).squeeze(1)
        gq, gfe = torch.autograd.grad(sdf.sum(), (q, feats), create_graph=True)
        c1 = torch.linspace(-1.0, 1.0, gq.numel(), device=dev).view_as(gq)
        c2 = torch.linspace(0.5, -0.5, gfe.numel(), device=dev).view_as(gfe)
        loss = ((gq.norm(dim=-1) - 1.0) ** 2).mean() + (gq * c1).sum() * 1e-3 + (gfe * c2).sum()
        leaves = [feats, q] + list(dec.parameters())
        outs = torch.autograd.grad(loss, leaves, allow_unused=True)
        res.append([torch.zeros_like(t) if o is None else o for o, t in zip(outs, leaves)])
    names = ["features", "q", "W1", "b1", "W2", "b2"]
    for name, a, b in zip(names, *res):
        print(f"{name}: max |restated| {float(a.abs().max()):.3e}, max |native - restated| {float((a - b).abs().max()):.3e}")
    for name, a, b in zip(names, *res):
        # float32 sums in another order: within 1e-4 of each output's largest element (1e-7 floor)
        assert float((a - b).abs().max()) <= 1e-4 * float(a.abs().max()) + 1e-7, name
