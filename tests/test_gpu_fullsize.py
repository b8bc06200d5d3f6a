"""Parity at BASELINE.json's full sizes (configs[1]: 1M-point map, 262,144 SDF+grad queries;
configs[3]: 4M-point map, 1M-row mapper batch), through the same entry points bench.py times.

The oracle (numpy) checks a strided subset of each batch: neighbour counts exact, SDF within the
north_star's 1e-5, gradients within the parity tolerance of test_gpu_parity.  Whole-batch
properties hold for every query: each query's outputs are independent of the batch order
(bitwise, under a random permutation), repeat calls are bitwise identical, counts lie in
[0, Kc], every output is finite.  The mapper's feature-gradient scatter (float atomics) is
checked against a torch index_add_ of the same per-row contributions."""
import numpy as np
import pytest
import torch

from oracle import pin_oracle as O
from tests import helpers as H
from tests.test_gpu_parity import SDF_ATOL, assert_grad_close

pytestmark = pytest.mark.gpu

N_SIDE, N_QUERY = 1000, 262144     # bench.py configs[1]
MAPPER_SIDE, MAPPER_BATCH = 2000, 1 << 20   # bench.py configs[3]


def _np(t):
    return t.detach().cpu().numpy()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


@pytest.mark.parametrize("wf", [True, False])
def test_headline_batch_vs_oracle(dev, wf):
    import pin_slam_amd as P
    nm, dec, pts = H.surface_map(N_SIDE, device=dev, buffer_size=int(5e7), weighted_first=wf)
    assert nm.count() == N_SIDE * N_SIDE and nm.backend() == "grid"
    q = H.surface_queries(pts, N_QUERY, seed=7, device=dev)

    def run(x):
        return P.query_sdf(nm, dec, x, query_locally=False, want_grad=True, want_certainty=False, want_std=True)
    sdf, grad, nn, _, std = run(q)
    torch.cuda.synchronize()
    # whole batch: finite outputs, counts in range, repeat and permutation invariance
    assert bool(torch.isfinite(sdf).all()) and bool(torch.isfinite(grad).all()) and bool(torch.isfinite(std).all())
    assert int(nn.min()) >= 0 and int(nn.max()) <= int(nm.neighbor_K)
    again = run(q)
    for a, b in zip(again, (sdf, grad, nn, None, std)):
        if b is not None:
            assert torch.equal(a, b)
    perm = torch.randperm(N_QUERY, generator=torch.Generator().manual_seed(3)).to(dev)
    ps, pg, pn, _, pd = run(q[perm].contiguous())
    assert torch.equal(ps, sdf[perm]) and torch.equal(pg, grad[perm]) and torch.equal(pn, nn[perm])
    assert torch.equal(pd, std[perm])
    # strided subset against the oracle
    sub = torch.arange(0, N_QUERY, 61, device=dev)
    st, mlp = H.oracle_state(nm), H.oracle_mlp(dec)
    osdf, ograd, ostd, oq = O.sdf_and_grad(st, mlp, _np(q[sub]), 8, O.neighbor_offsets(2, 0.2), nm.max_valid_dist2,
                                           wf, False)
    np.testing.assert_array_equal(_np(nn[sub]), oq.nn_counts)
    np.testing.assert_allclose(_np(sdf[sub]), osdf, rtol=0, atol=SDF_ATOL)
    assert_grad_close(_np(grad[sub]), ograd)
    if not wf:
        np.testing.assert_allclose(_np(std[sub]), ostd, rtol=0, atol=SDF_ATOL)


def test_mapper_batch_scatter_and_sdf(dev):
    """One configs[3] iteration (4M-point map, 1M batch rows + 6 x 100K stencil rows, frozen
    decoder): batch-row SDFs against the oracle on a subset, and the float-atomic feature
    gradient against torch.index_add_ of the saved per-row contributions (dL/dsdf x w_j x
    s dsdf/dx[0:8], the PIN_TRAIN_DX path)."""
    import pin_slam_amd as P
    from pin_slam_amd import _lib
    from pin_slam_amd.synthetic import surface_pool
    nm, dec, pts = H.surface_map(MAPPER_SIDE, device=dev, buffer_size=int(5e7))
    for p in dec.parameters():
        p.requires_grad_(False)
    cfg = nm.config
    cfg.bs = MAPPER_BATCH
    coord, label, ts = surface_pool(pts, MAPPER_BATCH, seed=11, device=dev)
    mapper = P.Mapper(cfg, None, nm, dec)
    fg = torch.zeros_like(nm.local_geo_features.data)
    loss = float(mapper.train_step(coord, label, ts, fg))
    assert np.isfinite(loss)
    b = mapper._buf
    n = MAPPER_BATCH
    # batch-row SDF (training-mode query: same values as inference) on a strided subset
    sub = torch.arange(0, n, 257, device=dev)
    st, mlp = H.oracle_state(nm), H.oracle_mlp(dec)
    osdf, _, _, _ = O.sdf_and_grad(st, mlp, _np(coord[sub]), 8, O.neighbor_offsets(2, 0.2), nm.max_valid_dist2,
                                   True, True)
    np.testing.assert_allclose(_np(mapper.last_sdf[sub]), osdf, rtol=0, atol=SDF_ATOL)
    # scatter == index_add_ of the per-slot contributions the backward scattered
    nd = (n + cfg.gradient_decimation - 1) // cfg.gradient_decimation
    rows = n + 6 * nd
    order = b.rows4[:rows, 3].contiguous().view(torch.int32).long() if mapper._order is not None else \
        torch.arange(rows, device=dev)
    dsdf = _row_dsdf(b.sdf[:rows], label, n, nd, cfg, float(np.float32(mapper.sdf_scale)))
    dx = b.x.view(-1)[:rows * _lib.FEATURE_DIM].view(rows, 1, _lib.FEATURE_DIM)   # PIN_TRAIN_DX: [rows, 8]
    contrib = dsdf[order][:, None, None] * b.weights[:rows, :, None] * dx
    ids = b.ids[:rows].long()
    ok = ids >= 0
    want = torch.zeros_like(fg, dtype=torch.float64)
    want.index_add_(0, ids[ok], contrib[ok].double())
    torch.testing.assert_close(fg.double(), want, rtol=1e-4, atol=1e-9)


def _row_dsdf(sdf, label, n, nd, cfg, sigma):
    """dL/dsdf per row (original order) of BCE(sdf/s, sigmoid(label/s)) over the n batch rows
    (utils/loss.py:40-47) + weight_e * mean((|g| - 1)^2) through the 6 * nd stencil rows
    (utils/mapper.py:546-547, central differences with step eps), in float64."""
    s = sdf.double()
    y = torch.sigmoid(label.double() / sigma)
    out = torch.zeros_like(s)
    out[:n] = (torch.sigmoid(s[:n] / sigma) - y) / (n * sigma)
    eps = float(np.float32(cfg.voxel_size_m * cfg.num_grad_step_ratio))
    st = s[n:].view(6, nd)
    g = (st[0::2] - st[1::2]) / (2 * eps)            # [3, nd]
    norm = g.norm(dim=0)
    coef = cfg.weight_e * 2 * (norm - 1) / torch.where(norm > 0, norm, torch.ones_like(norm)) / nd
    dg = coef[None, :] * g / (2 * eps)                # d/d s_plus; d/d s_minus = -that
    sten = torch.stack([dg[0], -dg[0], dg[1], -dg[1], dg[2], -dg[2]])
    out[n:] = sten.reshape(-1)
    return out


# ------------------------------------------------------------------ configs[2]: 200K-point registration
@pytest.fixture(scope="module")
def street(dev):
    from pin_slam_amd.synthetic import Q_SCALE, lidar_scan, perturb_pose, street_map
    from pin_slam_amd.tracker import transform_points
    nm, dec, cfg, scene, poses, rng = street_map(12, device=dev)
    T_true = poses[12]
    scan = torch.from_numpy(lidar_scan(T_true, scene, rng, cols=3200).astype(np.float32) / np.float32(Q_SCALE)).to(dev)
    guess = torch.tensor(perturb_pose(T_true), dtype=torch.float64, device=dev)
    return nm, dec, cfg, T_true, scan, guess, transform_points(scan, guess)


def test_registration_200k_tile_order_and_point_split(dev, street):
    """configs[2] (bench.py tracker leg): one registration step of a ~200K-point KITTI-style scan.
    The tile-sorted query (outputs and normal equations in tile order) gives the same accumulators
    as the unsorted input-order query (f64 sums in another order: rel 1e-9), the same valid points;
    and the accumulators of the two halves of the cloud, summed as the point-sharded Tracker's
    all-reduce does, equal the whole cloud's (the sharded step's increment therefore equals the
    single-process one)."""
    import pin_slam_amd as P
    from pin_slam_amd import query as Q
    nm, dec, cfg, _, scan, _, src = street
    n = src.shape[0]
    assert n > 190_000
    tr = P.Tracker(cfg, nm, dec)
    args = (None, None, cfg.reg_min_grad_norm, cfg.reg_max_grad_norm, cfg.reg_GM_dist_m, cfg.reg_GM_grad,
            cfg.reg_lm_lambda, False)

    def reg(pts):
        valid = torch.empty(pts.shape[0], dtype=torch.uint8, device=dev)
        r = tr._register(pts.contiguous(), *args, valid_out=valid)
        return r["acc"], r["status"], valid.clone()
    acc_t, st_t, v_t = reg(src)
    assert st_t[0] > n // 4, "the registration needs valid points"
    old = Q._TILE_QUERIES
    try:
        Q._TILE_QUERIES = False
        acc_i, st_i, v_i = reg(src)
    finally:
        Q._TILE_QUERIES = old
    assert torch.equal(v_t, v_i) and st_t[0] == st_i[0]
    np.testing.assert_allclose(acc_t, acc_i, rtol=1e-9, atol=1e-9 * np.abs(acc_t).max())
    h = n // 2
    acc_a, _, _ = reg(src[:h])
    acc_b, _, _ = reg(src[h:])
    np.testing.assert_allclose(acc_a + acc_b, acc_t, rtol=1e-9, atol=1e-9 * np.abs(acc_t).max())


def test_tracking_200k_converges_to_true_pose(dev, street):
    """The configs[2] tracking loop from the 0.2 m / 0.5 deg perturbed pose is valid and lands
    within 5 cm / 0.1 deg of the scan's true pose (the street map is built by the mapper's
    deterministic mode, so it is the same map on every run)."""
    import pin_slam_amd as P
    nm, dec, cfg, T_true, scan, guess, _ = street
    tr = P.Tracker(cfg, nm, dec)
    T, _, _, ok = tr.tracking(scan, guess)
    Te = T.cpu().numpy()
    assert ok, tr.last_status
    dR = Te[:3, :3].T @ T_true[:3, :3]
    rot = float(np.degrees(np.arccos(np.clip((np.trace(dR) - 1) / 2, -1.0, 1.0))))
    dt = float(np.linalg.norm(Te[:3, 3] - T_true[:3, 3]))
    print(f"tracking from the perturbed pose: {dt:.4f} m, {rot:.4f} deg from the true pose")
    assert dt <= 0.05 and rot <= 0.1, (dt, rot, Te, T_true)


# ------------------------------------------------------------------ configs[4]: 512^3 mesher grid
def test_mesher_512_slabs_equal_one_pass_and_subset_vs_oracle(dev):
    """configs[4] (bench.py mesher leg): the 512^3 grid at 0.1 m over the 1M-point map, SDF-only
    with zero_empty (Mesher.query_points, utils/mesher.py:41-136).  The z-slab split the bench
    gives each rank (here 4 slabs) reproduces one pass bitwise; a strided subset matches the
    oracle (counts exact, SDF 1e-5, empty cells 0)."""
    from pin_slam_amd.query import query_sdf
    nm, dec, pts = H.surface_map(N_SIDE, device=dev, buffer_size=int(5e7))
    R, res, batch = 512, 0.1, 1 << 20
    lo = pts.mean(0) - 0.5 * R * res

    def grid(z0, z1):
        i = torch.arange(R, device=dev, dtype=torch.float32)
        zs = torch.arange(z0, z1, device=dev, dtype=torch.float32)
        gx, gy, gz = torch.meshgrid(i, i, zs, indexing="ij")
        return torch.stack([gx.reshape(-1), gy.reshape(-1), gz.reshape(-1)], 1) * res + lo.to(dev)

    def run(coord):
        sdf = torch.empty(coord.shape[0], device=dev)
        nn = torch.empty(coord.shape[0], dtype=torch.int32, device=dev)
        for b0 in range(0, coord.shape[0], batch):
            s, _, c, _, _ = query_sdf(nm, dec, coord[b0:b0 + batch], query_locally=False, want_grad=False,
                                      zero_empty=True, want_certainty=False)
            sdf[b0:b0 + batch] = s
            nn[b0:b0 + batch] = c
        return sdf, nn
    coord = grid(0, R)
    sdf, nn = run(coord)
    assert bool(torch.isfinite(sdf).all()) and int(nn.max()) <= int(nm.neighbor_K)
    assert 0.0 < float((nn > 0).float().mean()) < 1.0
    full_sdf, full_nn = sdf.view(R, R, R), nn.view(R, R, R)
    for k in range(4):
        z0, z1 = k * R // 4, (k + 1) * R // 4
        s, c = run(grid(z0, z1))
        assert torch.equal(s.view(R, R, z1 - z0), full_sdf[:, :, z0:z1])
        assert torch.equal(c.view(R, R, z1 - z0), full_nn[:, :, z0:z1])
    del full_sdf, full_nn
    # strided subset, denser where the surface is (the cells with neighbours)
    occ = torch.nonzero(nn > 0).flatten()
    sub = torch.cat((torch.arange(0, coord.shape[0], 100_003, device=dev), occ[::max(1, occ.numel() // 3000)]))
    st, mlp = H.oracle_state(nm), H.oracle_mlp(dec)
    osdf, _, _, oq = O.sdf_and_grad(st, mlp, _np(coord[sub]), 8, O.neighbor_offsets(2, 0.2), nm.max_valid_dist2,
                                    True, False)
    np.testing.assert_array_equal(_np(nn[sub]), oq.nn_counts)
    empty = oq.nn_counts == 0
    assert (_np(sdf[sub])[empty] == 0).all()
    np.testing.assert_allclose(_np(sdf[sub])[~empty], osdf[~empty], rtol=0, atol=SDF_ATOL)
