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
