"""Edge cases of the HIP path (needs an MI355X): empty and ragged batches, queries with no
neighbours, an empty map, the smallest mapper batch, too few valid points for registration.
Expected values follow the reference's behaviour (file:line in each test)."""
import numpy as np
import pytest
import torch

import pin_slam_amd as P
from oracle import pin_oracle as O
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
