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

