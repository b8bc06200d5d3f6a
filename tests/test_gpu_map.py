"""Map maintenance on the device (pin_map.hip) against the reference's own outputs
(tests/golden/gen_golden.py gen_map_case): voxel down-sampling, NeuralPoints.update over six
frames (collisions in a 2^15-slot table, stale re-inserts, in-frame slot sharing),
reset_local_map in both ts modes, assign_local_to_global, prune_map, recreate_hash (both modes)
and adjust_map.

Exact: every index, count, table entry, mask, global2local entry, timestamp and copied float.
adjust_map's rotated positions / quaternions: abs 1e-5 / 1e-6 (the reference's batched 3x3
product sums in its BLAS's order).  New features are random in both implementations: only
their count, the padding row position and the untouched rows are compared."""
import numpy as np
import pytest
import torch

import pin_slam_amd as P
from pin_slam_amd import neural_points as NP

pytestmark = pytest.mark.gpu

CASES = ["map_seq", "map_seq_mid"]
VDS = ["cloud", "plane", "far", "one", "same_voxel"]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


def _np(t):
    return t.detach().cpu().numpy()


def _t(a, dev, dt=None):
    return torch.as_tensor(np.ascontiguousarray(a), device=dev, dtype=dt)


@pytest.mark.parametrize("key", VDS)
def test_voxel_down_sample(golden, dev, key):
    z = golden("map_seq")
    p = _t(z[f"vds_{key}_points"], dev)
    np.testing.assert_array_equal(_np(NP.voxel_down_sample(p, 0.3)), z[f"vds_{key}_idx"])
    v = _t(z[f"vds_{key}_values"], dev)
    np.testing.assert_array_equal(_np(NP.voxel_down_sample_min_value(p, 0.3, v)), z[f"vds_{key}_min_idx"])


def test_voxel_down_sample_large_random(dev):
    """A 2M-point cloud (multi-block reductions, 8-pass radix sort) against the oracle."""
    from oracle import pin_oracle as O
    g = np.random.default_rng(3)
    p = g.uniform(-40, 40, (2_000_000, 3)).astype(np.float32)
    p[:, 2] *= 0.05
    got = _np(NP.voxel_down_sample(_t(p, dev), 0.3))
    np.testing.assert_array_equal(got, O.voxel_down_sample(p, 0.3))
    val = g.integers(0, 50, p.shape[0]).astype(np.float32)
    got = _np(NP.voxel_down_sample_min_value(_t(p, dev), 0.3, _t(val, dev)))
    np.testing.assert_array_equal(got, O.voxel_down_sample(p, 0.3, val))


def _map(z, dev):
    cfg = P.Config(device=dev, voxel_size_m=float(z["voxel_size_m"]), num_nei_cells=2, search_alpha=0.2,
                   buffer_size=int(z["buffer_size"]), local_map_radius=float(z["local_map_radius"]),
                   local_map_travel_dist_ratio=1.0, use_mid_ts=bool(z["use_mid_ts"]), feature_std=0.0)
    nm = P.NeuralPoints(cfg)
    assert nm.diff_travel_dist_local == float(z["diff_travel_dist_local"])
    nm.travel_dist = _t(z["travel_dist"], dev, torch.float32)
    return nm


def _check_local(nm, z, mask_key, g2l_key=None):
    mask = z[mask_key]
    np.testing.assert_array_equal(_np(nm.local_mask), mask)
    if g2l_key:
        np.testing.assert_array_equal(_np(nm.global2local), z[g2l_key])
    m = mask[:-1]
    np.testing.assert_array_equal(_np(nm.local_neural_points), _np(nm.neural_points)[m])
    np.testing.assert_array_equal(_np(nm.local_point_orientations), _np(nm.point_orientations)[m])
    np.testing.assert_array_equal(_np(nm.local_point_certainties), _np(nm.point_certainties)[m])
    np.testing.assert_array_equal(_np(nm.local_point_ts_update), _np(nm.point_ts_update)[m])
    np.testing.assert_array_equal(_np(nm.local_geo_features), _np(nm.geo_features)[mask])


@pytest.mark.parametrize("case", CASES)
def test_map_sequence(golden, dev, case):
    z = golden(case)
    nm = _map(z, dev)
    last = int(z["frames"]) - 1
    for f in range(int(z["frames"])):
        M0 = nm.count()
        feats_before = _np(nm.geo_features[:-1]).copy()
        pts = _t(z[f"f{f}_points"], dev)
        np.testing.assert_array_equal(_np(NP.voxel_down_sample(pts, nm.resolution)), z[f"f{f}_sample_idx"])
        nm.update(pts, _t(z[f"f{f}_sensor"], dev), torch.eye(3, device=dev), f)
        assert nm.count() == int(z[f"f{f}_count"]), f"frame {f}"
        np.testing.assert_array_equal(_np(nm.buffer_pt_index), z[f"f{f}_table"], err_msg=f"frame {f} table")
        np.testing.assert_array_equal(_np(nm.geo_features[:M0]), feats_before)
        assert nm.geo_features.shape[0] == nm.count() + 1
        _check_local(nm, z, f"f{f}_local_mask", f"f{f}_global2local")
    M = nm.count()
    np.testing.assert_array_equal(_np(nm.neural_points), z["seq_positions"])
    np.testing.assert_array_equal(_np(nm.point_orientations), z["seq_orientations"])
    np.testing.assert_array_equal(_np(nm.point_ts_create), z["seq_ts_create"])
    np.testing.assert_array_equal(_np(nm.point_ts_update), z["seq_ts_update"])
    np.testing.assert_array_equal(_np(nm.point_certainties), z["seq_certainties"])

    # assign_local_to_global: the local copies written back, rows outside the local map untouched
    nm.point_certainties = _t(z["pre_certainties"], dev)
    nm.point_ts_update = _t(z["pre_ts_update"], dev)
    nm.geo_features = _t(z["pre_features"], dev)
    sensor = _t(z[f"f{last}_sensor"], dev)
    nm.reset_local_map(sensor, torch.eye(3, device=dev), last)
    mask = _np(nm.local_mask)
    with torch.no_grad():
        nm.local_geo_features.add_(1.0)
    nm.local_point_certainties += 0.5
    nm.local_point_ts_update.fill_(last)
    nm.assign_local_to_global()
    want_f = z["pre_features"].copy()
    want_f[mask] += np.float32(1.0)
    np.testing.assert_array_equal(_np(nm.geo_features), want_f)
    want_c = z["pre_certainties"].copy()
    want_c[mask[:-1]] += np.float32(0.5)
    np.testing.assert_array_equal(_np(nm.point_certainties), want_c)
    want_t = z["pre_ts_update"].copy()
    want_t[mask[:-1]] = last
    np.testing.assert_array_equal(_np(nm.point_ts_update), want_t)
    np.testing.assert_array_equal(_np(nm.neural_points), z["seq_positions"])

    # prune_map
    nm.point_certainties = _t(z["pre_certainties"], dev)
    nm.point_ts_update = _t(z["pre_ts_update"], dev)
    nm.geo_features = _t(z["pre_features"], dev)
    assert nm.count() == M
    assert nm.prune_map(float(z["prune_thre"])) == bool(z["prune_done"])
    for k, a in [("positions", nm.neural_points), ("orientations", nm.point_orientations),
                 ("ts_create", nm.point_ts_create), ("ts_update", nm.point_ts_update),
                 ("certainties", nm.point_certainties), ("features", nm.geo_features)]:
        np.testing.assert_array_equal(_np(a), z[f"prune_{k}"], err_msg=f"prune {k}")

    # recreate_hash(kept_points=True, with_ts=True) + local map
    nm.recreate_hash(sensor, torch.eye(3, device=dev), kept_points=True, with_ts=True, cur_ts=last)
    np.testing.assert_array_equal(_np(nm.buffer_pt_index), z["rehash_ts_table"])
    _check_local(nm, z, "rehash_ts_local_mask")

    # adjust_map
    nm.point_orientations = _t(z["adjust_orientations_in"], dev)
    nm.adjust_map(_t(z["adjust_pose_diff"], dev))
    np.testing.assert_allclose(_np(nm.neural_points), z["adjust_positions"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(_np(nm.point_orientations), z["adjust_orientations"], rtol=0, atol=1e-6)
    nm.neural_points = _t(z["adjust_positions"], dev)
    nm.point_orientations = _t(z["adjust_orientations"], dev)

    # recreate_hash(kept_points=False, with_ts=False): merge duplicates
    nm.recreate_hash(sensor, torch.eye(3, device=dev), kept_points=False, with_ts=False, cur_ts=last)
    for k, a in [("positions", nm.neural_points), ("orientations", nm.point_orientations),
                 ("ts_create", nm.point_ts_create), ("ts_update", nm.point_ts_update),
                 ("certainties", nm.point_certainties), ("features", nm.geo_features),
                 ("table", nm.buffer_pt_index)]:
        np.testing.assert_array_equal(_np(a), z[f"merge_{k}"], err_msg=f"merge {k}")
    _check_local(nm, z, "merge_local_mask", "merge_global2local")


def test_local_map_f64_sensor_and_ts_mode(golden, dev):
    """An f64 sensor position (the reference's tran_dtype pose) tests distances in f64; the
    delta-ts form (use_travel_dist=False) against a direct evaluation."""
    z = golden("map_seq")
    nm = _map(z, dev)
    for f in range(3):
        nm.update(_t(z[f"f{f}_points"], dev), _t(z[f"f{f}_sensor"], dev), torch.eye(3, device=dev), f)
    p = _np(nm.neural_points).astype(np.float64)
    s = np.array([3.1, -0.7, 1.5])
    nm.reset_local_map(torch.tensor(s, dtype=torch.float64, device=dev), None, 2)
    d2 = ((p - s) ** 2).sum(-1)
    td = z["travel_dist"]
    want = (d2 < 15.0 ** 2) & (np.abs(td[2] - td[_np(nm.point_ts_create)]) < np.float32(15.0))
    np.testing.assert_array_equal(_np(nm.local_mask)[:-1], want)
    nm.reset_local_map(torch.tensor(s, dtype=torch.float32, device=dev), None, 2, use_travel_dist=False,
                       diff_ts_local=1)
    d2f = ((_np(nm.neural_points) - s.astype(np.float32)) ** 2).sum(-1)
    want = (d2f < np.float32(225.0)) & (np.abs(2 - _np(nm.point_ts_create)) < 1)
    np.testing.assert_array_equal(_np(nm.local_mask)[:-1], want)


def test_empty_map_local_and_first_update(dev):
    cfg = P.Config(device=dev, voxel_size_m=0.3, buffer_size=1 << 16, local_map_radius=10.0)
    nm = P.NeuralPoints(cfg)
    nm.travel_dist = torch.zeros(4, device=dev)
    nm.reset_local_map(torch.zeros(3, device=dev), None, 0)
    assert nm.local_count() == 0 and _np(nm.local_mask).tolist() == [True]
    assert _np(nm.global2local).tolist() == [-1]
    pts = torch.rand(1000, 3, device=dev) * 3
    nm.update(pts, torch.zeros(3, device=dev), None, 0)
    assert nm.count() > 0 and nm.count() == int((nm.buffer_pt_index >= 0).sum())


def test_map_update_feeds_queries(golden, dev):
    """The maintained map is immediately queryable: with a collision-free table the grid
    backend is exact after the insert sequence and agrees bitwise with the hash backend."""
    z = golden("map_seq")
    cfg = P.Config(device=dev, voxel_size_m=0.3, num_nei_cells=2, search_alpha=0.2, buffer_size=1 << 22,
                   local_map_radius=15.0, local_map_travel_dist_ratio=1.0)
    nm = P.NeuralPoints(cfg)
    nm.travel_dist = _t(z["travel_dist"], dev, torch.float32)
    for f in range(int(z["frames"])):
        nm.update(_t(z[f"f{f}_points"], dev), _t(z[f"f{f}_sensor"], dev), torch.eye(3, device=dev), f)
    with torch.no_grad():
        nm.geo_features.normal_(0, 0.05)
    nm.reset_local_map(_t(z["f5_sensor"], dev), None, 5)
    dec = P.Decoder(nm.config, 64, 1, 1).to(dev)
    q = nm.neural_points[::7] + 0.05
    out = {}
    for backend in ("hash", "grid"):
        nm.config.query_backend = backend
        assert nm.backend() == backend
        out[backend] = P.query_sdf(nm, dec, q, query_locally=True, want_grad=True)
    assert int((out["hash"][2] > 0).sum()) > q.shape[0] // 2
    for a, b in zip(out["hash"], out["grid"]):
        if a is not None:
            assert torch.equal(a, b)
