"""Pin the map-maintenance oracle (voxel down-sampling, NeuralPoints.update, reset_local_map,
prune_map, recreate_hash, adjust_map) against the reference's own outputs
(tests/golden/gen_golden.py gen_map_case).  CPU only.

Index, count, table and mask outputs must match exactly; positions moved by adjust_map
(a float 3x3 product whose summation order the reference leaves to its BLAS) within 1e-6."""
import numpy as np
import pytest

from oracle import pin_oracle as O

CASES = ["map_seq", "map_seq_mid"]
VDS = ["cloud", "plane", "far", "one", "same_voxel"]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("key", VDS)
def test_voxel_down_sample(golden, case, key):
    z = golden(case)
    p = z[f"vds_{key}_points"]
    np.testing.assert_array_equal(O.voxel_down_sample(p, 0.3), z[f"vds_{key}_idx"])
    np.testing.assert_array_equal(O.voxel_down_sample(p, 0.3, z[f"vds_{key}_values"]), z[f"vds_{key}_min_idx"])


def test_key_aliasing_is_reproduced(golden):
    """The plane case merges voxels (v, y, 0) and (0, y + 1, 0): fewer samples than occupied voxels."""
    z = golden("map_seq")
    p = z["vds_plane_points"]
    voxels = np.unique(np.floor(p / np.float32(0.3)).astype(np.int64), axis=0).shape[0]
    assert z["vds_plane_idx"].shape[0] < voxels


def replay(z, st_cb=None):
    """Run the fixture's whole maintenance sequence through the oracle, checking each step."""
    use_mid = bool(z["use_mid_ts"])
    radius = float(z["local_map_radius"])
    st = O.empty_map(float(z["voxel_size_m"]), int(z["buffer_size"]), z["travel_dist"],
                     float(z["diff_travel_dist_local"]))
    for f in range(int(z["frames"])):
        sidx = O.map_update(st, z[f"f{f}_points"], f)
        np.testing.assert_array_equal(sidx, z[f"f{f}_sample_idx"], err_msg=f"frame {f} sample_idx")
        assert st.points.shape[0] == int(z[f"f{f}_count"]), f"frame {f} count"
        np.testing.assert_array_equal(st.table, z[f"f{f}_table"], err_msg=f"frame {f} table")
        O.reset_local_map(st, z[f"f{f}_sensor"], f, radius, use_mid)
        np.testing.assert_array_equal(st.local_mask, z[f"f{f}_local_mask"], err_msg=f"frame {f} local mask")
        np.testing.assert_array_equal(st.global2local, z[f"f{f}_global2local"], err_msg=f"frame {f} g2l")
    np.testing.assert_array_equal(st.points, z["seq_positions"])
    np.testing.assert_array_equal(st.orientations, z["seq_orientations"])
    np.testing.assert_array_equal(st.ts_create, z["seq_ts_create"])
    np.testing.assert_array_equal(st.ts_update, z["seq_ts_update"])
    last = int(z["frames"]) - 1
    # prune
    st.certainties = z["pre_certainties"].copy()
    st.ts_update = z["pre_ts_update"].copy()
    st.geo_features = z["pre_features"].copy()
    keep = O.prune_keep(st, float(z["prune_thre"]))
    assert bool(z["prune_done"]) == ((~keep).sum() > 100)
    O.select_rows(st, np.nonzero(keep)[0])
    for k, a in [("positions", st.points), ("orientations", st.orientations), ("ts_create", st.ts_create),
                 ("ts_update", st.ts_update), ("certainties", st.certainties), ("features", st.geo_features)]:
        np.testing.assert_array_equal(a, z[f"prune_{k}"], err_msg=f"prune {k}")
    # recreate_hash(kept_points=True, with_ts=True)
    O.recreate_hash(st, last, kept_points=True, with_ts=True, use_mid_ts=use_mid)
    np.testing.assert_array_equal(st.table, z["rehash_ts_table"])
    O.reset_local_map(st, z[f"f{last}_sensor"], last, radius, use_mid)
    np.testing.assert_array_equal(st.local_mask, z["rehash_ts_local_mask"])
    # adjust_map
    st.orientations = z["adjust_orientations_in"].copy()
    O.adjust_map(st, z["adjust_pose_diff"], use_mid)
    np.testing.assert_allclose(st.points, z["adjust_positions"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(st.orientations, z["adjust_orientations"], rtol=0, atol=1e-6)
    st.points = z["adjust_positions"].copy()  # continue from the reference's exact floats
    st.orientations = z["adjust_orientations"].copy()
    # recreate_hash(kept_points=False, with_ts=False): merge
    O.recreate_hash(st, last, kept_points=False, with_ts=False, use_mid_ts=use_mid)
    for k, a in [("positions", st.points), ("orientations", st.orientations), ("ts_create", st.ts_create),
                 ("ts_update", st.ts_update), ("certainties", st.certainties), ("features", st.geo_features),
                 ("table", st.table)]:
        np.testing.assert_array_equal(a, z[f"merge_{k}"], err_msg=f"merge {k}")
    O.reset_local_map(st, z[f"f{last}_sensor"], last, radius, use_mid)
    np.testing.assert_array_equal(st.local_mask, z["merge_local_mask"])
    np.testing.assert_array_equal(st.global2local, z["merge_global2local"])


@pytest.mark.parametrize("case", CASES)
def test_map_sequence(golden, case):
    replay(golden(case))


def test_sequence_exercises_every_rule(golden):
    """The fixture really contains collisions, stale re-inserts and in-frame slot sharing."""
    z = golden("map_seq")
    B = int(z["buffer_size"])
    res = float(z["voxel_size_m"])
    shared = stale = 0
    for f in range(int(z["frames"])):
        sp = z[f"f{f}_points"][z[f"f{f}_sample_idx"]]
        slots = O.hash_slots(O.voxel_coords(sp, res), B)
        shared += slots.shape[0] - np.unique(slots).shape[0]
        if f:
            stale += int(z[f"f{f}_count"]) - int(z[f"f{f - 1}_count"])
    assert shared > 20 and stale > 1000
