"""Pin the numpy oracle against the golden vectors produced by the reference itself
(tests/golden/gen_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import pin_oracle as O

QUERY_CASES = ["query_wf", "query_nwf", "query_kitti", "query_ties"]


def _cfg(z):
    dx = O.neighbor_offsets(int(z["num_nei_cells"]), float(z["search_alpha"]))
    maxd2 = float(z["map_max_valid_dist2"])
    # resolution is a python float in the reference config (0.3, not float32(0.3))
    res = float(np.float64(round(float(z["map_resolution"]), 6)))
    assert O.max_valid_dist2(int(z["num_nei_cells"]), res) == maxd2
    return dx, maxd2, int(z["nn_k"]), bool(z["weighted_first"])


def test_neighborhoods(golden):
    z = golden("neighborhoods")
    for c, a in [(1, 0.0), (2, 0.2), (2, 0.3), (2, 0.5), (2, 1.0), (2, 2.0), (3, 0.2), (3, 0.5), (3, 1.0)]:
        key = f"c{c}_a{int(round(a * 10))}"
        dx = O.neighbor_offsets(c, a)
        np.testing.assert_array_equal(dx, z[f"{key}_dx"])
        assert dx.shape[0] == int(z[f"{key}_K"])
        assert O.max_valid_dist2(c, 0.3) == pytest.approx(float(z[f"{key}_max_valid_dist2"]), rel=1e-12)
    # counts quoted in model/neural_points.py:441-451
    assert [O.neighbor_offsets(2, a).shape[0] for a in (0.2, 0.3, 0.5, 1.0, 2.0)] == [33, 57, 81, 93, 125]
    assert [O.neighbor_offsets(3, a).shape[0] for a in (0.2, 0.5, 1.0)] == [147, 179, 251]


@pytest.mark.parametrize("case", QUERY_CASES)
def test_table_rebuild(golden, case):
    """The fixture table was built by NeuralPoints.update (voxel down-sample + collision
    handling).  Every stored point must hash to the slot that holds it."""
    z = golden(case)
    st = O.map_from_fixture(z)
    slots = O.hash_slots(O.voxel_coords(st.points, st.resolution), st.buffer_size)
    occupied = z["map_table_slots"]
    vals = z["map_table_vals"]
    np.testing.assert_array_equal(slots[vals], occupied)
    # negative-hash wrap is exercised
    raw = (O.voxel_coords(st.points, st.resolution) * O.PRIMES).sum(-1)
    assert (raw < 0).any() and (raw > 0).any()


@pytest.mark.parametrize("case", QUERY_CASES)
@pytest.mark.parametrize("tf", [0, 1])
def test_radius_search(golden, case, tf):
    z = golden(case)
    st = O.map_from_fixture(z)
    dx, maxd2, _, _ = _cfg(z)
    d2, idx = O.radius_neighborhood_search(st, z["queries"], dx, maxd2, bool(tf))
    np.testing.assert_array_equal(idx, z[f"rns{tf}_idx"])
    np.testing.assert_array_equal(d2, z[f"rns{tf}_dist2"])


@pytest.mark.parametrize("case", QUERY_CASES)
@pytest.mark.parametrize("ql", [0, 1])
def test_query_sdf_grad(golden, case, ql):
    z = golden(case)
    st = O.map_from_fixture(z)
    mlp = O.mlp_from_fixture(z)
    dx, maxd2, k, wf = _cfg(z)
    sdf, grad, std, qry = O.sdf_and_grad(st, mlp, z["queries"], k, dx, maxd2, wf, bool(ql))
    p = f"q{ql}_"
    np.testing.assert_array_equal(qry.nn_counts, z[p + "nn_counts"])
    np.testing.assert_allclose(qry.weights, z[p + "weights"], rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(qry.feat, z[p + "feat"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(qry.certainty, z[p + "certainty"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(sdf, z[p + "sdf"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(grad, z[p + "grad"], rtol=1e-4, atol=2e-5)
    if not wf:
        np.testing.assert_allclose(std, z[p + "sdf_std"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("case", QUERY_CASES)
def test_query_after_pgo(golden, case):
    z = golden(case)
    st = O.map_from_fixture(z)
    st.orientations = z["pgo_point_orientations"].astype(np.float32)
    st.local_orientations = st.orientations[st.local_mask[:-1]]
    st.after_pgo = True
    mlp = O.mlp_from_fixture(z)
    dx, maxd2, k, wf = _cfg(z)
    sdf, grad, std, qry = O.sdf_and_grad(st, mlp, z["queries"], k, dx, maxd2, wf, True)
    np.testing.assert_allclose(qry.feat, z["qpgo_feat"], rtol=1e-5, atol=5e-6)  # cross-product cancellation
    np.testing.assert_allclose(sdf, z["qpgo_sdf"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(grad, z["qpgo_grad"], rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("case", QUERY_CASES)
def test_training_side_effects(golden, case):
    z = golden(case)
    st = O.map_from_fixture(z)
    np.testing.assert_array_equal(st.local_certainties, z["train_cert_before"])
    dx, maxd2, k, wf = _cfg(z)
    O.query_feature(st, z["queries"], k, dx, maxd2, wf, True, True, z["train_query_ts"])
    np.testing.assert_allclose(st.local_certainties, z["train_cert_after"], rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(st.local_ts_update, z["train_ts_after"])


@pytest.mark.parametrize("case", QUERY_CASES)
def test_query_certainty(golden, case):
    z = golden(case)
    st = O.map_from_fixture(z)
    np.testing.assert_array_equal(O.neighbor_offsets(1, 0.0), z["qc_neighbor_dx"])
    c = O.query_certainty(st, z["queries"], st.resolution)
    np.testing.assert_array_equal(c, z["qc_certainty"])


@pytest.mark.parametrize("case", ["mapper_wf", "mapper_nwf"])
def test_mapper_steps(golden, case):
    z = golden(case)
    st = O.map_from_fixture(z)
    mlp = O.mlp_from_fixture(z)
    dx, maxd2, k, wf = _cfg(z)
    np.testing.assert_array_equal(st.local_features, z["local_features_before"])
    lr, eps = float(z["lr"]), float(z["adam_eps"])
    mstate = {key: (np.zeros_like(getattr(mlp, key)), np.zeros_like(getattr(mlp, key))) for key in ("W1", "b1", "W2", "b2")}
    fm, fv = np.zeros_like(st.local_features), np.zeros_like(st.local_features)
    for it in range(int(z["iters"])):
        out = O.mapper_forward_backward(st, mlp, z[f"it{it}_coord"], z[f"it{it}_label"], z[f"it{it}_ts"], k, dx,
                                        maxd2, wf, float(z["sigma"]), float(z["weight_e"]),
                                        int(z["gradient_decimation"]), float(z["num_grad_eps"]))
        assert out["loss"] == pytest.approx(float(z[f"it{it}_loss"]), rel=1e-5)
        np.testing.assert_allclose(out["sdf"], z[f"it{it}_sdf"], atol=1e-6)
        np.testing.assert_allclose(out["numgrad"], z[f"it{it}_numgrad"], rtol=1e-3, atol=2e-4)
        np.testing.assert_allclose(out["feat_grad"], z[f"it{it}_feat_grad"], rtol=1e-4, atol=1e-8)
        for key in ("W1", "b1", "W2", "b2"):
            np.testing.assert_allclose(out["mlp_grads"][key], z[f"it{it}_grad_{key}"], rtol=1e-4, atol=1e-7)
        np.testing.assert_allclose(st.local_certainties, z[f"it{it}_cert_after"], rtol=1e-5, atol=1e-4)
        np.testing.assert_array_equal(st.local_ts_update, z[f"it{it}_ts_after"])
        # Adam on the reference's own gradients: isolates the optimizer arithmetic
        O.adam_step(st.local_features, z[f"it{it}_feat_grad"], fm, fv, it + 1, lr, eps=eps)
        np.testing.assert_allclose(st.local_features, z[f"it{it}_features_after"], rtol=1e-6, atol=1e-7)
        for key in ("W1", "b1", "W2", "b2"):
            p = getattr(mlp, key)
            O.adam_step(p, z[f"it{it}_grad_{key}"], mstate[key][0], mstate[key][1], it + 1, lr, eps=eps)
            np.testing.assert_allclose(p, z[f"it{it}_{key}_after"], rtol=1e-6, atol=1e-7)
    O.assign_local_to_global(st)
    np.testing.assert_allclose(st.geo_features, z["global_features_after"], rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(st.ts_update, z["global_ts_update_after"])


@pytest.mark.parametrize("case", ["tracker_wf", "tracker_nwf"])
def test_tracker_step(golden, case):
    z = golden(case)
    st = O.map_from_fixture(z)
    np.testing.assert_array_equal(st.local_features, z["local_features"])
    mlp = O.mlp_from_fixture(z)
    dx, maxd2, k, wf = _cfg(z)
    src = z["source"]
    sdf, grad, std, qry = O.sdf_and_grad(st, mlp, src, k, dx, maxd2, wf, True)
    np.testing.assert_allclose(sdf, z["sdf"], atol=1e-6)
    np.testing.assert_allclose(grad, z["grad"], rtol=1e-4, atol=2e-5)
    np.testing.assert_array_equal(qry.nn_counts >= k, z["mask"])
    max_std = float(z["surface_sample_range_m"]) * float(z["max_sdf_std_ratio"])
    T, cnt, resid, valid, Nm, gv = O.registration_step(
        st, mlp, src, np.zeros(src.shape[0]), k, dx, maxd2, wf, float(z["reg_min_grad_norm"]),
        float(z["reg_max_grad_norm"]), float(z["reg_GM_dist_m"]), float(z["reg_GM_grad"]),
        float(z["reg_lm_lambda"]), max_std)
    assert cnt == int(z["valid_count"])
    assert resid == pytest.approx(float(z["resid_cm"]), rel=1e-4)
    np.testing.assert_allclose(T, z["delta_T"], atol=2e-6)


def test_mesher_query_points(golden):
    z = golden("mesher_wf")
    st = O.map_from_fixture(z)
    mlp = O.mlp_from_fixture(z)
    dx, maxd2, k, wf = _cfg(z)
    sdf, mask = O.mesher_query_points(st, mlp, z["coord"], k, dx, maxd2, wf, int(z["mesh_min_nn"]))
    np.testing.assert_array_equal(mask, z["mc_mask"])
    np.testing.assert_allclose(sdf, z["sdf"], atol=1e-6)


# ---------------------------------------------------------------- the PyTorch-CPU restatement
def _torch_map(z, ql):
    """oracle.pin_torch_cpu.TorchMap over a fixture's map, global (ql=0) or local (ql=1) mode."""
    import torch
    from oracle import pin_torch_cpu as T
    st = O.map_from_fixture(z)
    dx, maxd2, k, wf = _cfg(z)
    t = torch.from_numpy
    if not ql:
        return T.TorchMap(st.resolution, st.buffer_size, t(st.table), t(st.points), t(st.geo_features),
                          t(st.certainties), dx, maxd2, k, wf), st
    dtd = np.abs(st.travel_dist[st.cur_ts] - st.travel_dist[st.ts_create])
    return T.TorchMap(st.resolution, st.buffer_size, t(st.table), t(st.points), t(st.local_features),
                      t(st.local_certainties), dx, maxd2, k, wf, time_ok=t(dtd < np.float32(st.diff_travel_dist_local)),
                      global2local=t(st.global2local), local_points=t(st.local_points)), st


@pytest.mark.parametrize("case", QUERY_CASES)
@pytest.mark.parametrize("ql", [0, 1])
def test_torch_cpu_query_sdf_grad(golden, case, ql):
    """bench.py's CPU baseline (oracle/pin_torch_cpu.py) reproduces the reference's SDF and
    autograd gradient: nn_count exact, SDF 1e-6, gradient rel 1e-4 / abs 2e-5."""
    import torch
    from oracle import pin_torch_cpu as T
    z = golden(case)
    m, _ = _torch_map(z, ql)
    mlp = T.TorchMLP(z["dec_W1"], z["dec_b1"], z["dec_W2"], z["dec_b2"], float(z["dec_sdf_scale"]))
    sdf, grad, nn = T.sdf_and_grad(m, mlp, torch.from_numpy(z["queries"]))
    p = f"q{ql}_"
    np.testing.assert_array_equal(nn.numpy(), z[p + "nn_counts"])
    np.testing.assert_allclose(sdf.numpy(), z[p + "sdf"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(grad.numpy(), z[p + "grad"], rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("case", ["mapper_wf", "mapper_nwf"])
def test_torch_cpu_mapping_iteration(golden, case):
    """The restatement's mapping iteration: loss and feature / decoder gradients of the
    reference's first iteration (rel 1e-5 / 1e-4)."""
    import torch
    from oracle import pin_torch_cpu as T
    z = golden(case)
    m, st = _torch_map(z, 1)
    mlp = T.TorchMLP(z["dec_W1"], z["dec_b1"], z["dec_W2"], z["dec_b2"], float(z["dec_sdf_scale"]),
                     requires_grad=True)
    feats = torch.nn.Parameter(torch.from_numpy(st.local_features.copy()))

    class NoStep:   # keep the gradients for the comparison
        def zero_grad(self, set_to_none=True):
            feats.grad = None
            for p in mlp.params:
                p.grad = None

        def step(self):
            pass
    loss = T.mapping_iteration(m, mlp, feats, NoStep(), torch.from_numpy(z["it0_coord"]),
                               torch.from_numpy(z["it0_label"]), float(z["sigma"]), float(z["weight_e"]),
                               int(z["gradient_decimation"]), float(z["num_grad_eps"]))
    assert loss == pytest.approx(float(z["it0_loss"]), rel=1e-5)
    np.testing.assert_allclose(feats.grad.numpy(), z["it0_feat_grad"], rtol=1e-4, atol=1e-8)
    for key, p in zip(("W1", "b1", "W2", "b2"), mlp.params):
        np.testing.assert_allclose(p.grad.numpy(), z[f"it0_grad_{key}"].reshape(p.shape), rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("case", ["tracker_wf", "tracker_nwf"])
def test_torch_cpu_registration_step(golden, case):
    """bench.py's tracker CPU baseline (pin_torch_cpu.registration_step): the reference's query
    (SDF 1e-6, gradient, IDW std), its valid-point count and its pose increment
    (utils/tracker.py:277-520)."""
    import torch
    from oracle import pin_torch_cpu as T
    z = golden(case)
    m, _ = _torch_map(z, 1)
    mlp = T.TorchMLP(z["dec_W1"], z["dec_b1"], z["dec_W2"], z["dec_b2"], float(z["dec_sdf_scale"]))
    src = torch.from_numpy(z["source"])
    sdf, grad, nn, std = T.sdf_grad_std(m, mlp, src)
    np.testing.assert_allclose(sdf.numpy(), z["sdf"], atol=1e-6)
    np.testing.assert_allclose(grad.numpy(), z["grad"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(std.numpy(), z["sdf_std"], rtol=1e-4, atol=1e-6)
    k = int(z["nn_k"])
    np.testing.assert_array_equal((nn >= k).numpy(), z["mask"])
    max_std = float(z["surface_sample_range_m"]) * float(z["max_sdf_std_ratio"])
    t, cnt = T.registration_step(m, mlp, src, torch.zeros(src.shape[0]), float(z["reg_min_grad_norm"]),
                                 float(z["reg_max_grad_norm"]), float(z["reg_GM_dist_m"]), float(z["reg_GM_grad"]),
                                 float(z["reg_lm_lambda"]), max_std, k)
    assert cnt == int(z["valid_count"])
    dT = z["delta_T"]
    np.testing.assert_allclose(t[3:].numpy(), dT[:3, 3], atol=2e-6)
    w = t[:3].numpy()
    th = np.linalg.norm(w)
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]) / max(th, 1e-30)
    R = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K    # utils/tools.py expmap (Rodrigues)
    np.testing.assert_allclose(R, dT[:3, :3], atol=2e-6)


def test_torch_cpu_mesher_batch(golden):
    """bench.py's mesher CPU baseline (pin_torch_cpu.sdf_only): the reference's query_points SDF
    and marching-cubes mask (utils/mesher.py:41-136)."""
    import torch
    from oracle import pin_torch_cpu as T
    z = golden("mesher_wf")
    m, _ = _torch_map(z, 0)
    mlp = T.TorchMLP(z["dec_W1"], z["dec_b1"], z["dec_W2"], z["dec_b2"], float(z["dec_sdf_scale"]))
    sdf, mask = T.sdf_only(m, mlp, torch.from_numpy(z["coord"]), int(z["mesh_min_nn"]))
    np.testing.assert_array_equal(mask.numpy(), z["mc_mask"])
    np.testing.assert_allclose(sdf.numpy(), z["sdf"], atol=1e-6)


def test_tie_fixture_needs_the_reference_sort(golden, monkeypatch):
    """query_ties (neural points on cell centres, queries on the half-cell lattice) holds equal
    neighbour distances in almost every row; the reference's features come out in the order its
    unstable sort leaves them, which a stable sort does not reproduce."""
    z = golden("query_ties")
    d2 = np.where(z["rns1_idx"] < 0, 9e3, z["rns1_dist2"])
    s = np.sort(d2, 1)
    assert ((s[:, 1:] == s[:, :-1]) & (s[:, 1:] < 9e3)).any(1).mean() > 0.9
    st = O.map_from_fixture(z)
    mlp = O.mlp_from_fixture(z)
    dx, maxd2, k, wf = _cfg(z)
    monkeypatch.setattr(O, "ref_sort_order", lambda d: np.argsort(d, axis=1, kind="stable"))
    _, _, _, qry = O.sdf_and_grad(st, mlp, z["queries"], k, dx, maxd2, wf, True)
    assert not np.allclose(qry.feat, z["q1_feat"], rtol=1e-5, atol=1e-6)


def antiqsort_row(n):
    """McIlroy's adversary ("A killer adversary for quicksort") run against ref_sort_row: keys
    fixed lazily so that every median-of-three pivot is near the minimum, which drives libstdc++'s
    introsort past its depth limit into the heap sort.  Returns the keys it fixed (distinct)."""
    gas = n
    val = [gas] * n
    state = {"solid": 0, "cand": 0}

    class Item:
        __slots__ = ("i",)

        def __init__(self, i):
            self.i = i

        def __lt__(self, other):
            x, y = self.i, other.i
            if val[x] == gas and val[y] == gas:
                z = x if x == state["cand"] else y
                val[z] = state["solid"]
                state["solid"] += 1
            if val[x] == gas:
                state["cand"] = x
            elif val[y] == gas:
                state["cand"] = y
            return val[x] < val[y]
    O.ref_sort_row([Item(i) for i in range(n)], raw=True)
    return np.asarray(val, np.float32)


def ref_sort_test_rows(n, rng):
    """Rows for the sort restatements: tie-heavy random rows (some with 9e3 entries), sorted and
    reversed rows, and adversarial rows with and without ties (heap-sort fallback)."""
    rows = []
    for t in range(60):
        v = rng.integers(0, max(2, n // 3), n).astype(np.float32)
        if t % 3 == 0:
            v[rng.random(n) < 0.3] = 9e3
        if t % 5 == 0:
            v = np.sort(v)
        if t % 7 == 0:
            v = np.sort(v)[::-1].copy()
        rows.append(v)
    if n >= 17:
        a = antiqsort_row(n)
        rows += [a, np.floor(a / 2).astype(np.float32), np.floor(a / 3).astype(np.float32)]
    return rows


def test_adversarial_rows_reach_the_heap_sort():
    for n in (40, 81, 128):
        a = antiqsort_row(n)
        for w in (a, np.floor(a / 2).astype(np.float32)):
            stats = {}
            O.ref_sort_row(w, stats=stats)
            assert stats.get("heap", 0) > 0, n


@pytest.mark.parametrize("n", [2, 16, 17, 27, 33, 57, 81, 93, 125, 128, 343])
def test_ref_sort_row_is_torch_cpu_sort(n):
    """ref_sort_row restates the sort the reference calls (torch.sort(dists2, dim=1) on the CPU):
    the permutation it leaves rows with many equal keys in, 9e3 entries included, and adversarial
    rows that end in the heap sort."""
    import torch
    for v in ref_sort_test_rows(n, np.random.default_rng(n)):
        _, o = torch.sort(torch.from_numpy(v)[None], dim=1)
        assert O.ref_sort_row(v) == o[0].tolist()
