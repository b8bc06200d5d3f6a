"""BASELINE configs[0], the plumbing run: the reference's pin_slam.py frame loop (:96-257) over
synthetic 64-beam street sequences (64K points per scan): 30 frames of an accelerating street
(three window filters of the sample pool, frames 9, 19, 29) and, since round 5, the 100 frames
BASELINE configs[0] names on a longer street at ~1.2 m/frame (window filters at frames 9..99,
the pool's capacity discards at frame 99); the decoder frozen after frame 15; replayed through
pin_slam_amd's classes and compared with the reference's own run of the same loop
(tests/golden/slam_seq.npz, written by tests/golden/gen_golden.py gen_slam_sequence with the
reference's Tracker / Mapper / NeuralPoints / DataSampler and its dataset bookkeeping methods).

Both runs take every random draw of the sampler and of get_batch from the same ReplayDraws
stream (tests/replay.py), in the reference's call order, so they differ only by floating-point
summation order.  The loop is chaotic in that difference: the reference itself, run again at other
torch thread counts (or even at the same one), ends centimetres apart.  tests/golden/
gen_slam_envelope.py ran the reference's loop 11 times on slam_seq (1-7, 8, 10, 12, 16 threads) and
8 times on slam_seq100 (1, 2, 3, 4, 6, 8, 16 threads and a second 8-thread run) and stored every
run's poses, counts and surface SDFs in the fixture (env_*): that envelope is what a legitimate run
looks like, and the
bounds below place our run in it, widened by stated factors (W_POSE, W_COUNT, W_SURFACE: the
smallest at which every reference run passes against the others), with small floors where the
envelope is a single value.  They were fixed and committed
before the run they judge; a run outside them is a defect to find (first failing frame and part)
and fix, not a bound to widen.  Element-wise feature parity after hundreds of iterations is not a
property the reference has (a single 15-iteration mapping() call is pinned element-wise in
tests/test_gpu_mapper.py::test_whole_mapping_call_fixture).

Both training modes run: deterministic=True (fixed-point gradient and certainty sums,
stable tile order -- two runs are bitwise equal, test_slam_sequence_bitwise_reproducible) and
deterministic=False (float atomics: a run is one draw of our own run-to-run spread).  Checks:
  * preprocessed cloud / source point counts, tracking validity, draw-stream position: exact;
  * pose: |t - c_k| <= max(1 cm, W_POSE x e_k), c_k the mean of the reference runs' positions at
    frame k, e_k the largest distance of any reference run from its frame's mean up to frame k;
    the same for the rotation (chordal mean, angle floor 0.05 deg);
  * counts (neural points, local map, pool, new samples): |n - mean_k| / mean_k within
    max(floor, W_COUNT x the largest relative deviation of a run from its frame's mean up to frame
    k), floors 0.2 %, 0.2 %, 0.01 %, 2 %; at the window-filter frames the pool may instead differ
    from the stored run by the difference carried in plus the samples whose side of the filter
    sphere our pose differences can change (counted on our pre-filter pool: displacement
    |dt_j| + theta_j * range per sample, |dt_k| for the centre);
  * the map's SDF on the surface (scan points placed by the TRUE poses) after frame 0 and at the
    end: mean |SDF| at most the runs' largest + (W_SURFACE - 1) x their range + 1 mm, and the
    median over probes of |ours - the runs' mean| at most W_SURFACE x the largest such median of
    a run + 1 mm;
  * the end-of-run merge (recreate_hash(kept_points=False), pin_slam.py:366) raises where the
    reference's runs do, and otherwise leaves a map whose size passes the count bound against
    the runs' merged sizes.
Every check is made on every frame; the failures are listed together at the end.
"""
import json
import math

import numpy as np
import pytest
import torch

import pin_slam_amd as P
from pin_slam_amd.synthetic import FrameLoop, lidar_scan, sequence_scene
from tests.replay import ReplayDraws

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


def _pose_err(a, b):
    dt = float(np.linalg.norm(a[:3, 3] - b[:3, 3]))
    c = (np.trace(a[:3, :3].T @ b[:3, :3]) - 1.0) / 2.0
    return dt, math.degrees(math.acos(min(1.0, max(-1.0, c))))


# Widening factors of the envelope (module docstring).  Calibrated on the reference alone, before
# any run of ours: the smallest factor, rounded up to 0.5, at which EVERY reference run passes when
# judged against the other runs of its fixture (tests/test_slam_envelope.py recomputes this
# leave-one-out check).  On the first 7 / 8 runs: poses 1.93, counts 4.05 (the reference's own
# outliers: slam_seq100's stored run ends 1.5-1.9 % above the seven others), surface SDF 1.59; with
# slam_seq's four later runs (5, 7, 10, 12 threads): 1.72, 4.05, 1.59 -- the same factors.
W_POSE = 2.0
W_COUNT = 4.5
W_SURFACE = 2.0
COUNT_FLOORS = {"map_count": 0.002, "local_count": 0.002, "pool": 0.0001, "new": 0.02}


def count_check(got, runs, floor):
    """got against the runs' counts up to its frame (runs [R, k+1]): |got - mean| / mean within
    max(floor, W_COUNT x the largest relative deviation of a run from its frame's mean so far)."""
    runs = np.asarray(runs, np.float64)
    m = np.maximum(runs.mean(0), 1.0)
    e = float((np.abs(runs - m[None]) / m[None]).max())
    lim = max(floor, W_COUNT * e)
    return abs(float(got) - m[-1]) / m[-1] <= lim, (m[-1] * (1 - lim), m[-1] * (1 + lim))


def surface_bounds(got, env):
    """The map's SDF at the probes (got [P]) against the runs' (env [R, P]): (ok, message)."""
    got, env = np.asarray(got, np.float64), np.asarray(env, np.float64)
    means = np.abs(env).mean(1)
    mine = float(np.abs(got).mean())
    centre = env.mean(0)
    diff = float(np.median(np.abs(got - centre)))
    run_diff = float(np.median(np.abs(env - centre[None]), axis=1).max())
    mean_lim = float(means.max()) + (W_SURFACE - 1.0) * float(means.max() - means.min()) + 1e-3
    diff_lim = W_SURFACE * run_diff + 1e-3
    msg = (f"mean |SDF| ours {mine:.4f} m, reference runs {np.round(means, 4)} (limit {mean_lim:.4f}); "
           f"median |ours - runs' mean| {diff:.4f} m, runs' largest {run_diff:.4f} m (limit {diff_lim:.4f})")
    return mine <= mean_lim and diff <= diff_lim, msg


def pose_check(T, k, env):
    """Pose T of frame k against pose_envelope(z) = env: (ok, distance, limit, angle, limit)."""
    centre, Rmean, e_t, e_r = env
    d_c = float(np.linalg.norm(T[:3, 3] - centre[k]))
    a_c = _angle(T[:3, :3], Rmean[k])
    tol_t, tol_r = max(0.01, W_POSE * float(e_t[k])), max(0.05, W_POSE * float(e_r[k]))
    return d_c <= tol_t and a_c <= tol_r, d_c, tol_t, a_c, tol_r


def _rot_mean(Rs):
    """Chordal mean of rotation matrices [n, 3, 3]: the arithmetic mean projected onto SO(3)."""
    U, _, Vt = np.linalg.svd(Rs.mean(0))
    D = np.diag([1.0, 1.0, np.sign(np.linalg.det(U @ Vt))])
    return U @ D @ Vt


def _angle(A, B):
    c = (np.trace(A.T @ B) - 1.0) / 2.0
    return math.degrees(math.acos(min(1.0, max(-1.0, c))))


def pose_envelope(z):
    """Per frame: the runs' mean position c_k and mean rotation, and the running maxima e_t(k),
    e_r(k) of any run's distance / angle from its frame's mean (module docstring)."""
    P = np.asarray(z["env_hist_pose"], np.float64)             # [runs, frames, 4, 4]
    c = P[:, :, :3, 3].mean(0)
    Rm = np.stack([_rot_mean(P[:, k, :3, :3]) for k in range(P.shape[1])])
    et = np.maximum.accumulate(np.linalg.norm(P[:, :, :3, 3] - c[None], axis=-1).max(0))
    er = np.maximum.accumulate(np.array([max(_angle(P[r, k, :3, :3], Rm[k]) for r in range(P.shape[0]))
                                         for k in range(P.shape[1])]))
    return c, Rm, et, er


def _surface_check(nm, dec, z, dev, probes_key, sdf_key):
    """The map's SDF at surface points against the reference runs' (surface_bounds)."""
    probes = torch.from_numpy(z[probes_key]).to(dev)
    sdf, _, _, _, _ = P.query_sdf(nm, dec, probes, query_locally=False, want_grad=False, want_certainty=False)
    ok, msg = surface_bounds(sdf.cpu().numpy(), z["env_" + sdf_key])
    print(f"{sdf_key}: {msg}")
    return ok


def _shell_count(pre, ours, ref, k, radius):
    """Samples of our pre-filter pool whose membership in the window-filter sphere (radius around
    the frame-k position, utils/mapper.py:226-262) can differ from the reference's: a sample of
    frame j sits at our pose_j applied to the same sensor-frame point, so it is displaced from the
    reference's by at most |dt_j| + theta_j * r (r: its range from the frame-j sensor, theta_j:
    the rotation difference in radians), and the sphere's centre moves by |dt_k|."""
    x = pre["global_coord"].double()
    fid = pre["time"].long()
    P_o = torch.tensor(np.stack(ours[:k + 1]), dtype=torch.float64, device=x.device)
    P_r = torch.tensor(np.asarray(ref[:k + 1], dtype=np.float64), device=x.device)
    dt = torch.linalg.norm(P_o[:, :3, 3] - P_r[:, :3, 3], dim=1)
    cos = ((P_o[:, :3, :3].transpose(1, 2) @ P_r[:, :3, :3]).diagonal(dim1=1, dim2=2).sum(-1) - 1.0) / 2.0
    theta = torch.arccos(cos.clamp(-1.0, 1.0))
    r = torch.linalg.norm(x - P_o[fid, :3, 3], dim=1)
    disp = dt[fid] + theta[fid] * r + dt[k]
    d = torch.linalg.norm(x - P_o[k, :3, 3], dim=1)
    return int(((d - radius).abs() <= disp).sum())


def _sequence(z, dev, frames):
    """The drop-in classes set up as the fixture's reference run was (config, initial decoder,
    replayed draws) and the scans regenerated from the seed (checked against the digests):
    (nm, dec, mapper, loop, replay, draws, scans)."""
    import hashlib
    conf = json.loads(str(z["config_json"]))
    cfg = P.Config(**conf)
    cfg.device = dev
    nm = P.NeuralPoints(cfg)
    dec = P.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1)
    with torch.no_grad():
        dec.layers[0].weight.copy_(torch.as_tensor(z["dec_init_W1"]))
        dec.layers[0].bias.copy_(torch.as_tensor(z["dec_init_b1"]))
        dec.lout.weight.copy_(torch.as_tensor(z["dec_init_W2"]))
        dec.lout.bias.copy_(torch.as_tensor(z["dec_init_b2"]))
    dec.to(dev)
    tracker = P.Tracker(cfg, nm, dec)
    # the deterministic training mode: the run is a function of the scans and the draws (two runs
    # are bitwise equal), so the bounds judge one reproducible trajectory
    mapper = P.Mapper(cfg, None, nm, dec, deterministic=True)
    loop = FrameLoop(cfg, nm, dec, tracker, mapper)     # pin_slam.py:96-257 on the drop-in classes
    replay = ReplayDraws(int(z["replay_seed"]))
    mapper._randint = lambda high, n: torch.from_numpy(replay.randint(high, n)).to(dev)
    S, Ff, Fb = int(cfg.surface_sample_n), int(cfg.free_front_n), int(cfg.free_behind_n)

    def draws(n):
        return (torch.from_numpy(replay.randn(n * S)), torch.from_numpy(replay.rand(n * Ff)),
                torch.from_numpy(replay.rand(n * Fb)))
    rng = np.random.default_rng(int(z["scan_seed"]))
    scene, poses = sequence_scene(str(z["scene"]) if "scene" in z else "street", rng, int(z["frames"]))
    scans = [lidar_scan(T, scene, rng) for T in poses][:frames]
    for k, sc in enumerate(scans):
        assert hashlib.sha256(np.ascontiguousarray(sc).tobytes()).hexdigest() == str(z["scan_sha256"][k]), \
            f"frame {k}: regenerated scan differs from the reference run's"
    scans = [torch.from_numpy(sc.astype(np.float32) / np.float32(z["q_scale"])).to(dev) for sc in scans]
    return nm, dec, mapper, loop, replay, draws, scans


def test_slam_sequence_bitwise_reproducible(golden, dev):
    """The deterministic mode makes the whole frame loop a function of its inputs: two runs of
    the fixture's first 12 frames (frame 0's 600 mapping iterations, a pool filter, tracking,
    the decoder training) end with bitwise-equal poses, map, features, certainties and decoder."""
    z = golden("slam_seq")
    runs = []
    for _ in range(2):
        nm, dec, mapper, loop, replay, draws, scans = _sequence(z, dev, 12)
        poses = []
        for k, pts in enumerate(scans):
            loop.frame(pts, draws=draws, next_pts=scans[k + 1] if k + 1 < len(scans) else None)
            poses.append(np.array(loop.cur_pose_ref))
        runs.append((np.stack(poses), [nm.neural_points.clone(), nm.geo_features.clone(),
                                       nm.point_certainties.clone(), nm.point_ts_update.clone()]
                     + [p.detach().clone() for p in dec.parameters()]))
    np.testing.assert_array_equal(runs[0][0], runs[1][0])
    for k, (a, b) in enumerate(zip(runs[0][1], runs[1][1])):
        assert torch.equal(a, b), f"state {k} differs between two runs"


@pytest.mark.parametrize("deterministic", [True, False], ids=["det", "atomic"])
@pytest.mark.parametrize("fixture", ["slam_seq", "slam_seq100"])
def test_slam_sequence_matches_reference(golden, dev, fixture, deterministic):
    """slam_seq: 30 frames of the accelerating street; slam_seq100: BASELINE configs[0]'s 100
    frames on the long street (synthetic.sequence_scene("long"); window filters at frames 9..99,
    the pool's capacity discards at frame 99).  Bounds: the module docstring."""
    z = golden(fixture)
    frames = int(z["frames"])
    nm, dec, mapper, loop, replay, draws, scans = _sequence(z, dev, frames)
    mapper.deterministic = deterministic
    cfg = nm.config
    penv = pose_envelope(z)
    report, failures, our_poses = [], [], []
    # the whole pool as each window filter sees it (Mapper._pool_compact_many is called by the
    # filter with the pre-filter pools): the filter frames' pool counts are checked against the
    # geometry
    pre = {}
    compact = mapper._pool_compact_many

    def capture(pools, keep):
        for name, cur in pools:
            if name in ("global_coord", "time"):
                pre[name] = cur.clone()
        return compact(pools, keep)
    mapper._pool_compact_many = capture

    def expect(ok, msg):
        """Soft assertion: every frame is checked and reported, the test fails at the end."""
        if not ok:
            failures.append(msg)
            print("FAIL", msg, flush=True)
    for k in range(frames):
        pts = scans[k]
        seen = {}

        def check(part, k=k):
            """Per-part checks, called by FrameLoop.frame at the end of each part."""
            if part == "tracking":
                assert loop.cur_point_cloud_torch.shape[0] == int(z["hist_n_cloud"][k]), f"frame {k}: cloud size"
                if k > 0:
                    assert loop.cur_source_points.shape[0] == int(z["hist_n_source"][k]), f"frame {k}: source size"
            if part == "process_frame":
                seen["counts"] = (nm.count(), nm.local_count(), int(mapper.pool_sample_count),
                                  int(mapper.new_idx.shape[0]))
        valid = loop.frame(pts, draws=draws, timer=check, next_pts=scans[k + 1] if k + 1 < frames else None)
        assert bool(valid) == bool(z["hist_valid"][k]), f"frame {k}: tracking validity"
        assert replay.calls == int(z["hist_draws_after"][k]), f"frame {k}: draw stream out of step"
        counts = seen["counts"]
        want = tuple(int(z[f"hist_{n_}"][k]) for n_ in ("map_count", "local_count", "pool", "new"))
        T = np.asarray(loop.cur_pose_ref, dtype=np.float64)
        pose_ok, d_c, tol_t, a_c, tol_r = pose_check(T, k, penv)
        dt_true, _ = _pose_err(T, z["truth_poses"][k])
        ref_true = max(_pose_err(Pr, z["truth_poses"][k])[0] for Pr in z["env_hist_pose"][:, k])
        our_poses.append(T)
        report.append((k, round(d_c, 4), round(tol_t, 4), round(a_c, 4), round(tol_r, 4), round(dt_true, 4),
                       round(ref_true, 4), counts, want))
        print("frame", *report[-1], flush=True)
        expect(pose_ok,
               f"frame {k}: pose {d_c:.4f} m / {a_c:.4f} deg from the runs' mean (limits {tol_t:.4f} m / {tol_r:.4f} deg)")
        # implied by the pose bound (triangle inequality); checked for the report
        expect(dt_true <= ref_true + 2 * tol_t, f"frame {k}: pose {dt_true:.4f} m from the ground truth")
        filt = k % int(cfg.pool_filter_freq) == int(cfg.pool_filter_freq) - 1   # the pool's window filter ran
        for name, g, w in zip(("map_count", "local_count", "pool", "new"), counts, want):
            ok, (lo, hi) = count_check(g, z[f"env_hist_{name}"][:, :k + 1], COUNT_FLOORS[name])
            if name == "pool" and filt and not ok:
                # the filter keeps the samples within window_radius of the CURRENT position: beyond
                # the difference carried in from the previous frame, the count can differ from the
                # stored run's only by samples that lie, in our pool, within their displacement
                # bound of the sphere
                prev = report[-2][7][2] - report[-2][8][2] if k > 0 else 0
                lim = abs(prev) + _shell_count(pre, our_poses, z["hist_pose"], k, float(cfg.window_radius))
                print(f"frame {k}: pool {g} vs {w}: |diff| {abs(g - w)}, geometric bound {lim}", flush=True)
                ok = abs(g - w) <= lim
            expect(ok, f"frame {k}: {name} {g} outside the reference runs' envelope [{lo:.0f}, {hi:.0f}]")
        if k == 0:
            expect(_surface_check(nm, dec, z, dev, "f0_surface_probes", "f0_surface_sdf"), "frame 0: surface")
    print("frame, |t - runs' mean| m, limit, angle deg, limit, |dt| m vs truth (ours, runs' worst), "
          "(map, local, pool, new) ours / stored run")
    for r in report:
        print(*r)
    expect(_surface_check(nm, dec, z, dev, "surface_probes", "end_surface_sdf"), "end of run: surface")
    assert not failures, failures
    # pin_slam.py:366-367: merge + prune
    raises = np.asarray(z["env_merged_raises"], bool)
    assert raises.all() or not raises.any(), "the reference runs disagree on the merge"
    if raises.all():
        with pytest.raises(IndexError):
            nm.recreate_hash(None, None, False, False)
    else:
        nm.recreate_hash(None, None, False, False)
        merged = nm.count()
        nm.prune_map(cfg.max_prune_certainty)
        pruned = merged - nm.count()
        assert pruned == 0 or pruned > 100           # prune_map removes points only above 100 candidates
        env_merged, env_end = np.asarray(z["env_merged_map_count"]), np.asarray(z["env_end_map_count"])
        # the end-of-run map count bound, one frame further (the runs' merged sizes as a last frame)
        runs = np.concatenate([np.asarray(z["env_hist_map_count"]), env_merged[:, None]], 1)
        if (env_merged == env_end).all() and pruned > 0:
            # the reference runs pruned nothing (<= 100 candidates: its own cut-off), this run > 100:
            # the counts before the prune are the comparable ones
            ok, lim = count_check(merged, runs, COUNT_FLOORS["map_count"])
        else:
            ok, lim = count_check(nm.count(), runs, COUNT_FLOORS["map_count"])
        assert ok, f"merged map {merged} / {nm.count()} outside the reference runs' envelope {lim}"
