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
summation order.  The loop is chaotic in that difference: the reference run twice, with 1 and with
8 torch threads (only its reduction order changes), ends frame 0's 15 x 40-iteration mapping()
with different decoders (|dW1| up to 1.7) and features, yet poses within ~2 cm / 0.03 deg and
the same surface.  That spread is stored in the fixture (spread_*) and the tolerances below are
stated against it -- element-wise feature parity after hundreds of iterations is not a property
the reference has.  (A single 15-iteration mapping() call is pinned element-wise in
tests/test_gpu_mapper.py::test_whole_mapping_call_fixture.)

Our side runs the deterministic training mode (Mapper(deterministic=True): fixed-point gradient
and certainty sums, stable tile order), so this test judges ONE reproducible trajectory -- two
runs are bitwise equal -- against bounds fixed before it was run:
  * preprocessed cloud / source point counts, tracking validity, draw-stream position: exact;
  * pose within max(5 cm, 3 x spread) and max(0.1 deg, 3 x spread) of the reference's estimate
    (spread: the largest 1- vs 8-thread difference of the reference up to that frame); the
    distance to the ground truth is reported (bounded by the reference's own error + that
    tolerance, which the pose bound implies);
  * neural-point / local-map counts within max(1 %, 3 x spread), pool size within
    max(0.1 %, 3 x spread), new samples within max(15 %, 3 x spread), the spread being the
    largest relative 1- vs 8-thread count difference up to that frame (they follow the certainty
    threshold); at the window-filter frames the pool count may differ by the difference carried in
    plus the samples whose side of the filter sphere the pose differences can change (counted on
    our pre-filter pool: displacement |dt_j| + theta_j * range per sample, |dt_k| for the centre);
  * the map's SDF on the surface (scan points placed by the TRUE poses) after frame 0 and at the
    end: mean |SDF| at most 1.25 x the reference's + 1 mm, and median |ours - reference| at most
    3 x the median 1- vs 8-thread spread + 1 mm;
  * the end-of-run merge (recreate_hash(kept_points=False), pin_slam.py:366) raises where the
    reference's does, and otherwise leaves a map of the same size within 1 %.
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


def _within(got, want, rel):
    return abs(int(got) - int(want)) <= max(1, rel * abs(int(want)))


def _surface_check(nm, dec, z, dev, probes_key, sdf_key, ratio=1.25):
    """The map's SDF at surface points against the reference's (see the module docstring);
    returns whether both bounds hold."""
    probes = torch.from_numpy(z[probes_key]).to(dev)
    sdf, _, _, _, _ = P.query_sdf(nm, dec, probes, query_locally=False, want_grad=False, want_certainty=False)
    got = sdf.cpu().numpy()
    want = z[sdf_key]
    mine, ref = float(np.abs(got).mean()), float(np.abs(want).mean())
    diff = float(np.median(np.abs(got - want)))
    spread = float(np.median(z["spread_abs_" + sdf_key]))
    print(f"{sdf_key}: mean |SDF| ours {mine:.4f} m, reference {ref:.4f} m (1 thread "
          f"{float(z['t1_mean_abs_' + sdf_key]):.4f}); median |ours - reference| {diff:.4f} m, reference spread "
          f"{spread:.4f} m")
    return mine <= ratio * ref + 1e-3 and diff <= 3 * spread + 1e-3


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


@pytest.mark.parametrize("fixture", ["slam_seq", "slam_seq100"])
def test_slam_sequence_matches_reference(golden, dev, fixture):
    """slam_seq: 30 frames of the accelerating street; slam_seq100: BASELINE configs[0]'s 100
    frames on the long street (synthetic.sequence_scene("long"); window filters at frames 9..99,
    the pool's capacity discards at frame 99)."""
    z = golden(fixture)
    frames = int(z["frames"])
    nm, dec, mapper, loop, replay, draws, scans = _sequence(z, dev, frames)
    cfg = nm.config
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
        dt, dr = _pose_err(loop.cur_pose_ref, z["hist_pose"][k])
        dt_true, _ = _pose_err(loop.cur_pose_ref, z["truth_poses"][k])
        ref_true, _ = _pose_err(z["hist_pose"][k], z["truth_poses"][k])
        our_poses.append(np.array(loop.cur_pose_ref, dtype=np.float64))
        report.append((k, round(dt, 4), round(dr, 4), round(dt_true, 4), round(ref_true, 4), counts, want))
        print("frame", *report[-1], flush=True)
        # the reference's own 1- vs 8-thread runs differ by up to 3.3 cm by frame 13 and re-converge
        # and diverge again afterwards: the spread up to frame k bounds how far two legitimate runs
        # may be apart at frame k
        tol_t = max(0.05, 3 * float(np.max(z["spread_pose_dt"][:k + 1])))
        tol_r = max(0.1, 3 * float(np.max(z["spread_pose_dr"][:k + 1])))
        expect(dt <= tol_t and dr <= tol_r, f"frame {k}: pose differs from the reference by {dt:.4f} m / {dr:.4f} deg")
        # the reference itself drifts from the truth over the 30 frames (6-7 cm by frame 29); with
        # the pose bound above this is implied (triangle inequality), checked for the report
        expect(dt_true <= max(0.05, ref_true + tol_t), f"frame {k}: pose {dt_true:.4f} m from the ground truth")
        filt = k % int(cfg.pool_filter_freq) == int(cfg.pool_filter_freq) - 1   # the pool's window filter ran
        for name, g, w, rel in zip(("map_count", "local_count", "pool", "new"), counts, want, (0.01, 0.01, 0.001, 0.15)):
            # the spread up to frame k, as for the pose (a count difference persists: points
            # inserted differently stay in the map)
            rel = max(rel, 3 * float(np.max(z[f"spread_rel_{name}"][:k + 1])))
            if name == "pool" and filt:
                # the filter keeps the samples within window_radius of the CURRENT position: beyond
                # the difference carried in from the previous frame, the count can differ only by
                # samples that lie, in our pool, within their displacement bound of the sphere
                prev = report[-2][5][2] - report[-2][6][2] if k > 0 else 0
                lim = abs(prev) + _shell_count(pre, our_poses, z["hist_pose"], k, float(cfg.window_radius))
                print(f"frame {k}: pool {g} vs {w}: |diff| {abs(g - w)}, geometric bound {lim}", flush=True)
                expect(abs(g - w) <= max(lim, rel * w), f"frame {k}: pool {g} vs reference {w} (bound {lim})")
                continue
            expect(_within(g, w, rel), f"frame {k}: {name} {g} vs reference {w} (rel {rel:.4f})")
        if k == 0:
            expect(_surface_check(nm, dec, z, dev, "f0_surface_probes", "f0_surface_sdf"), "frame 0: surface")
    print("frame, |dt| m, |dR| deg vs reference, |dt| m vs truth (ours, reference), (map, local, pool, new) ours / "
          "reference")
    for r in report:
        print(*r)
    # the map at the end of the loop: mean |SDF| at the probes (placed by the TRUE poses) at most
    # 1.25 x the reference's + 1 mm
    expect(_surface_check(nm, dec, z, dev, "surface_probes", "end_surface_sdf"), "end of run: surface")
    assert not failures, failures
    # pin_slam.py:366-367: merge + prune
    if bool(z["merged_raises"]):
        with pytest.raises(IndexError):
            nm.recreate_hash(None, None, False, False)
    else:
        nm.recreate_hash(None, None, False, False)
        merged = nm.count()
        nm.prune_map(cfg.max_prune_certainty)
        pruned = merged - nm.count()
        assert pruned == 0 or pruned > 100           # prune_map removes points only above 100 candidates
        # the map-count bound of the last frame (max(1 %, 3 x the running count spread))
        rel = max(0.01, 3 * float(np.max(z["spread_rel_map_count"])))
        if int(z["merged_map_count"]) == int(z["end_map_count"]) and pruned > 0:
            # the reference pruned nothing (<= 100 candidates: its own cut-off), this run > 100: the
            # counts before the prune are the comparable ones
            assert _within(merged, int(z["merged_map_count"]), rel)
        else:
            assert _within(nm.count(), int(z["merged_map_count"]), rel)
