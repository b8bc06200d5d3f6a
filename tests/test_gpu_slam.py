"""BASELINE configs[0], the plumbing run: the reference's pin_slam.py frame loop (:96-257) over a
30-frame synthetic 64-beam street sequence (64K points per scan; three window filters of the
sample pool, frames 9, 19, 29, and the decoder frozen after frame 15), replayed through
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

Tolerances, checked per frame:
  * preprocessed cloud / source point counts, tracking validity, draw-stream position: exact;
  * pose within max(5 cm, 3 x spread) and max(0.1 deg, 3 x spread) of the reference's estimate
    (spread: the largest 1- vs 8-thread difference of the reference up to that frame),
    and within max(5 cm, the reference's own error + that tolerance) of the ground truth;
  * neural-point / local-map counts within max(1 %, 3 x spread), pool size within 0.1 %, new
    samples within max(15 %, 3 x spread) (they follow the certainty threshold);
  * the map's SDF on the surface (scan points placed by the TRUE poses) after frame 0 and at the
    end: mean |SDF| at most 1.25 x the reference's + 1 mm after frame 0, 1.5 x after the 30 frames
    (the drifted runs' own range), and median |ours - reference| at most 3 x the median 1- vs
    8-thread spread + 1 mm;
  * the end-of-run merge (recreate_hash(kept_points=False), pin_slam.py:366) raises where the
    reference's does, and otherwise leaves a map of the same size within 1 %.
"""
import json
import math

import numpy as np
import pytest
import torch

import pin_slam_amd as P
from pin_slam_amd.synthetic import FrameLoop, lidar_scan, slam_poses, street_scene
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


def _surface_check(nm, dec, z, dev, probes_key, sdf_key, ratio=1.25, slack=0.0):
    """The map's SDF at surface points against the reference's (see the module docstring).
    slack: metres added to the mean-|SDF| bound (the end-of-run check: drift beyond the reference's)."""
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
    assert mine <= ratio * ref + 1e-3 + slack, (mine, ref, slack)
    assert diff <= 3 * spread + 1e-3, (diff, spread)


def test_slam_sequence_matches_reference(golden, dev):
    z = golden("slam_seq")
    conf = json.loads(str(z["config_json"]))
    cfg = P.Config(**conf)
    cfg.device = dev
    frames = int(z["frames"])
    nm = P.NeuralPoints(cfg)
    dec = P.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1)
    with torch.no_grad():
        dec.layers[0].weight.copy_(torch.as_tensor(z["dec_init_W1"]))
        dec.layers[0].bias.copy_(torch.as_tensor(z["dec_init_b1"]))
        dec.lout.weight.copy_(torch.as_tensor(z["dec_init_W2"]))
        dec.lout.bias.copy_(torch.as_tensor(z["dec_init_b2"]))
    dec.to(dev)
    tracker = P.Tracker(cfg, nm, dec)
    mapper = P.Mapper(cfg, None, nm, dec)
    loop = FrameLoop(cfg, nm, dec, tracker, mapper)     # pin_slam.py:96-257 on the drop-in classes
    replay = ReplayDraws(int(z["replay_seed"]))
    mapper._randint = lambda high, n: torch.from_numpy(replay.randint(high, n)).to(dev)
    S, Ff, Fb = int(cfg.surface_sample_n), int(cfg.free_front_n), int(cfg.free_behind_n)

    def draws(n):
        return (torch.from_numpy(replay.randn(n * S)), torch.from_numpy(replay.rand(n * Ff)),
                torch.from_numpy(replay.rand(n * Fb)))
    # the scans, regenerated as the generator made them (same seed and call order), checked
    # against the fixture's digests
    import hashlib
    rng = np.random.default_rng(int(z["scan_seed"]))
    scene = street_scene(rng)
    scans = [lidar_scan(T, scene, rng) for T in slam_poses(frames)]
    for k, sc in enumerate(scans):
        assert hashlib.sha256(np.ascontiguousarray(sc).tobytes()).hexdigest() == str(z["scan_sha256"][k]), \
            f"frame {k}: regenerated scan differs from the reference run's"
    report = []
    for k in range(frames):
        pts = torch.from_numpy(scans[k].astype(np.float32) / np.float32(z["q_scale"])).to(dev)
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
        valid = loop.frame(pts, draws=draws, timer=check)
        assert bool(valid) == bool(z["hist_valid"][k]), f"frame {k}: tracking validity"
        assert replay.calls == int(z["hist_draws_after"][k]), f"frame {k}: draw stream out of step"
        counts = seen["counts"]
        want = tuple(int(z[f"hist_{n_}"][k]) for n_ in ("map_count", "local_count", "pool", "new"))
        dt, dr = _pose_err(loop.cur_pose_ref, z["hist_pose"][k])
        dt_true, _ = _pose_err(loop.cur_pose_ref, z["truth_poses"][k])
        report.append((k, round(dt, 4), round(dr, 4), round(dt_true, 4), counts, want))
        print("frame", *report[-1], flush=True)
        # the reference's own 1- vs 8-thread runs differ by up to 3.3 cm by frame 13 and re-converge
        # and diverge again afterwards: the spread up to frame k bounds how far two legitimate runs
        # may be apart at frame k
        tol_t = max(0.05, 3 * float(np.max(z["spread_pose_dt"][:k + 1])))
        tol_r = max(0.1, 3 * float(np.max(z["spread_pose_dr"][:k + 1])))
        assert dt <= tol_t and dr <= tol_r, f"frame {k}: pose differs from the reference by {dt:.4f} m / {dr:.4f} deg"
        # the reference itself drifts from the truth over the 30 frames (6-7 cm by frame 29)
        ref_true, _ = _pose_err(z["hist_pose"][k], z["truth_poses"][k])
        assert dt_true <= max(0.05, ref_true + tol_t), f"frame {k}: pose {dt_true:.4f} m from the ground truth"
        filt = k % int(cfg.pool_filter_freq) == int(cfg.pool_filter_freq) - 1   # the pool's window filter ran
        for name, g, w, rel in zip(("map_count", "local_count", "pool", "new"), counts, want, (0.01, 0.01, 0.001, 0.15)):
            rel = max(rel, 3 * float(z[f"spread_rel_{name}"][k]))
            if name == "pool" and filt:
                # the filter drops every sample beyond the window radius of the CURRENT position: the
                # samples near that sphere move in or out with the pose, ~0.025 % of the pool per cm at
                # frame 29 (the dense early frames lie on the sphere); 0.05 % per cm of pose difference
                rel = max(rel, 0.0005 * 100.0 * dt)
            if name in ("map_count", "local_count"):
                # a frame registered a few cm apart inserts its points into partly other voxels: the
                # counts drift with the pose difference (measured 0.2-0.22 % per cm over frames
                # 25-29 of a run 3-4.6 cm apart); 0.3 % per cm of pose difference
                rel = max(rel, 0.003 * 100.0 * dt)
            assert _within(g, w, rel), f"frame {k}: {name} {g} vs reference {w}"
        if k == 0:
            _surface_check(nm, dec, z, dev, "f0_surface_probes", "f0_surface_sdf")
    print("frame, |dt| m, |dR| deg vs reference, |dt| m vs truth, (map, local, pool, new) ours / reference")
    for r in report:
        print(*r)
    # the map at the end of the loop
    # after 30 frames the runs have drifted apart (ours 5-10 cm from the truth at frame 29 over five
    # runs, the reference's two runs 6.8 / 7.3 cm), and the probes sit at the TRUE poses: mean |SDF|
    # measured 0.023-0.037 m over five runs of ours against the reference's 0.027 / 0.028 m
    # a run that drifted further from the truth than the reference did sees its surface shifted
    # against the probes by part of the excess (measured: 0.0445 m at 11.4 cm vs the reference's
    # 7 cm of drift at frame 29); a quarter of the excess drift is allowed on top
    dt_last, _ = _pose_err(loop.cur_pose_ref, z["truth_poses"][frames - 1])
    ref_last, _ = _pose_err(z["hist_pose"][frames - 1], z["truth_poses"][frames - 1])
    _surface_check(nm, dec, z, dev, "surface_probes", "end_surface_sdf", ratio=1.5,
                   slack=0.25 * max(0.0, dt_last - ref_last))
    # pin_slam.py:366-367: merge + prune
    if bool(z["merged_raises"]):
        with pytest.raises(IndexError):
            nm.recreate_hash(None, None, False, False)
    else:
        nm.recreate_hash(None, None, False, False)
        nm.prune_map(cfg.max_prune_certainty)
        assert _within(nm.count(), int(z["merged_map_count"]), 0.01)
