#!/usr/bin/env python3
"""The reference's own run-to-run envelope for the configs[0] SLAM replays (slam_seq,
slam_seq100).

The reference's CPU reductions (index_add_ / scatter sums, BLAS) change order with the number of
torch threads, and its frame loop is chaotic in that order: two legitimate runs of
pin_slam.py:96-257 on the same scans and the same draws end centimetres apart.  gen_golden.py's
gen_slam_sequence stores one 8-thread run plus its difference to a 1-thread run; this script runs
the SAME loop (gen_golden._slam_sequence_run: the reference's Tracker / Mapper / NeuralPoints /
DataSampler, draws replayed) at further thread counts, each in its own process, and folds every
run into the fixture as an envelope (keys env_*): per run and frame the pose, the map / local /
pool / new-sample counts, and the surface SDF after frame 0 and at the end.

Runs ONLY in the build container (imports /root/reference through gen_golden).

Usage:
  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_slam_envelope.py run slam_seq 4 [rep]
  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_slam_envelope.py combine slam_seq
  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_slam_envelope.py forced slam_seq 1
"""
import glob
import os
import sys
import time

import numpy as np

RUN_DIR = os.environ.get("PIN_ENV_DIR", "/tmp/slam_env")
DUMP = {int(v) for v in os.environ.get("DUMP", "").split(",") if v}   # run_forced: frames whose state is saved
CASES = {"slam_seq": dict(frames=30, scene="street"), "slam_seq100": dict(frames=100, scene="long")}
# per-run arrays kept in the envelope (everything else of a run must equal the stored run's)
PER_RUN = ("hist_pose", "hist_map_count", "hist_local_count", "hist_pool", "hist_new", "f0_surface_sdf",
           "end_surface_sdf", "end_map_count")
SAME = ("hist_valid", "hist_n_cloud", "hist_n_source", "hist_draws_after", "hist_iters", "scan_sha256")


def run(name, threads, rep=0):
    """One reference run of the fixture's loop at `threads` torch threads -> RUN_DIR."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import gen_golden as G
    c = CASES[name]
    t0 = time.time()
    rec = G._slam_sequence_run(f"{name}[{threads} threads]", c["frames"], 21, 2024, threads, c["scene"])
    os.makedirs(RUN_DIR, exist_ok=True)
    keep = {k: rec[k] for k in PER_RUN + SAME + ("merged_raises",) if k in rec}
    if "merged_map_count" in rec:
        keep["merged_map_count"] = rec["merged_map_count"]
    keep["torch_threads"] = np.int64(threads)
    keep["wall_s"] = np.float64(time.time() - t0)
    import torch
    keep["torch_version"] = np.asarray(torch.__version__)
    np.savez_compressed(os.path.join(RUN_DIR, f"{name}_t{threads}_r{rep}.npz"), **keep)
    print(name, threads, "threads done in", round(time.time() - t0, 1), "s", flush=True)


def run_forced(name, threads):
    """The reference's frame loop at `threads` torch threads with the tracking RESULT replaced by
    the stored run's pose of each frame (pose forcing; tools/slam_forced.py is the same on the
    drop-in classes): the map is then built from the stored trajectory, and the reference's own
    tracker, still run every frame from the stored run's guess, shows how far a second reference
    run lands from the stored pose on a map that differs only by its reduction order.  Writes
    RUN_DIR/<name>_forced_t<threads>.npz with the per-frame tracked poses."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import types
    import torch
    import gen_golden as G
    import dataset.slam_dataset as rds_mod
    import utils.data_sampler as rds
    z = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{name}.npz"), allow_pickle=False))
    c = CASES[name]
    frames = c["frames"]
    torch.set_num_threads(threads)
    rng = np.random.default_rng(21)
    scene, poses = G.sequence_scene(c["scene"], rng, frames)
    scans = [G.lidar_scan(T, scene, rng) for T in poses]
    cfg = G.slam_config()
    replay = G.ReplayDraws(2024)
    rt = G._ReplayTorch(replay)
    saved = (rds.torch, G.rmapper.torch)
    rds.torch = rt
    G.rmapper.torch = rt
    rds_mod.get_time = time.time
    tracked = []
    try:
        torch.manual_seed(42)
        geo_mlp = G.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1)
        npm = G.NeuralPoints(cfg)
        ds = types.SimpleNamespace(config=cfg, silence=True, dtype=cfg.dtype, device="cpu", gt_pose_provided=False,
                                   odom_poses=[], pgo_poses=None, gt_poses=None, travel_dist=[], processed_frame=0,
                                   lose_track=False, consecutive_lose_track_frame=0, last_pose_ref=np.eye(4),
                                   last_odom_tran=np.eye(4), cur_pose_ref=np.eye(4), stop_count=0, stop_status=False,
                                   cur_point_cloud_torch=None, cur_point_ts_torch=None, cur_sem_labels_torch=None,
                                   cur_source_points=None, cur_source_normals=None, cur_source_colors=None)
        preprocess = types.MethodType(rds_mod.SLAMDataset.preprocess_frame, ds)
        update_odom = types.MethodType(rds_mod.SLAMDataset.update_odom_pose, ds)
        tracker = G.rtracker.Tracker(cfg, npm, geo_mlp, None, None)
        mapper = G.rmapper.Mapper(cfg, ds, npm, geo_mlp, None, None)
        for frame_id in range(frames):
            used = ds.processed_frame
            ds.cur_pose_ref = np.eye(4)
            ds.cur_pose_torch = torch.tensor(ds.cur_pose_ref, dtype=cfg.dtype)
            ds.cur_point_cloud_torch = torch.from_numpy(scans[frame_id].astype(np.float32) / np.float32(G.Q_SCALE))
            ds.cur_point_ts_torch = None
            preprocess(frame_id)
            if used > 0:
                if frame_id in DUMP:   # the state this tracking call sees (tools/ref_track_dump.py --compare)
                    torch.save({"npm": npm, "dec": geo_mlp.state_dict(), "source": ds.cur_source_points,
                                "guess": ds.cur_pose_guess_torch},
                               os.path.join(RUN_DIR, f"refdump_{name}_f{frame_id}_t{threads}.pt"))
                T, _, _, valid = tracker.tracking(ds.cur_source_points, ds.cur_pose_guess_torch, None, None,
                                                  vis_result=False)
                tracked.append(np.asarray(T, dtype=np.float64))
                ds.lose_track = False
                mapper.lose_track = False
                update_odom(torch.tensor(z["hist_pose"][frame_id], dtype=torch.float64))
            else:
                tracked.append(np.eye(4))
            npm.travel_dist = torch.tensor(np.array(ds.travel_dist), dtype=cfg.dtype)
            if not mapper.lose_track and not ds.stop_status:
                mapper.process_frame(ds.cur_point_cloud_torch, ds.cur_sem_labels_torch, ds.cur_pose_torch, used, False)
            else:
                npm.reset_local_map(ds.cur_pose_torch[:3, 3], None, used)
            iters = cfg.iters * cfg.init_iter_ratio if used == 0 else cfg.iters
            if used == cfg.freeze_after_frame:
                G.rtools.freeze_decoders(geo_mlp, None, None, cfg)
            if used % cfg.mapping_freq_frame == 0:
                mapper.mapping(iters)
            ds.processed_frame += 1
            ref = z["hist_pose"][frame_id]
            d = ref[:3, :3].T @ (tracked[-1][:3, 3] - ref[:3, 3])
            print(f"{name} forced [{threads} threads] frame {frame_id}: tracked - stored (body frame) "
                  f"{np.round(d, 4)}", flush=True)
    finally:
        rds.torch, G.rmapper.torch = saved
    os.makedirs(RUN_DIR, exist_ok=True)
    np.savez_compressed(os.path.join(RUN_DIR, f"{name}_forced_t{threads}.npz"), tracked=np.stack(tracked),
                        stored=z["hist_pose"][:frames], torch_threads=np.int64(threads))
    D = np.stack([p[:3, :3].T @ (t[:3, 3] - p[:3, 3]) for t, p in zip(tracked[1:], z["hist_pose"][1:frames])])
    print(name, "forced", threads, "threads: body-frame tracked - stored mean", np.round(D.mean(0), 4), "std",
          np.round(D.std(0), 4), "t", np.round(D.mean(0) / (D.std(0) / np.sqrt(len(D)) + 1e-12), 2))


TRACE_STEPS = (1, 2, 3, 5, 10, 20, 50, 100, 200, 400, 600)


def run_f0_trace(name, threads):
    """Frame 0 of the fixture's loop (update, process_frame, the 15 x 40-iteration mapping() call)
    at `threads` torch threads, recording the decoder and the feature statistics after the Adam
    steps in TRACE_STEPS: where the reference's own runs part ways, and where ours (the same
    record from tools/slam_forced.py) parts from them."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import types
    import torch
    import gen_golden as G
    import dataset.slam_dataset as rds_mod
    import utils.data_sampler as rds
    c = CASES[name]
    torch.set_num_threads(threads)
    rng = np.random.default_rng(21)
    scene, poses = G.sequence_scene(c["scene"], rng, c["frames"])
    scan0 = G.lidar_scan(poses[0], scene, rng)
    cfg = G.slam_config()
    replay = G.ReplayDraws(2024)
    rt = G._ReplayTorch(replay)
    saved = (rds.torch, G.rmapper.torch, G.rmapper.setup_optimizer)
    rds.torch = rt
    G.rmapper.torch = rt
    rds_mod.get_time = time.time
    rec = {}
    saved_np_torch = G.rnp.torch
    if os.environ.get("TIE_PROBE"):   # experiment: rows whose top-k set depends on the sort's tie order
        class _Probe:
            count = [0, 0]

            def __getattr__(self, k):
                return getattr(torch, k)

            def sort(self, x, dim=-1, descending=False):
                out = torch.sort(x, dim=dim, descending=descending)
                st = torch.sort(x, dim=dim, descending=descending, stable=True)
                k = cfg.query_nn_k
                big = torch.tensor(1 << 40)
                gidx = self.last_idx                 # the radius search's candidates, local ids
                lidx = npm.global2local[gidx] if gidx is not None else None
                # the valid candidates' local ids among the k first, compared as sets
                va = torch.where(out[0][:, :k] < 9e3, lidx.gather(1, out[1][:, :k]), big)
                vb = torch.where(st[0][:, :k] < 9e3, lidx.gather(1, st[1][:, :k]), big)
                a = torch.sort(va, 1)[0]
                b = torch.sort(vb, 1)[0]
                bad = (a != b).any(1)
                first = self.count[0] == 0
                self.count[0] += int(bad.sum())
                self.count[1] += x.shape[0]
                if bad.any() and first:
                    r = int(torch.nonzero(bad)[0])
                    print("tie row:", np.round(x[r].numpy(), 7).tolist(), "unstable", out[1][r, :k].tolist(),
                          "stable", st[1][r, :k].tolist(), "global ids", gidx[r].tolist(), "local ids",
                          lidx[r].tolist(), flush=True)
                return out
        probe = _Probe()
        probe.last_idx = None
        G.rnp.torch = probe
        orig_rns = G.NeuralPoints.radius_neighborhood_search

        def rns(self_, points, time_filtering=False):
            d2, idx = orig_rns(self_, points, time_filtering)
            probe.last_idx = idx.clone()
            return d2, idx
        G.NeuralPoints.radius_neighborhood_search = rns
    if os.environ.get("STABLE_SORT"):   # experiment: the reference with a stable k-NN sort
        class _StableSort:
            def __getattr__(self, k):
                return getattr(torch, k)

            @staticmethod
            def sort(x, dim=-1, descending=False):
                return torch.sort(x, dim=dim, descending=descending, stable=True)
        G.rnp.torch = _StableSort()
    try:
        torch.manual_seed(42)
        geo_mlp = G.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1)
        npm = G.NeuralPoints(cfg)
        ds = types.SimpleNamespace(config=cfg, silence=True, dtype=cfg.dtype, device="cpu", gt_pose_provided=False,
                                   odom_poses=[], pgo_poses=None, gt_poses=None, travel_dist=[], processed_frame=0,
                                   lose_track=False, consecutive_lose_track_frame=0, last_pose_ref=np.eye(4),
                                   last_odom_tran=np.eye(4), cur_pose_ref=np.eye(4), stop_count=0, stop_status=False,
                                   cur_point_cloud_torch=None, cur_point_ts_torch=None, cur_sem_labels_torch=None,
                                   cur_source_points=None, cur_source_normals=None, cur_source_colors=None)
        preprocess = types.MethodType(rds_mod.SLAMDataset.preprocess_frame, ds)
        mapper = G.rmapper.Mapper(cfg, ds, npm, geo_mlp, None, None)

        def setup(*a, **kw):
            opt = saved[2](*a, **kw)
            step = opt.step
            count = [0]

            def rec_step(*sa, **skw):
                out = step(*sa, **skw)
                count[0] += 1
                if count[0] in TRACE_STEPS:
                    for k, p in zip(("W1", "b1", "W2", "b2"), geo_mlp.parameters()):
                        rec[f"s{count[0]}_{k}"] = p.detach().numpy().copy()
                    rec[f"s{count[0]}_feat"] = npm.local_geo_features.detach().numpy().copy()
                return out
            opt.step = rec_step
            return opt
        G.rmapper.setup_optimizer = setup
        ds.cur_pose_ref = np.eye(4)
        ds.cur_pose_torch = torch.tensor(ds.cur_pose_ref, dtype=cfg.dtype)
        ds.cur_point_cloud_torch = torch.from_numpy(scan0.astype(np.float32) / np.float32(G.Q_SCALE))
        ds.cur_point_ts_torch = None
        preprocess(0)
        npm.travel_dist = torch.tensor(np.array(ds.travel_dist), dtype=cfg.dtype)
        mapper.process_frame(ds.cur_point_cloud_torch, ds.cur_sem_labels_torch, ds.cur_pose_torch, 0, False)
        mapper.mapping(cfg.iters * cfg.init_iter_ratio)
    finally:
        rds.torch, G.rmapper.torch, G.rmapper.setup_optimizer = saved
        G.rnp.torch = saved_np_torch
    os.makedirs(RUN_DIR, exist_ok=True)
    tag = "_stable" if os.environ.get("STABLE_SORT") else ""
    if os.environ.get("TIE_PROBE"):
        print("rows whose top-k set depends on the tie order:", probe.count[0], "of", probe.count[1], flush=True)
        return
    np.savez_compressed(os.path.join(RUN_DIR, f"{name}_f0trace{tag}_t{threads}.npz"), **rec)
    print(name, "frame-0 trace", threads, "threads:",
          [(s, round(float(rec[f"s{s}_b2"][0]), 5)) for s in TRACE_STEPS if f"s{s}_b2" in rec])


def combine(name):
    """Fold the stored run and every RUN_DIR run of `name` into tests/golden/<name>.npz."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{name}.npz")
    z = dict(np.load(path, allow_pickle=False))
    runs = [dict(np.load(p, allow_pickle=False)) for p in sorted(glob.glob(os.path.join(RUN_DIR, f"{name}_t*_r*.npz")))]
    for r in runs:
        for k in SAME:
            if k in r:
                assert np.array_equal(r[k], z[k]), f"{name}: run at {int(r['torch_threads'])} threads differs in {k}"
    labels = ["stored (%d threads)" % int(z["torch_threads"])] + \
        ["%d threads" % int(r["torch_threads"]) for r in runs]
    for k in PER_RUN:
        z["env_" + k] = np.stack([z[k]] + [r[k] for r in runs])
    z["env_merged_map_count"] = np.asarray([int(z.get("merged_map_count", -1))] +
                                           [int(r.get("merged_map_count", -1)) for r in runs], np.int64)
    z["env_merged_raises"] = np.asarray([bool(z["merged_raises"])] + [bool(r["merged_raises"]) for r in runs])
    z["env_threads"] = np.asarray([int(z["torch_threads"])] + [int(r["torch_threads"]) for r in runs], np.int64)
    z["env_labels"] = np.asarray(labels)
    z["env_torch"] = np.asarray([str(r["torch_version"]) for r in runs])
    z["env_generated"] = np.asarray(time.strftime("%Y-%m-%d"))
    np.savez_compressed(path, **z)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import build_manifest
    build_manifest.update(name, envelope_runs=labels, envelope_generated=str(z["env_generated"]),
                          envelope_torch=sorted(set(str(v) for v in z["env_torch"])))
    P = z["env_hist_pose"]
    dt = np.linalg.norm(P[:, :, :3, 3] - P[:1, :, :3, 3], axis=-1)
    m = np.abs(z["env_end_surface_sdf"]).mean(axis=1)
    print(name, len(labels), "runs:", labels)
    print("  largest pose offset from the stored run per run (m):", np.round(dt.max(axis=1), 4))
    print("  end mean |SDF| per run (m):", np.round(m, 4))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 0)
    elif sys.argv[1] == "forced":
        run_forced(sys.argv[2], int(sys.argv[3]))
    elif sys.argv[1] == "f0trace":
        run_f0_trace(sys.argv[2], int(sys.argv[3]))
    else:
        combine(sys.argv[2])
