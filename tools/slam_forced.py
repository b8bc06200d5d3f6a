#!/usr/bin/env python3
"""Diagnostic for the configs[0] replay (tests/test_gpu_slam.py): where does our trajectory leave
the reference's?  Runs the fixture's frame loop on the drop-in classes with the TRACKING RESULT
REPLACED by the reference's own pose of each frame (pose forcing): the map, pools and decoder are
then built from the reference's trajectory, so

  * the map's end-of-run surface SDF against the reference's isolates process_frame + mapping
    (an unbiased map side lands inside the reference runs' envelope), and
  * our tracker, still run every frame from the same guess the reference used, gives per frame
    the pose it would have returned: its distance to the reference's pose isolates tracking.

Usage: python tools/slam_forced.py [slam_seq|slam_seq100] [det 0|1] [frames]
"""
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.test_gpu_slam import _pose_err, _sequence  # noqa: E402
import pin_slam_amd as P  # noqa: E402


DUMP = {int(v) for v in __import__("os").environ.get("DUMP", "").split(",") if v}


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "slam_seq"
    det = (sys.argv[2] if len(sys.argv) > 2 else "1") == "1"
    z = dict(np.load(f"tests/golden/{name}.npz", allow_pickle=False))
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else int(z["frames"])
    nm, dec, mapper, loop, replay, draws, scans = _sequence(z, "cuda", frames)
    mapper.deterministic = det
    ref = z["hist_pose"]
    tracker = loop.tracker
    c = loop.config
    rows = []
    for k in range(frames):
        used = loop.processed_frame
        loop.read_and_preprocess(scans[k])
        if used > 0:
            hist = []
            tracker._iteration_done = lambda i, dT, st: hist.append(np.asarray(dT.cpu() if torch.is_tensor(dT) else dT))
            if k in DUMP:   # the state this tracking call sees, for tools/ref_track_dump.py
                import os
                from pin_slam_amd.mapio import save_implicit_map
                d = f"gpurun_out/dump/{name}_f{k}"
                os.makedirs(d, exist_ok=True)
                path = save_implicit_map(d, nm, dec, tensor_device="cpu")
                import gzip
                import shutil
                with open(path, "rb") as fi, gzip.open(path + ".gz", "wb", compresslevel=1) as fo:
                    shutil.copyfileobj(fi, fo)   # the 5e7-slot table is mostly -1: a few MB compressed
                os.remove(path)
            T, _, _, valid = tracker.tracking(loop.cur_source_points, loop.cur_pose_guess_torch, None, None)
            ours = T.detach().cpu().numpy()
            if k in DUMP:
                np.savez(f"{d}/track.npz", source=loop.cur_source_points.cpu().numpy(),
                         guess=loop.cur_pose_guess_torch.cpu().numpy(), ours=ours, ref=ref[k],
                         iterations=int(tracker.last_iterations), deltas=np.stack(hist), valid=bool(valid))
            dt, dr = _pose_err(ours, ref[k])
            g_dt, g_dr = _pose_err(loop.cur_pose_guess_torch.cpu().numpy(), ref[k])
            # the difference in the reference pose's body frame (x: along the street)
            dvec = ref[k][:3, :3].T @ (ours[:3, 3] - ref[k][:3, 3])
            rows.append((k, dt, dr, g_dt, g_dr, dvec))
            loop.lose_track = False
            mapper.lose_track = False
            loop.update_odom_pose(torch.tensor(ref[k], dtype=torch.float64, device="cuda"))
        loop.nm.travel_dist = torch.tensor(np.array(loop.travel_dist), dtype=torch.float32, device="cuda")
        if not mapper.lose_track and not loop.stop_status:
            d = draws(loop.cur_point_cloud_torch.shape[0])
            mapper.process_frame(loop.cur_point_cloud_torch, None, loop.cur_pose_torch, used, False, draws=d)
        else:
            nm.reset_local_map(loop.cur_pose_torch[:3, 3], None, used)
        iters = c.iters * c.init_iter_ratio if used == 0 else c.iters
        if used == c.freeze_after_frame:
            for p in dec.parameters():
                p.requires_grad_(False)
        if used % c.mapping_freq_frame == 0:
            mapper.mapping(iters)
        loop.processed_frame += 1
        counts = (nm.count(), nm.local_count(), int(mapper.pool_sample_count), int(mapper.new_idx.shape[0]))
        if k in (0, 3) and __import__("os").environ.get("DECSTATS"):
            W1, b1, W2, b2 = (p.detach().double() for p in dec.parameters())
            print(f"decoder after frame {k}: b2 {float(b2):.5f} mean b1 {float(b1.mean()):.4f} mean W2 "
                  f"{float(W2.mean()):.4f} mean |W1| {float(W1.abs().mean()):.4f} feature mean "
                  f"{float(nm.local_geo_features.detach().double().mean()):.5f}", flush=True)
        want = tuple(int(z[f"hist_{n}"][k]) for n in ("map_count", "local_count", "pool", "new"))
        print(f"frame {k}: counts {counts} ref {want}" + (
            f"  tracking from the reference's guess: {rows[-1][1]:.4f} m / {rows[-1][2]:.4f} deg off the reference "
            f"(guess was {rows[-1][3]:.4f} m / {rows[-1][4]:.4f} deg)" if used > 0 else ""), flush=True)
    probes = torch.from_numpy(z["surface_probes"]).cuda()
    sdf, _, _, _, _ = P.query_sdf(nm, dec, probes, query_locally=False, want_grad=False, want_certainty=False)
    got = sdf.cpu().numpy()
    env = z.get("env_end_surface_sdf")
    refs = np.abs(env).mean(1) if env is not None else [np.abs(z["end_surface_sdf"]).mean()]
    print(f"end mean |SDF| ours (pose-forced) {np.abs(got).mean():.4f} m; reference runs {np.round(refs, 4)}; "
          f"median |ours - stored| {np.median(np.abs(got - z['end_surface_sdf'])):.4f} m")
    a = np.array([r[1] for r in rows])
    print(f"tracking vs reference pose: mean {a.mean():.4f} m, max {a.max():.4f} m at frame {rows[int(a.argmax())][0]}; "
          f"mean rot {np.mean([r[2] for r in rows]):.4f} deg")
    D = np.stack([r[5] for r in rows])
    print("body-frame difference ours - reference (x along the street): mean", np.round(D.mean(0), 4),
          "std", np.round(D.std(0), 4), "n", len(D), "t", np.round(D.mean(0) / (D.std(0) / math.sqrt(len(D)) + 1e-12), 2))


if __name__ == "__main__":
    main()
