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
"""
import glob
import os
import sys
import time

import numpy as np

RUN_DIR = os.environ.get("PIN_ENV_DIR", "/tmp/slam_env")
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
    P = z["env_hist_pose"]
    dt = np.linalg.norm(P[:, :, :3, 3] - P[:1, :, :3, 3], axis=-1)
    m = np.abs(z["env_end_surface_sdf"]).mean(axis=1)
    print(name, len(labels), "runs:", labels)
    print("  largest pose offset from the stored run per run (m):", np.round(dt.max(axis=1), 4))
    print("  end mean |SDF| per run (m):", np.round(m, 4))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 0)
    else:
        combine(sys.argv[2])
