#!/usr/bin/env python3
"""Our own run-to-run scatter on a configs[0] replay: the fixture's frame loop run R times in one
training mode, each run's pose checked against the reference runs' envelope exactly as
tests/test_gpu_slam.py does (pose_check).  Prints per run the largest ratio of the position /
angle deviation to its limit and the frame, and per frame the spread of our runs.

Usage: python tools/slam_runs.py [slam_seq|slam_seq100] [det 0|1] [runs]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import pin_slam_amd as P  # noqa: E402
from tests import test_gpu_slam as S  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "slam_seq"
    det = (sys.argv[2] if len(sys.argv) > 2 else "0") == "1"
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    z = dict(np.load(f"tests/golden/{name}.npz", allow_pickle=False))
    frames = int(z["frames"])
    penv = S.pose_envelope(z)
    allp = []
    for r in range(R):
        nm, dec, mapper, loop, replay, draws, scans = S._sequence(z, "cuda", frames)
        mapper.deterministic = det
        worst_t, worst_r, poses = (0.0, -1), (0.0, -1), []
        for k in range(frames):
            loop.frame(scans[k], draws=draws, next_pts=scans[k + 1] if k + 1 < frames else None)
            T = np.asarray(loop.cur_pose_ref, dtype=np.float64)
            poses.append(T)
            _, d, tt, a, tr = S.pose_check(T, k, penv)
            worst_t = max(worst_t, (d / tt, k))
            worst_r = max(worst_r, (a / tr, k))
        allp.append(np.stack(poses))
        probes = torch.from_numpy(z["surface_probes"]).cuda()
        sdf, _, _, _, _ = P.query_sdf(nm, dec, probes, query_locally=False, want_grad=False, want_certainty=False)
        ok, msg = S.surface_bounds(sdf.cpu().numpy(), z["env_end_surface_sdf"])
        dtrue = np.linalg.norm(poses[-1][:3, 3] - z["truth_poses"][frames - 1][:3, 3])
        print(f"run {r}: worst position / limit {worst_t[0]:.3f} at frame {worst_t[1]}, worst angle / limit "
              f"{worst_r[0]:.3f} at frame {worst_r[1]}; last pose {dtrue:.4f} m from the truth; end surface "
              f"{'ok' if ok else 'OUT'}: {msg}", flush=True)
    Q = np.stack(allp)
    import os
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez(f"gpurun_out/slam_runs_{name}_det{int(det)}.npz", poses=Q)
    c = Q[:, :, :3, 3].mean(0)
    print("our runs' largest distance from their mean per frame (m):",
          np.round(np.linalg.norm(Q[:, :, :3, 3] - c[None], axis=-1).max(0), 4).tolist())
    print("our runs' largest angle from their mean per frame (deg):",
          np.round([max(S._angle(Q[r, k, :3, :3], S._rot_mean(Q[:, k, :3, :3])) for r in range(R))
                    for k in range(frames)], 4).tolist())
    print("reference runs' e_r (deg):", np.round(penv[3], 4).tolist())
    ref_true = [float(np.linalg.norm(Pr[frames - 1][:3, 3] - z["truth_poses"][frames - 1][:3, 3]))
                for Pr in z["env_hist_pose"]]
    print("reference runs' last pose from the truth (m):", np.round(ref_true, 4).tolist())


if __name__ == "__main__":
    main()
