#!/usr/bin/env python3
"""Frame 0 of the configs[0] replay (tests/golden/slam_seq.npz) on the drop-in classes: the
decoder and the local features after the first n Adam steps of frame 0's 600-iteration mapping()
call, for the n of tests/golden/gen_slam_envelope.py's TRACE_STEPS (its f0trace mode records the
same for the reference).  Each n is a fresh run of frame 0 with mapping(n): the replayed draws and
the fresh optimiser make it the first n iterations of the long call.

Usage: python tools/f0_trace.py [det 0|1] -> gpurun_out/f0trace_det<det>.npz
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests.test_gpu_slam import _sequence  # noqa: E402

STEPS = (1, 2, 3, 5, 10, 20, 50, 100, 200, 400, 600)


def main(det):
    z = dict(np.load("tests/golden/slam_seq.npz", allow_pickle=False))
    rec = {}
    for n in STEPS:
        nm, dec, mapper, loop, replay, draws, scans = _sequence(z, "cuda", 1)
        mapper.deterministic = det
        loop.read_and_preprocess(scans[0])
        nm.travel_dist = torch.tensor(np.array(loop.travel_dist), dtype=torch.float32, device="cuda")
        d = draws(loop.cur_point_cloud_torch.shape[0])
        mapper.process_frame(loop.cur_point_cloud_torch, None, loop.cur_pose_torch, 0, False, draws=d)
        mapper.mapping(n)
        for k, p in zip(("W1", "b1", "W2", "b2"), dec.parameters()):
            rec[f"s{n}_{k}"] = p.detach().cpu().numpy().copy()
        rec[f"s{n}_feat"] = nm.local_geo_features.detach().cpu().numpy().copy()
        print(n, "b2", float(rec[f"s{n}_b2"][0]), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(f"gpurun_out/f0trace_det{int(det)}.npz", **rec)


if __name__ == "__main__":
    main((sys.argv[1] if len(sys.argv) > 1 else "1") == "1")
