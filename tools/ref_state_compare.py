#!/usr/bin/env python3
"""Build container only (imports /root/reference): the map state the tracking call of frame k
sees in the reference's pose-forced run (tests/golden/gen_slam_envelope.py forced, DUMP=k) against
this package's (tools/slam_forced.py, DUMP=k): field by field, then the reference's tracker on
hybrid states -- the reference's map with our features, with our decoder, with both -- so a
difference in the tracked pose can be traced to the field that carries it.

Usage: PYTHONDONTWRITEBYTECODE=1 python tools/ref_state_compare.py slam_seq 8 [threads]
"""
import copy
import os
import sys
import time
from unittest import mock

import numpy as np
import torch

sys.dont_write_bytecode = True
for _name in ["open3d", "roma", "wandb", "skimage", "skimage.measure", "natsort", "pyquaternion", "pypose", "laspy",
              "gtsam", "evo"]:
    sys.modules[_name] = mock.MagicMock(name=_name)
sys.path.insert(0, "/root/reference")
import utils.tools as rtools  # noqa: E402
rtools.get_time = time.time
import model.neural_points as rnp  # noqa: E402
rnp.get_time = time.time
from model.decoder import Decoder  # noqa: E402
import utils.tracker as rtracker  # noqa: E402
rtracker.get_time = time.time
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ref_track_dump import _load_ours  # noqa: E402


def _stats(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    if a.shape != b.shape:
        return f"shape {a.shape} vs {b.shape}"
    d = a - b
    return f"max |d| {np.abs(d).max():.3g}, mean d {d.mean():.3g}, rms {np.sqrt((d ** 2).mean()):.3g}, equal {np.mean(d == 0):.4f}"


def _track(npm, dec_sd, cfg, src, guess):
    dec = Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1)
    dec.load_state_dict(dec_sd)
    tr = rtracker.Tracker(cfg, npm, dec, None, None)
    T, _, _, _ = tr.tracking(src, guess, None, None)
    return T.numpy()


def main(name, k, threads=8):
    ref = torch.load(f"/tmp/slam_env/refdump_{name}_f{k}_t{threads}.pt", weights_only=False)   # written here
    rn, rdec = ref["npm"], ref["dec"]
    on, odec, z = _load_ours(f"gpurun_out/dump/{name}_f{k}")
    cfg = rn.config
    cfg.silence = True
    src = torch.from_numpy(z["source"])
    guess = torch.from_numpy(z["guess"])
    print(f"== {name} frame {k}: source {tuple(src.shape)} vs reference {tuple(ref['source'].shape)}; "
          f"guess diff {np.abs(z['guess'] - ref['guess'].numpy()).max():.3g}")
    for f in ("neural_points", "point_ts_create", "point_ts_update", "point_certainties", "geo_features",
              "local_neural_points", "local_point_certainties", "local_point_ts_update", "global2local", "local_mask",
              "travel_dist", "point_orientations"):
        a, b = getattr(on, f, None), getattr(rn, f, None)
        if a is None or b is None:
            print(f"  {f}: missing ({a is None}, {b is None})")
            continue
        print(f"  {f}: {_stats(a.detach().cpu().numpy(), b.detach().cpu().numpy())}")
    print(f"  local_geo_features: {_stats(on.local_geo_features.detach().numpy(), rn.local_geo_features.detach().numpy())}")
    print(f"  cur_ts ours {on.cur_ts} ref {rn.cur_ts}; table equal "
          f"{bool(torch.equal(on.buffer_pt_index.long(), rn.buffer_pt_index.long()))}")
    for key in rdec:
        print(f"  decoder {key}: {_stats(odec[key].numpy(), rdec[key].numpy())}")
    R = z["ref"][:3, :3]
    base = _track(copy.deepcopy(rn), rdec, cfg, src, guess)

    def rel(T):
        return np.round(R.T @ (T[:3, 3] - base[:3, 3]), 5)
    print("  reference tracker, reference state vs the stored pose:", np.round(R.T @ (base[:3, 3] - z["ref"][:3, 3]), 5))
    h = copy.deepcopy(rn)
    h.local_geo_features = torch.nn.Parameter(on.local_geo_features.detach().clone())
    h.geo_features = on.geo_features.detach().clone()
    print("  our features, reference decoder:", rel(_track(h, rdec, cfg, src, guess)))
    print("  reference features, our decoder:", rel(_track(copy.deepcopy(rn), odec, cfg, src, guess)))
    print("  our features and decoder:", rel(_track(h, odec, cfg, src, guess)))
    h2 = copy.deepcopy(rn)
    h2.point_certainties = on.point_certainties.clone()
    h2.local_point_certainties = on.local_point_certainties.clone()
    print("  our certainties only:", rel(_track(h2, rdec, cfg, src, guess)))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 8)
