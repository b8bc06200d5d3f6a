#!/usr/bin/env python3
"""Build container only (imports /root/reference): the reference's Tracker.tracking on a map state
this package's GPU run saved (tools/slam_forced.py with DUMP=frames: save_implicit_map of the map
the tracking call saw, plus the source cloud, the guess, our result and our per-iteration
increments).  Same map, same cloud, same guess: any difference is the trackers'.

Usage: PYTHONDONTWRITEBYTECODE=1 python tools/ref_track_dump.py gpurun_out/dump/slam_seq_f20 [threads]
"""
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


def _load_ours(d):
    """(reference NeuralPoints over our saved state, our decoder state_dict, track.npz)."""
    path = os.path.join(d, "model", "pin_map.pth")
    if not os.path.exists(path):
        import gzip
        import shutil
        with gzip.open(path + ".gz", "rb") as fi, open(path, "wb") as fo:
            shutil.copyfileobj(fi, fo)
    m = torch.load(path, weights_only=False, map_location="cpu")   # a file this package wrote
    npm = m["neural_points"]
    npm.config.device = "cpu"
    npm.config.silence = True
    npm.device = "cpu"
    return npm, m["geo_decoder"], np.load(os.path.join(d, "track.npz"))


def main(d, threads=8):
    torch.set_num_threads(threads)
    npm, dec_sd, z = _load_ours(d)
    cfg = npm.config
    dec = Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1)
    dec.load_state_dict(dec_sd)
    tr = rtracker.Tracker(cfg, npm, dec, None, None)
    deltas = []
    orig = tr.registration_step

    def step(*a, **kw):
        out = orig(*a, **kw)
        deltas.append(out[0].numpy().copy())
        return out
    tr.registration_step = step
    T, _, _, valid = tr.tracking(torch.from_numpy(z["source"]), torch.from_numpy(z["guess"]), None, None)
    T = T.numpy()
    ours = z["ours"]
    R = z["ref"][:3, :3]
    print(d, "valid", bool(valid), "iterations: reference", len(deltas), "ours", int(z["iterations"]))
    print("  reference tracker on our map vs the stored reference pose (body frame):",
          np.round(R.T @ (T[:3, 3] - z["ref"][:3, 3]), 5))
    print("  our tracker vs the reference tracker on the same map (body frame):",
          np.round(R.T @ (ours[:3, 3] - T[:3, 3]), 5))
    od = z["deltas"]
    for i in range(max(len(deltas), len(od))):
        a = deltas[i][:3, 3] if i < len(deltas) else None
        b = od[i][:3, 3] if i < len(od) else None
        print(f"  iter {i}: reference dt {None if a is None else np.round(a, 6)}  ours {None if b is None else np.round(b, 6)}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8)
