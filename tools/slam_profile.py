"""Per-frame attribution of bench.py's whole-frame leg (configs[0]): part times of every frame,
and the pieces of process_frame / mapping that are worth tracking, synchronised around each."""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import FrameLoop, Q_SCALE, lidar_scan, slam_poses, street_scene  # noqa: E402


def main(frames=16):
    dev = "cuda"
    rng = np.random.default_rng(21)
    scene = street_scene(rng)
    poses = slam_poses(frames + 1)
    scans = [torch.from_numpy(lidar_scan(T, scene, rng).astype(np.float32) / np.float32(Q_SCALE)).to(dev)
             for T in poses]
    cfg = P.Config(device=dev, reg_iter_n=20, track_on=True)
    nm = P.NeuralPoints(cfg)
    torch.manual_seed(42)
    dec = P.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1).to(dev)
    tracker = P.Tracker(cfg, nm, dec)
    mapper = P.Mapper(cfg, None, nm, dec)
    loop = FrameLoop(cfg, nm, dec, tracker, mapper, build_index=True)
    loop.frame(scans[0])
    torch.cuda.synchronize()
    inner = {}

    def timed(obj, name, label):
        fn = getattr(obj, name)

        def wrap(*a, **kw):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn(*a, **kw)
            torch.cuda.synchronize()
            inner.setdefault(label, []).append(time.perf_counter() - t0)
            return out
        setattr(obj, name, wrap)
    timed(mapper.sampler, "sample", "pf.sample")
    timed(nm, "update", "pf.map_update")
    timed(nm, "query_certainty", "pf.query_certainty")
    timed(mapper, "_pool_compact", "pf.pool_compact")
    timed(mapper, "train_step", "map.train_step")
    timed(mapper, "_adam", "map.adam")
    timed(nm, "assign_local_to_global", "map.assign_local_to_global")
    timed(tracker, "_register", "trk.register")
    rows = []
    for k in range(1, frames + 1):
        stamps = []

        def mark(name):
            torch.cuda.synchronize()
            stamps.append((name, time.perf_counter()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.frame(scans[k], timer=mark)
        prev, row = t0, {}
        for name, t in stamps:
            row[name] = (t - prev) * 1e3
            prev = t
        row["total"] = (prev - t0) * 1e3
        rows.append(row)
        print(f"frame {k:2d} " + " ".join(f"{n} {v:7.3f}" for n, v in row.items()), flush=True)
    print("mean  " + " ".join(f"{n} {statistics.mean(r[n] for r in rows):7.3f}" for n in rows[0]))
    for k, v in inner.items():
        print(f"  {k:28s} n={len(v):4d} mean {statistics.mean(v) * 1e3:8.4f} ms  total {sum(v) * 1e3:9.3f} ms")


if __name__ == "__main__":
    main()
