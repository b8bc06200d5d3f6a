"""References per map point in one SLAM-frame mapping iteration (GPU only): how many (row,
neighbour) pairs of the 16K-row batch + stencil land on each local point -- the contention the
backward's feature scatter sees."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import FrameLoop, Q_SCALE, lidar_scan, slam_poses, street_scene  # noqa: E402


def main(frames=12):
    dev = "cuda"
    rng = np.random.default_rng(21)
    scene = street_scene(rng)
    poses = slam_poses(frames)
    scans = [torch.from_numpy(lidar_scan(T, scene, rng).astype(np.float32) / np.float32(Q_SCALE)).to(dev)
             for T in poses]
    cfg = P.Config(device=dev, reg_iter_n=20, track_on=True)
    nm = P.NeuralPoints(cfg)
    torch.manual_seed(42)
    dec = P.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1).to(dev)
    tracker = P.Tracker(cfg, nm, dec)
    mapper = P.Mapper(cfg, None, nm, dec)
    loop = FrameLoop(cfg, nm, dec, tracker, mapper, build_index=True)
    for k in range(frames):
        loop.frame(scans[k])
    mapper.mapping(1)
    torch.cuda.synchronize()
    b = mapper._buf
    nn_k = int(cfg.query_nn_k)
    n = int(cfg.bs)
    c = cfg
    eik = bool(c.ekional_loss_on and c.weight_e > 0) and bool(c.numerical_grad)
    dec_ = int(c.gradient_decimation)
    nd = (n + dec_ - 1) // dec_ if eik else 0
    rows = n + 6 * nd
    ids = b.ids.flatten()[: rows * nn_k]
    print("rows", rows, "batch", n, "stencil groups", nd)
    print("local points", nm.local_geo_features.shape[0], "ids buffer", ids.numel(), "nn_k", nn_k)
    ids = ids[ids >= 0]
    cnt = torch.bincount(ids.long())
    cnt = cnt[cnt > 0].cpu().numpy()
    s = np.sort(cnt)[::-1]
    print(f"pairs {ids.numel()}, distinct points {cnt.size}, mean {cnt.mean():.2f}, max {s[0]}, "
          f"top10 {s[:10].tolist()}, p99 {np.percentile(cnt, 99):.0f}, p90 {np.percentile(cnt, 90):.0f}")
    print("share of pairs on the 1% most referenced points:", float(s[: max(1, s.size // 100)].sum() / s.sum()))


if __name__ == "__main__":
    main()
