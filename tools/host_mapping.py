"""Host cost of the SLAM leg's mapping(15) calls: wall time of the call (its one closing sync
included) against the GPU time of its kernels, and a cProfile of the host side."""
import cProfile
import os
import pstats
import sys
import time

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
    torch.cuda.synchronize()
    walls = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mapper.mapping(15)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    print("mapping(15) wall ms:", [round(w * 1e3, 3) for w in walls])
    # host-side only: the calls queued behind a long sleep kernel (the GPU never waits on the host)
    def host_ms(fn, reps=3):
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            torch.cuda._sleep(200_000_000)
            t0 = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t0)
            torch.cuda.synchronize()
        return best * 1e3
    print(f"host only: mapping(15) {host_ms(lambda: mapper.mapping(15)):.3f} ms")
    idx = mapper._batch_parts
    print(f"host only: 15 x _batch_parts {host_ms(lambda: [idx() for _ in range(15)]):.3f} ms")
    print(f"host only: 15 x torch.randint pair {host_ms(lambda: [(torch.randint(0, 1000, (16384,), device=dev), torch.randint(0, 100, (100,), device=dev)) for _ in range(15)]):.3f} ms")
    nm.mark_modified(nm.local_geo_features)
    print(f"host only: 15 x _views {host_ms(lambda: [nm._views('local', True) for _ in range(15)]):.3f} ms")
    from pin_slam_amd.query import mlp_view
    print(f"host only: 15 x mlp_view(packed) after a decoder step "
          f"{host_ms(lambda: [(torch.autograd.graph.increment_version(dec.lout.bias), mlp_view(dec, packed=True)) for _ in range(15)]):.3f} ms")
    # the fused mapping loop by hand (mapping()'s dense branch), behind a sleep, timed per phase
    feats = nm.local_geo_features
    fdata = feats.data
    f_grad, f_m, f_v = torch.zeros_like(fdata), torch.zeros_like(fdata), torch.zeros_like(fdata)
    mlp_params = [p for p in dec.parameters() if p.requires_grad]
    m_grad = m_m = m_v = None
    if mlp_params:
        m_grad = torch.zeros((P._lib.MLP_GRAD_SIZE,), dtype=torch.float32, device=dev)
        m_m, m_v = torch.zeros_like(m_grad), torch.zeros_like(m_grad)
    packed = mapper._packed_pool()
    acc = {"batch": 0.0, "train_step": 0.0, "adam": 0.0}
    for rep in range(3):
        torch.cuda.synchronize()
        torch.cuda._sleep(100_000_000)
        for _ in range(15):
            t0 = time.perf_counter()
            index, new_sel, index_new = mapper._batch_parts()
            t1 = time.perf_counter()
            mapper.train_step(mapper.global_coord_pool, mapper.sdf_label_pool, mapper.time_pool, f_grad, m_grad, 1,
                              index=index, weight=mapper.weight_pool, packed=packed,
                              index_new=None if new_sel is None else (new_sel, index_new))
            t2 = time.perf_counter()
            mapper._adam(fdata, f_grad, f_m, f_v, mlp_params, m_grad, m_m, m_v)
            t3 = time.perf_counter()
            if rep == 2:
                acc["batch"] += t1 - t0
                acc["train_step"] += t2 - t1
                acc["adam"] += t3 - t2
        torch.cuda.synchronize()
    print("host only, 15 iterations by hand (ms):", {k: round(v * 1e3, 3) for k, v in acc.items()})
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    pr.enable()
    for _ in range(300):
        index, new_sel, index_new = mapper._batch_parts()
        mapper.train_step(mapper.global_coord_pool, mapper.sdf_label_pool, mapper.time_pool, f_grad, m_grad, 1,
                          index=index, weight=mapper.weight_pool, packed=packed,
                          index_new=None if new_sel is None else (new_sel, index_new))
        mapper._adam(fdata, f_grad, f_m, f_v, mlp_params, m_grad, m_m, m_v)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(40)


if __name__ == "__main__":
    main()
