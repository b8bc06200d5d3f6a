#!/usr/bin/env python3
"""One frame of the SLAM loop (default: the pool window-filter frame 19 of the bench leg; argv[1]
another) under torch.profiler: per op, host and device time, and per part of the frame the wall
time, the device-busy time (union of kernel intervals), kernel launches and blocking host reads.
Writes gpurun_out/filter_frame_trace.json (chrome trace) beside the printed tables."""
import os
import sys
import time

import numpy as np
import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import FrameLoop, Q_SCALE, lidar_scan, slam_poses, street_scene  # noqa: E402


def main(upto=19):
    dev = "cuda"
    rng = np.random.default_rng(21)
    scene = street_scene(rng)
    poses = slam_poses(upto + 2)
    scans = [torch.from_numpy(lidar_scan(T, scene, rng).astype(np.float32) / np.float32(Q_SCALE)).to(dev)
             for T in poses]
    cfg = P.Config(device=dev, reg_iter_n=20, track_on=True)
    nm = P.NeuralPoints(cfg)
    torch.manual_seed(42)
    dec = P.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1).to(dev)
    loop = FrameLoop(cfg, nm, dec, P.Tracker(cfg, nm, dec), P.Mapper(cfg, None, nm, dec), build_index=True)
    for k in range(upto - 1):
        loop.frame(scans[k])
    torch.cuda.synchronize()
    for k in (upto - 1, upto):
        parts = {}

        def mark(name, t=[None]):
            torch.cuda.synchronize()
            now = time.perf_counter()
            parts[name] = (now - t[0]) * 1e3
            t[0] = now
        torch.cuda.synchronize()
        mark.__defaults__[0][0] = time.perf_counter()
        if k == upto:
            rf = [torch.autograd.profiler.record_function("part:preprocess")]

            def mark_ranges(name):
                mark(name)
                rf[0].__exit__(None, None, None)
                nxt = {"preprocess": "index", "index": "tracking", "tracking": "process_frame",
                       "process_frame": "mapping"}.get(name, "end")
                rf[0] = torch.autograd.profiler.record_function("part:" + nxt)
                rf[0].__enter__()
            with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
                rf[0].__enter__()
                loop.frame(scans[k], timer=mark_ranges)
                rf[0].__exit__(None, None, None)
                torch.cuda.synchronize()
        else:
            loop.frame(scans[k], timer=mark)
        print(f"frame {k}: " + ", ".join(f"{a} {b:.3f}" for a, b in parts.items()), flush=True)
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=30, max_name_column_width=70))
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30, max_name_column_width=70))
    os.makedirs("gpurun_out", exist_ok=True)
    prof.export_chrome_trace("gpurun_out/filter_frame_trace.json")
    parts_report("gpurun_out/filter_frame_trace.json")


def parts_report(path):
    import json
    ev = json.load(open(path))["traceEvents"]
    parts = sorted([e for e in ev if e.get("cat") == "user_annotation" and e["name"].startswith("part:")],
                   key=lambda e: e["ts"])
    kern = sorted([e for e in ev if e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset")], key=lambda e: e["ts"])
    rt = [e for e in ev if e.get("cat") == "cuda_runtime"]
    print("part: wall ms, device busy ms, kernels, launches, blocking reads / syncs")
    for p in parts:
        a, b = p["ts"], p["ts"] + p["dur"]
        # kernels launched inside the part (their runtime call lies in it), busy = union of intervals
        ks = [k for k in kern if a <= k["ts"] < b]
        busy, end = 0.0, -1e30
        for k in ks:
            s0, s1 = max(k["ts"], end), k["ts"] + k["dur"]
            if s1 > s0:
                busy += s1 - s0
            end = max(end, s1)
        launches = sum(1 for r in rt if a <= r["ts"] < b and r["name"] == "hipLaunchKernel")
        reads = sum(1 for r in rt if a <= r["ts"] < b and r["name"] in ("hipMemcpyWithStream", "hipEventSynchronize",
                                                                        "hipStreamSynchronize"))
        print(f"  {p['name'][5:]:14s} {p['dur'] / 1e3:7.3f} {busy / 1e3:7.3f} {len(ks):5d} {launches:5d} {reads:4d}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 19)
