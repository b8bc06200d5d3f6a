#!/usr/bin/env python3
"""Headline benchmark: SDF + analytic gradient queries/s over a 1M-neural-point map.

Workload (BASELINE.json configs[1]): synthetic 1M-point
surface map (1000 x 1000 voxels of 0.3 m, hash table B = 5e7), 262,144 queries
per step = map points + N(0, 0.25^2), Kc = 33 cells (num_nei_cells 2, alpha 0.2),
k = 8, F = 8, decoder 11 -> 64 -> 1, weighted_first, fp32, query_locally=False.
One step = the Tracker's fused query over the batch (pin_query_sort: the queries counting-sorted
into spatial tiles, then one pin_query_sdf_grid_sorted launch whose outputs stay in tile order,
PIN_QUERY_OUT_TILE, as the registration's normal equations consume them), inputs resident in HBM;
the same step with the outputs scattered back to input order (what a generic query_sdf caller
gets) is reported beside it as "input_order".  Multi-GPU: one process per GPU, each rank queries its own 262,144-point
batch against its replica of the map ("weak" scaling, no data-path collective);
the barrier + max-over-ranks timing is the only collective.

Further legs in the same line (informational; `value` stays the headline): "tracker"
(configs[2], registration steps/s on 200K source points), "mesher" (configs[4], 512^3 grid
SDF+mask, z-slabs per rank) and "mapper" (configs[3], iterations/s of Mapper.mapping on a
4M-point map with 1M queries per iteration per GPU; when N > 1 the feature gradients are
reduce-scattered over RCCL, each rank steps its 1/N of the rows and the rows are all-gathered).

Prints ONE JSON line (rank 0).  Roofline: achieved = 944 B/query (SURVEY.md 8(d):
12 q + 8*Kc slots + 12*Kc positions + 4*F*k features + 16 out) x queries per launch /
mean duration of the SDF+grad kernel alone (HIP events on the launch stream around
pin_query_sdf_grid_sorted with the sort precomputed); the ordering pass is reported beside it.  cpu_baseline: the
PyTorch-CPU restatement (oracle/pin_torch_cpu.py, every core the process may use, median of 5) on one full batch,
rank 0 at N=1 only.
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import pin_slam_amd as P  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_pool, surface_queries  # noqa: E402

N_SIDE = 1000            # 1,000,000 neural points
N_QUERY = 262144
BYTES_PER_QUERY = 944    # SURVEY.md 8(d), Kc=33, k=8, F=8
HBM_PEAK = 8.0e12        # MI355X_MICROARCH.md (spec)
REF_CPU_QPS = 0.37e6     # the reference's SDF+grad queries/s on 8 Xeon cores (configs[1])
MAPPER_SIDE = 2000       # 4,000,000 neural points (configs[3])
MAPPER_BS = 1 << 20      # 1M sampled queries per iteration per GPU
MAPPER_POOL = 1 << 22    # training-sample pool


def mapper_bytes_per_iter(n, L, dec=10):
    """SURVEY.md 8(d) mapper bytes: forward 932 B/row over the batch + stencil rows, feature-grad
    scatter 2*4*F*k = 512 B/row, dense Adam (read p,g,m,v; write p,m,v,g=0) 32 B per feature."""
    rows = n + 6 * ((n + dec - 1) // dec)
    return rows * (932 + 512) + 32 * 8 * (L + 1)


TRAFFIC_FILE = os.path.join("profiles", "r06", "traffic.json")


def measured_traffic(kernel_prefix, path=TRAFFIC_FILE):
    """HBM-side bytes per launch of a kernel from a committed PMC pass (tools/traffic.sh ->
    profiles/r06/*.json: FETCH_SIZE x 2 + WRITE_SIZE per launch), or None."""
    try:
        with open(os.path.join(ROOT, path)) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    for k in t.get("kernels", []):
        if k["name"].startswith(kernel_prefix):
            return k["bytes_per_launch"]
    return None


MFMA_FILE = os.path.join(ROOT, "profiles", "mfma.json")
F16_DENSE_PEAK = 2.5e15   # MI355X_MICROARCH.md: BF16/F16 MFMA ~2.5 PF dense
ENGINE_CLOCK = 2.4e9


def mfma_evidence(kernel, wf, kern_ms):
    """The headline decoder's matrix-core work: F16 FLOPs per launch (48 v_mfma_f32_16x16x32_f16
    per 64-query wave per decode, weighted_first one decode per query, else 8) against the dense
    F16 peak at the live kernel time, plus the busy fraction from the committed PMC pass
    (tools/mfma_pmc.sh: SQ_VALU_MFMA_BUSY_CYCLES per launch over kernel cycles x 1024 SIMDs)."""
    waves = (N_QUERY + 63) // 64
    flop = waves * 48 * (16 * 16 * 32 * 2) * (1 if wf else 8)
    res = {"dtype": "f16 operands (f32 values split hi/lo), f32 accumulate", "instr": "v_mfma_f32_16x16x32_f16",
           "flop_per_launch": flop, "achieved_tflops": flop / (kern_ms * 1e-3) / 1e12,
           "peak_tflops": F16_DENSE_PEAK / 1e12, "frac": flop / (kern_ms * 1e-3) / F16_DENSE_PEAK,
           "busy_frac": None, "pmc_flop_per_launch": None, "source": "profiles/mfma.json"}
    try:
        with open(MFMA_FILE) as f:
            for k in json.load(f).get("kernels", []):
                if k["name"].startswith(kernel):
                    res["pmc_flop_per_launch"] = k.get("f16_flop")
                    if k.get("mfma_busy_cycles"):
                        res["busy_frac"] = k["mfma_busy_cycles"] / (kern_ms * 1e-3 * ENGINE_CLOCK * 1024)
    except (OSError, ValueError):
        pass
    return res


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--nwf", action="store_true", help="weighted_first=False variant (per-neighbour decoding)")
    ap.add_argument("--backend", default="auto", choices=["auto", "hash", "grid"])
    ap.add_argument("--no-mapper", action="store_true", help="skip the mapper leg (configs[3])")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (nccl = RCCL on ROCm; gloo only to rehearse N ranks on "
                         "fewer GPUs -- ranks then share devices round robin)")
    ap.add_argument("--no-tracker", action="store_true", help="skip the tracker leg (configs[2])")
    ap.add_argument("--no-mesher", action="store_true", help="skip the mesher leg (configs[4])")
    ap.add_argument("--no-map-update", action="store_true", help="skip the map-maintenance leg (8f rank 1)")
    ap.add_argument("--no-process-frame", action="store_true", help="skip the process_frame leg (8f rank 4)")
    ap.add_argument("--no-nwf-leg", action="store_true", help="skip the per-neighbour-decoding leg")
    ap.add_argument("--no-slam", action="store_true", help="skip the whole-frame leg (configs[0])")
    ap.add_argument("--no-input-order", action="store_true",
                    help="skip the input-order headline variant (profiles of the tile-order kernel alone)")
    ap.add_argument("--mapper-steps", type=int, default=10)
    ap.add_argument("--no-mapper-nwf", action="store_true",
                    help="skip the per-neighbour-decoding mapper leg (weighted_first False, configs[3] sizes)")
    ap.add_argument("--mapper-shard", default="dense", choices=["space", "dense"],
                    help="N > 1 mapper data parallelism of the 'mapper' leg: the dense all-reduce of the feature "
                         "gradient over RCCL (north_star's design, default) or owner-partitioned cells with halo "
                         "exchange (space); the other mode is reported beside it unless --no-mapper-alt")
    ap.add_argument("--no-mapper-alt", action="store_true",
                    help="N > 1: skip the mapper leg of the other shard mode")
    ap.add_argument("--mapper-warmup", type=int, default=3)
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="PMC-measured HBM bytes per launch (from profiles/), reported as roofline.traffic")
    return ap.parse_args()


def cpu_threads():
    """The CPU baseline's thread count: the cores this process may run on (BASELINE.md's plan),
    capped by OMP_NUM_THREADS when the host sets it (the GPU box gives one GPU's job 16)."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _timed_median(fn, runs=5):
    """One warm-up run, then the median of `runs` (BASELINE.md CPU-baseline plan)."""
    fn()
    times = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    return statistics.median(times)


def _torch_cpu_map(nm, wf, local=False):
    """The map of a drop-in NeuralPoints as oracle/pin_torch_cpu tensors on the host (the whole
    map is local in the synthetic workloads: global2local is the identity there)."""
    from oracle import pin_torch_cpu as T
    c = nm.config
    feats = nm.local_geo_features.detach() if local else nm.geo_features
    if local:
        assert nm.local_count() == nm.count(), "CPU baseline expects the whole map local"
    return T.TorchMap(nm.resolution, nm.buffer_size, nm.buffer_pt_index.cpu(), nm.neural_points.cpu(), feats.cpu(),
                      nm.point_certainties.cpu(), nm.neighbor_dx.cpu(), nm.max_valid_dist2, c.query_nn_k, wf)


def cpu_baseline(nm, dec, q, wf):
    """The PyTorch-CPU restatement (oracle/pin_torch_cpu.py: hash probes, sort, IDW, decoder,
    autograd gradient -- the reference's own algorithm as torch CPU ops) on one full batch of the
    same workload, on this process's cores; one warm-up, median of 5."""
    import torch as _t
    from oracle import pin_torch_cpu as T
    threads = cpu_threads()
    old = _t.get_num_threads()
    _t.set_num_threads(threads)
    try:
        m = _torch_cpu_map(nm, wf)
        mlp = T.TorchMLP(dec.layers[0].weight.detach().cpu(), dec.layers[0].bias.detach().cpu(),
                         dec.lout.weight.detach().cpu(), dec.lout.bias.detach().cpu(), dec.sdf_scale)
        qh = q.cpu()
        t = _timed_median(lambda: T.sdf_and_grad(m, mlp, qh))
    finally:
        _t.set_num_threads(old)
    return {"value": qh.shape[0] / t, "unit": "queries/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"one full {qh.shape[0]}-query batch over the same 1M-point map: oracle/pin_torch_cpu.py "
                      f"(torch {_t.__version__} CPU, {threads} threads, autograd gradient), one warm-up, median of 5 "
                      f"({t:.3f} s each)"}


def time_kernel(nm, dec, q, wf, backend, steps, flags=1, mode="global", nn_k=8, want_grad=True, zero_empty=False):
    """Mean duration (ms) of one query kernel alone -- HIP events on the launch stream around
    each pin_query_sdf(_grid) launch, with the tile order precomputed; flags 1: outputs in tile
    order (PIN_QUERY_OUT_TILE), 0: in input order -- and of the ordering pass (pin_query_sort) that
    each step also runs.  mode "local": the map as the tracker queries it (query_locally, the
    travel-distance filter); want_grad False / zero_empty: the mesher's SDF-only launch."""
    import ctypes  # noqa: F401
    from pin_slam_amd import _lib
    from pin_slam_amd.query import mlp_view, query_sort
    n = q.shape[0]
    hv, pv = nm._views(mode, mode == "local")
    mv = mlp_view(dec, packed=want_grad)
    sdf = torch.empty(n, device=q.device)
    grad = torch.empty((n, 3), device=q.device) if want_grad else None
    nn = torch.empty(n, dtype=torch.int32, device=q.device)
    std = None if wf else torch.empty(n, device=q.device)
    if backend == "grid":
        gv = nm.grid_view(mode, True)
        q4 = query_sort(gv, q)

        def launch():
            _lib.call("pin_query_sdf_grid_sorted_ex", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q4), n, nn_k, int(wf),
                      int(zero_empty), _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn), None, _lib.ptr(std), int(flags),
                      _lib.stream())

        def order_pass():
            query_sort(gv, q, out=q4)
    else:
        def launch():
            _lib.call("pin_query_sdf", hv.ref(), pv.ref(), mv.ref(), _lib.ptr(q), n, nn_k, int(wf), int(zero_empty),
                      _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn), None, _lib.ptr(std), _lib.stream())
        order_pass = None

    def mean_ms(fn):
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        return statistics.mean(a.elapsed_time(b) for a, b in ev)
    return mean_ms(launch), (mean_ms(order_pass) if order_pass else 0.0)


def query_kernel_name(backend, wf, want_grad=True):
    """rocprof name of the launched query instance: <WF, PGO, GRAD, FAT, MF> (grid), <WF, PGO,
    GRAD, MF> (hash); the SDF-only instance (mesher) decodes on the VALU."""
    from pin_slam_amd.query import _MLP_PACK
    mf = str(bool(_MLP_PACK) and want_grad).lower()
    g = str(bool(want_grad)).lower()
    if backend == "grid":
        return f"k_query_sdf_grid<{str(wf).lower()}, false, {g}, true, {mf}>"
    return f"k_query_sdf<{str(wf).lower()}, false, {g}, {mf}>"


def query_roofline(bytes_per_query, n, kern_ms, kernel, traffic_file=None, note=None):
    """roofline object of a query leg: algorithmic bytes per launch / the kernel's mean launch
    time (HIP events), HBM peak; traffic = the PMC bytes per launch of the same kernel from the
    committed profile (or None)."""
    achieved = bytes_per_query * n / (kern_ms * 1e-3)
    traffic = measured_traffic(kernel, traffic_file) if traffic_file else measured_traffic(kernel)
    out = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
           "frac": achieved / HBM_PEAK, "traffic": traffic, "kernel": kernel, "kernel_ms": kern_ms,
           "algorithmic_bytes_per_query": bytes_per_query, "queries_per_launch": n,
           "traffic_source": traffic_file or TRAFFIC_FILE}
    if note:
        out["note"] = note
    return out


def nwf_leg(nm, dec, q, args, world, rank=0, backend="grid"):
    """The same batch and map with per-neighbour decoding (weighted_first False: SDF = IDW mean
    of the 8 neighbours' decoded SDFs, plus its std and gradient) -- what the reference's lidar
    configs (config/lidar_slam/run_kitti.yaml:25 etc.) run.  Roofline: the same 944 algorithmic
    bytes per query as the headline (the decoder's 8 evaluations per query read no more memory),
    over the per-neighbour kernel's own launch time; CPU baseline: the restatement with
    per-neighbour decoding on one full batch."""
    def step():
        return P.query_sdf(nm, dec, q, query_locally=False, want_grad=True, want_certainty=False, want_std=True,
                           weighted_first=False, out_order="tile")
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    # median of 5 timed windows of K steps: the leg is a few ms long, and a one-off host stall
    # (allocator / garbage collection) inside a single window would otherwise set its number
    windows = []
    for _ in range(5):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        windows.append(time.perf_counter() - t0)
    el = statistics.median(windows)
    kern_ms, order_ms = time_kernel(nm, dec, q, False, backend, args.steps, flags=1)
    t = torch.tensor([el, kern_ms], dtype=torch.float64, device=q.device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el, kern_ms = float(t[0]), float(t[1])
    res = {"metric": "SDF+grad+std queries/sec, per-neighbour decoding", "value": q.shape[0] * args.steps * world / el,
           "unit": "queries/s", "ms_per_step": el / args.steps * 1e3, "scaling": "weak",
           "windows_ms_per_step": [w / args.steps * 1e3 for w in windows],
           "roofline": query_roofline(BYTES_PER_QUERY, q.shape[0], kern_ms, query_kernel_name(backend, False),
                                      note="the query kernel alone (tile order precomputed); ms_per_step adds the "
                                           "sort (outputs in tile order, as the headline)"),
           "config": {"workload": "configs[1] batch and map, weighted_first False (8 decoder evaluations per query)"}}
    res["roofline"]["order_pass_ms"] = order_ms
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(nm, dec, q, False)
    return res


TRACKER_SRC = 200_000      # configs[2]: source points per registration step
MESH_RES = 512             # configs[4]: 512^3 grid
MESH_BATCH = 1 << 20       # Mesher infer_bs (utils/config.py:569: bs * 64)
MAP_FRAME = 131_072        # 8f rank 1: points per scan frame (a 64-beam lidar sweep)


TRACKER_MAP_FRAMES = 12    # configs[2]: street map built from 12 frames with the known poses
TRACKER_COLS = 3200        # 64 beams x 3200 columns: ~200K hits per registration scan


def tracker_leg(args, dev, world, rank):
    """configs[2]: point-to-implicit registration of a KITTI-style 64-beam scan (64 x 3200 rays,
    ~200K points, no down-sampling) against a neural-point map of the synthetic street
    (pin_slam_amd.synthetic.street_map: 12 frames of process_frame + mapping with the known poses,
    run_kitti.yaml settings: voxel 0.4, k 6, alpha 0.5, per-neighbour decoding, GM 0.1 / 0.2,
    iter_n 100).  The scan is taken at the next pose along the street and registered from that
    pose perturbed by 0.2 m / 0.5 deg.  Timed: Tracker.registration_step (one fused SDF+grad query
    of every point, validity + Geman-McClure weights + f64 normal equations, 6x6 solve) per
    iteration, and the whole tracking() loop (utils/tracker.py:39-174) from the perturbed pose,
    whose result is checked against the true pose."""
    from pin_slam_amd.synthetic import Q_SCALE, lidar_scan, perturb_pose, street_map
    nm, dec, cfg, scene, poses, rng = street_map(TRACKER_MAP_FRAMES, device=dev, seed=21 + 1000 * rank)
    T_true = poses[TRACKER_MAP_FRAMES]
    scan = torch.from_numpy(lidar_scan(T_true, scene, rng, cols=TRACKER_COLS).astype(np.float32)
                            / np.float32(Q_SCALE)).to(dev)
    n_src = int(scan.shape[0])
    T_guess = perturb_pose(T_true)
    guess = torch.tensor(T_guess, dtype=torch.float64, device=dev)
    from pin_slam_amd.tracker import transform_points
    src = transform_points(scan, guess)                 # the scan posed with the guess (world frame)
    tr = P.Tracker(cfg, nm, dec)
    zeros = torch.zeros(n_src, device=dev)

    def step():
        return tr.registration_step(src, None, zeros, None, TRACKER_MAP_FRAMES, cfg.reg_min_grad_norm,
                                    cfg.reg_max_grad_norm, cfg.reg_GM_dist_m, cfg.reg_GM_grad, cfg.reg_lm_lambda)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    steps = max(args.steps // 2, 5)
    windows = []   # median of 5 timed windows (see nwf_leg)
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = step()
        torch.cuda.synchronize()
        windows.append(time.perf_counter() - t0)
    el = statistics.median(windows)
    if out[4].shape[0] < n_src // 4:   # a registration without valid points returns early: not the workload
        print(f"WARNING: tracker leg has only {out[4].shape[0]} valid points of {n_src}", file=sys.stderr)
    # the whole tracking() loop from the perturbed pose: the pipelined iterations (tile sort once,
    # re-posed sorted rows, one iteration enqueued ahead of the host)
    T_est, _, _, ok = tr.tracking(scan, guess)
    calls, its, twin = max(args.steps // 10, 3), [], []
    for _ in range(5):
        n_it = 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            T_est, _, _, ok = tr.tracking(scan, guess)
            n_it += tr.last_iterations
        torch.cuda.synchronize()
        twin.append(time.perf_counter() - t0)
        its.append(n_it)
    k = int(np.argsort(twin)[len(twin) // 2])
    Te = tr.last_pose.cpu().numpy()
    dR = Te[:3, :3].T @ T_true[:3, :3]
    rot_err = float(np.degrees(np.arccos(np.clip((np.trace(dR) - 1) / 2, -1.0, 1.0))))
    pos_err = float(np.linalg.norm(Te[:3, 3] - T_true[:3, 3]))
    loop = {"metric": "tracking-loop registration iterations/sec", "value": its[k] / twin[k], "unit": "iters/s",
            "ms_per_iter": twin[k] / its[k] * 1e3, "ms_per_call": twin[k] / calls * 1e3,
            "iterations_per_call": its[k] / calls, "valid": bool(ok), "status": tr.last_status,
            "pose_error_m": pos_err, "rot_error_deg": rot_err,
            "initial_error_m": float(np.linalg.norm(T_guess[:3, 3] - T_true[:3, 3])),
            "final_residual_cm": tr.last_residual_cm,
            "residual_bound_cm": cfg.surface_sample_range_m * 0.5 * 100.0,
            "note": "Tracker.tracking from the perturbed pose (0.2 m, 0.5 deg), median of 5 windows; iterations "
                    "counted as run; pose error against the true pose of the scan"}
    # the step's dominant kernel alone: the fused SDF + gradient (+ std) query of every source point
    # in the tracker's local mode, tile order precomputed.  Algorithmic bytes per query (SURVEY.md
    # 8(d) at run_kitti settings): 12 q + (8 slot + 12 position) x Kc + 4 F k features + 20 out
    # (sdf, grad, std; 16 with weighted_first)
    wf = bool(cfg.weighted_first)
    kc, k, F = int(nm.neighbor_K), int(cfg.query_nn_k), int(cfg.feature_dim)
    bpq = 12 + 20 * kc + 4 * F * k + (16 if wf else 20)
    kern_ms, order_ms = time_kernel(nm, dec, src, wf, nm.backend(), steps, flags=1, mode="local", nn_k=k)
    roof = query_roofline(bpq, n_src, kern_ms, query_kernel_name(nm.backend(), wf),
                          os.path.join("profiles", "r06", "tracker_traffic.json"),
                          note=f"12 + 20 x Kc {kc} + 4 x F {F} x k {k} + {16 if wf else 20} B per query; the query "
                               f"kernel of one registration step alone (tile order precomputed)")
    roof["order_pass_ms"] = order_ms
    res = {"metric": "tracker registration iterations/sec", "value": steps / el, "unit": "iters/s",
           "queries_per_sec": n_src * steps / el, "ms_per_iter": el / steps * 1e3, "steps": steps,
           "source_points": n_src, "valid_points": int(out[4].shape[0]), "map_points": nm.count(),
           "scaling": "replicas", "tracking_loop": loop, "roofline": roof,
            "config": {"workload": "Tracker.registration_step, KITTI-style 64 x 3200-ray scan (~200K points) against "
                                   "a 12-frame synthetic street map, run_kitti.yaml settings (configs[2])",
                       "note": "registration_step: one call (query, normal equations, device solve, one host "
                               "read of 39 doubles, valid-point gather) per timed iteration"}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = tracker_cpu_baseline(nm, dec, cfg, src)
    return res


def _torch_cpu_local_map(nm, wf):
    """The drop-in map in the tracker's local mode as oracle/pin_torch_cpu tensors: the hash
    table over every point, the travel-distance filter (model/neural_points.py:480-488), the
    global2local table and the local points / features the neighbours are read from."""
    from oracle import pin_torch_cpu as T
    c = nm.config
    td = nm.travel_dist.detach().cpu().numpy()
    ts_c = nm.point_ts_create.detach().cpu().numpy()
    dtd = np.abs(td[int(nm.cur_ts)] - td[ts_c])
    time_ok = torch.from_numpy(dtd < np.float32(nm.diff_travel_dist_local))
    return T.TorchMap(nm.resolution, nm.buffer_size, nm.buffer_pt_index.cpu(), nm.neural_points.cpu(),
                      nm.local_geo_features.detach().cpu(), nm.local_point_certainties.cpu(), nm.neighbor_dx.cpu(),
                      nm.max_valid_dist2, c.query_nn_k, wf, time_ok=time_ok, global2local=nm.global2local.cpu(),
                      local_points=nm.local_neural_points.cpu())


def tracker_cpu_baseline(nm, dec, cfg, src):
    """One registration step of the same ~200K-point cloud in the PyTorch-CPU restatement
    (oracle/pin_torch_cpu.registration_step: local-mode query with autograd gradient and IDW std,
    validity, Geman-McClure weights, normal equations, f64 solve -- utils/tracker.py:277-520) on
    this process's cores; one warm-up, median of 5."""
    import torch as _t
    from oracle import pin_torch_cpu as T
    threads = cpu_threads()
    old = _t.get_num_threads()
    _t.set_num_threads(threads)
    try:
        m = _torch_cpu_local_map(nm, bool(cfg.weighted_first))
        mlp = T.TorchMLP(dec.layers[0].weight.detach().cpu(), dec.layers[0].bias.detach().cpu(),
                         dec.lout.weight.detach().cpu(), dec.lout.bias.detach().cpu(), dec.sdf_scale)
        ph = src.detach().cpu()
        zeros = _t.zeros(ph.shape[0])
        max_std = float(cfg.surface_sample_range_m * cfg.max_sdf_std_ratio)
        valid = []

        def one():
            valid.append(T.registration_step(m, mlp, ph, zeros, cfg.reg_min_grad_norm, cfg.reg_max_grad_norm,
                                             cfg.reg_GM_dist_m, cfg.reg_GM_grad, cfg.reg_lm_lambda, max_std,
                                             int(cfg.query_nn_k))[1])
        t = _timed_median(one)
    finally:
        _t.set_num_threads(old)
    return {"value": 1.0 / t, "unit": "iters/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "queries_per_sec": ph.shape[0] / t, "valid_points": valid[-1],
            "sample": f"one registration step of the same {ph.shape[0]}-point cloud: oracle/pin_torch_cpu.py "
                      f"registration_step (torch {_t.__version__} CPU, {threads} threads, autograd gradient), one "
                      f"warm-up, median of 5 ({t:.3f} s each)"}


def mesher_leg(nm, dec, pts, args, dev, world, rank):
    """configs[4]: SDF-only + mc_mask (nn_count >= mesh_min_nn) over a 512^3 grid at 0.1 m
    (Mesher.query_points' device work, batches of infer_bs), split in z-slabs over the ranks
    (strong scaling); grid coordinates resident in HBM."""
    from pin_slam_amd.query import query_sdf
    from pin_slam_amd.synthetic import train_surface
    fit_loss = train_surface(nm, dec, pts, iters=300)   # a fitted SDF, so the mesh is of a real surface
    res = 0.1
    lo = pts.mean(0) - 0.5 * MESH_RES * res
    z0 = rank * MESH_RES // world
    z1 = (rank + 1) * MESH_RES // world
    i = torch.arange(MESH_RES, device=dev, dtype=torch.float32)
    zs = torch.arange(z0, z1, device=dev, dtype=torch.float32)
    gx, gy, gz = torch.meshgrid(i, i, zs, indexing="ij")
    coord = torch.stack([gx.reshape(-1), gy.reshape(-1), gz.reshape(-1)], 1) * res + lo.to(dev)
    n = coord.shape[0]
    mask = torch.empty(n, dtype=torch.bool, device=dev)
    sdf = torch.empty(n, device=dev)
    min_nn = int(nm.config.mesh_min_nn)

    def run():
        for b0 in range(0, n, MESH_BATCH):
            s, _, nn, _, _ = query_sdf(nm, dec, coord[b0:b0 + MESH_BATCH], query_locally=False, want_grad=False,
                                       zero_empty=True, want_certainty=False)
            sdf[b0:b0 + MESH_BATCH] = s
            mask[b0:b0 + MESH_BATCH] = nn >= min_nn
    run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t[0])
    # the query kernel alone over the whole slab: every batch's tile order precomputed, HIP events
    # around each SDF-only launch (zero_empty, mc mask from nn_count, outputs in grid order as the
    # mesher needs them), summed over the batches.
    # Algorithmic bytes split by the outcome of each query: a query with
    # neighbours reads 12 q + 8 Kc slots + 12 Kc positions + 4 F k features and writes 4 = 932 B;
    # an empty one (nn_count 0: every probed cell empty or out of range) only its 12 + 8 Kc + 4
    roof = None
    if nm.backend() == "grid":
        roof = mesher_kernel_roofline(nm, dec, coord)
    # marching cubes over this rank's slab (the reference runs skimage on the host, mesher.py:327)
    from pin_slam_amd.mesher import marching_cubes
    nzs = z1 - z0
    grid = sdf.view(MESH_RES, MESH_RES, nzs)
    gmask = mask.view(MESH_RES, MESH_RES, nzs)
    marching_cubes(grid, gmask)
    torch.cuda.synchronize()
    tm = time.perf_counter()
    reps = 3
    for _ in range(reps):
        mv, mf = marching_cubes(grid, gmask)
    torch.cuda.synchronize()
    mc_ms = (time.perf_counter() - tm) / reps * 1e3
    res = {"metric": "mesher grid SDF queries/sec", "value": MESH_RES ** 3 / el, "unit": "queries/s",
           "ms_per_grid": el * 1e3, "map_fit_loss": fit_loss, "scaling": "strong", "masked_fraction": float(mask.float().mean()),
           "roofline": roof,
            "marching_cubes": {"ms_per_slab": mc_ms, "vertices": int(mv.shape[0]), "faces": int(mf.shape[0]),
                               "note": "device marching cubes over this rank's masked slab, incl. the count "
                                       "read-back and degenerate-face filter"},
            "config": {"workload": "512^3 grid at 0.1 m over the 1M-point map, SDF + mc_mask, batches of 2^20, "
                                   "z-slabs per rank (configs[4])"}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        mid = (n // MESH_BATCH // 2) * MESH_BATCH
        res["cpu_baseline"] = mesher_cpu_baseline(nm, dec, coord[mid:mid + MESH_BATCH])
    return res


def mesher_kernel_roofline(nm, dec, coord):
    """roofline of the mesher's query kernel: algorithmic bytes of every query by outcome (932 B
    with neighbours, 12 + 8 Kc + 4 B without) over the summed HIP-event time of the SDF-only
    launches of every batch (tile order precomputed)."""
    from pin_slam_amd import _lib
    from pin_slam_amd.query import mlp_view, query_sort
    c = nm.config
    wf, k, F, kc = bool(c.weighted_first), int(c.query_nn_k), int(c.feature_dim), int(nm.neighbor_K)
    n = coord.shape[0]
    gv = nm.grid_view("global", True)
    _, pv = nm._views("global", False)
    mv = mlp_view(dec, packed=False)
    spans = [(a, min(n, a + MESH_BATCH)) for a in range(0, n, MESH_BATCH)]
    q4s = [query_sort(gv, coord[a:b]) for a, b in spans]
    sdf = torch.empty(n, device=coord.device)
    nn = torch.empty(n, dtype=torch.int32, device=coord.device)
    std = None if wf else torch.empty(n, device=coord.device)

    def launch(j):
        a, b = spans[j]
        _lib.call("pin_query_sdf_grid_sorted_ex", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q4s[j]), b - a, k, int(wf), 1,
                  _lib.ptr(sdf[a:b]), None, _lib.ptr(nn[a:b]), None, _lib.ptr(None if std is None else std[a:b]),
                  0, _lib.stream())
    for j in range(len(spans)):
        launch(j)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in spans]
    for j, (a, b) in enumerate(ev):
        a.record()
        launch(j)
        b.record()
    torch.cuda.synchronize()
    kern_ms = sum(a.elapsed_time(b) for a, b in ev)
    n_occ = int((nn >= 1).sum())
    b_occ = 12 + 20 * kc + 4 * F * k + 4
    b_empty = 12 + 8 * kc + 4
    algo = n_occ * b_occ + (n - n_occ) * b_empty
    achieved = algo / (kern_ms * 1e-3)
    kernel = query_kernel_name("grid", wf, want_grad=False)
    per_launch = measured_traffic(kernel)
    return {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK,
            "traffic": per_launch, "traffic_source": TRAFFIC_FILE + " (per 2^20-query launch)",
            "kernel": kernel, "kernel_ms_per_grid": kern_ms, "launches": len(spans),
            "queries_with_neighbours": n_occ, "queries_empty": n - n_occ,
            "algorithmic_bytes": {"with_neighbours": b_occ, "empty": b_empty, "per_grid": algo,
                                  "per_launch": algo / len(spans)},
            "note": "the SDF-only query kernel alone (tile order precomputed), summed over the grid's batches; "
                    "ms_per_grid adds the sorts, the mask and the output copies"}


def mesher_cpu_baseline(nm, dec, coord):
    """One 2^20-query batch of the same grid (the middle z-range of the slab) in the PyTorch-CPU
    restatement (oracle/pin_torch_cpu.sdf_only: Mesher.query_points' SDF + mc_mask,
    utils/mesher.py:41-136) on this process's cores; one warm-up, median of 5."""
    import torch as _t
    from oracle import pin_torch_cpu as T
    threads = cpu_threads()
    old = _t.get_num_threads()
    _t.set_num_threads(threads)
    try:
        m = _torch_cpu_map(nm, bool(nm.config.weighted_first))
        mlp = T.TorchMLP(dec.layers[0].weight.detach().cpu(), dec.layers[0].bias.detach().cpu(),
                         dec.lout.weight.detach().cpu(), dec.lout.bias.detach().cpu(), dec.sdf_scale)
        qh = coord.cpu()
        out = []
        t = _timed_median(lambda: out.append(T.sdf_only(m, mlp, qh, int(nm.config.mesh_min_nn))))
    finally:
        _t.set_num_threads(old)
    return {"value": qh.shape[0] / t, "unit": "queries/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"one {qh.shape[0]}-query batch of the grid (middle of the slab, "
                      f"{float(out[-1][1].float().mean()):.4f} masked): oracle/pin_torch_cpu.py sdf_only (torch "
                      f"{_t.__version__} CPU, {threads} threads), one warm-up, median of 5 ({t:.3f} s each)"}


_FRAME_TIMING = ("each frame timed on its own (synchronised before and after; the frame's own host syncs "
                 "already serialise it): value = frames / (mean frame time x frames), max over ranks; the "
                 "median frame time is reported beside it")


def _frame_times(run, frames):
    """Wall time of each call run(k), k in frames, each bracketed by device synchronisation."""
    out = []
    for k in frames:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(k)
        torch.cuda.synchronize()
        out.append(time.perf_counter() - t0)
    return out


def _frames_el(per_frame, nsteps, world, dev):
    """(mean frame time x nsteps, median frame time), each the max over ranks: the value is the
    whole sequence's throughput (the mean), the median is reported beside it."""
    t = torch.tensor([statistics.mean(per_frame) * nsteps, statistics.median(per_frame)], dtype=torch.float64,
                     device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), float(t[1])


def map_leg(args, dev, world, rank):
    """NeuralPoints.update per frame (voxel down-sample, hash probe +
    insert, reset_local_map over the whole map + local gathers) of a 131,072-point scan
    (50 m disk, the sensor advancing 2 m per frame) into the 1M-point surface map."""
    from pin_slam_amd.synthetic import surface_scan
    nm, _, pts = surface_map(N_SIDE, device=dev, buffer_size=int(5e7))
    nm.local_map_radius = 50.0
    nm.diff_travel_dist_local = 250.0
    nsteps = max(args.steps // 2, 5)
    nw = 3
    T = nw + nsteps
    nm.travel_dist = torch.arange(T, dtype=torch.float32, device=dev) * 2.0
    frames = [surface_scan(100.0 + 2.0 * k, 150.0, 50.0, MAP_FRAME, seed=100 + k + 1000 * rank, device=dev)
              for k in range(T)]
    sensors = [torch.tensor([100.0 + 2.0 * k, 150.0, 1.7], device=dev) for k in range(T)]
    M0 = nm.count()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = map_cpu_baseline(nm, frames[0], sensors[0])
    for k in range(nw):
        nm.update(frames[k], sensors[k], None, k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    per_frame = _frame_times(lambda k: nm.update(frames[k], sensors[k], None, k), range(nw, T))
    el, med = _frames_el(per_frame, nsteps, world, dev)
    res = {"metric": "map update frames/sec", "value": nsteps * world / el, "unit": "frames/s",
           "points_per_sec": MAP_FRAME * nsteps * world / el, "ms_per_frame": el / nsteps * 1e3,
           "median_ms_per_frame": med * 1e3, "timing": _FRAME_TIMING, "steps": nsteps,
           "frame_ms": [round(t * 1e3, 3) for t in per_frame],
           "map_points_before": M0, "map_points_after": nm.count(), "local_points": nm.local_count(),
           "scaling": "replicas",
           "config": {"workload": "NeuralPoints.update (+ reset_local_map) of 131072-point scans into the 1M-point "
                                  "surface map, 5e7-slot table, local radius 50 m (SURVEY.md 8f rank 1)",
                      "note": "per frame: two host syncs (new-point and local-point counts size the new tensors)"}}
    if cpu is not None:
        res["cpu_baseline"] = cpu
    return res


FRAME_RAYS = 65_536         # 8f rank 4: rays per mapping frame (a down-sampled 64-beam sweep)


def process_frame_leg(args, dev, world, rank):
    """Mapper.process_frame per frame -- DataSampler.sample of 65,536 rays
    (7 samples each, sensor + world frame in one launch), NeuralPoints.update with the near-surface
    samples, data-pool append, window filter every 10th frame, query_certainty of the new samples
    -- on the 1M-point surface map, the sensor advancing 2 m per frame."""
    import types
    from pin_slam_amd.synthetic import surface_scan
    nm, dec, pts = surface_map(N_SIDE, device=dev, buffer_size=int(5e7))
    cfg = nm.config
    cfg.bs_new_sample = 2048
    cfg.pool_filter_freq = 10
    cfg.track_on = True
    nsteps = max(args.steps // 2, 10)
    # warm-up frames cover the first window filters, up to one that finds the pool above
    # pool_capacity (frame 29: the capacity discards): the first run of each allocates pool-sized
    # buffers and loads ATen kernels never used before (the discards' randint and boolean sum took
    # ~16 ms of lazy code-object loading, once per process) -- not the steady state the metric
    # describes; the timed frames then include steady-state filters with discards (frames 39, 49)
    nw = 3 * int(cfg.pool_filter_freq)
    T = nw + nsteps
    nm.local_map_radius = 50.0
    nm.diff_travel_dist_local = 250.0
    nm.travel_dist = torch.arange(T, dtype=torch.float32, device=dev) * 2.0
    poses, frames = [], []
    for k in range(T):
        c = np.array([100.0 + 2.0 * k, 150.0, 1.7])
        pose = np.eye(4)
        pose[:3, 3] = c
        poses.append(pose)
        w = surface_scan(c[0], c[1], 50.0, FRAME_RAYS, seed=300 + k + 1000 * rank, device=dev)
        frames.append((w - torch.as_tensor(c, dtype=torch.float32, device=dev)).contiguous())
    ds = types.SimpleNamespace(odom_poses=poses, stop_status=False, gt_pose_provided=False)
    mapper = P.Mapper(cfg, ds, nm, dec)
    pose_t = [torch.as_tensor(p, device=dev) for p in poses]
    for k in range(nw):
        mapper.process_frame(frames[k], None, pose_t[k], k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    per_frame = _frame_times(lambda k: mapper.process_frame(frames[k], None, pose_t[k], k), range(nw, T))
    el, med = _frames_el(per_frame, nsteps, world, dev)
    res = {"metric": "mapper frames/sec (process_frame)", "value": nsteps * world / el, "unit": "frames/s",
           "samples_per_sec": FRAME_RAYS * mapper.ray_sample_count * nsteps * world / el,
           "ms_per_frame": el / nsteps * 1e3, "median_ms_per_frame": med * 1e3, "timing": _FRAME_TIMING,
           "frame_ms": [round(t * 1e3, 3) for t in per_frame],
           "steps": nsteps, "pool_samples": int(mapper.pool_sample_count),
           "map_points": nm.count(), "new_samples": int(mapper.new_idx.shape[0]), "scaling": "replicas",
           "config": {"workload": "Mapper.process_frame: 65536-ray frames, 7 samples/ray, into the 1M-point surface "
                                  "map (SURVEY.md 8f rank 4)"}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = sampler_cpu_baseline(cfg, frames[0])
    return res


def sampler_cpu_baseline(cfg, frame):
    """The numpy oracle's DataSampler.sample + transform of one frame (1 core); map update and
    pool bookkeeping excluded (the map_update leg times the former)."""
    from oracle import pin_oracle as O
    f = frame.cpu().numpy()
    n = f.shape[0]
    rng = np.random.default_rng(0)
    rs, rf, rb = rng.normal(size=3 * n).astype(np.float32), rng.random(2 * n, np.float32), rng.random(n, np.float32)
    t0 = time.perf_counter()
    coord, _, _ = O.sample_rays(f, rs, rf, rb, 3, 2, 1, cfg.surface_sample_range_m, cfg.free_sample_begin_ratio,
                                cfg.free_sample_end_dist_m, cfg.dist_weight_on, cfg.dist_weight_scale, cfg.max_range,
                                cfg.behind_dropoff_on)
    O.transform_points(coord, np.eye(4))
    el = time.perf_counter() - t0
    return {"value": 1.0 / el, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": "oracle sample_rays + transform of one 65536-ray frame (sampling only)"}


def map_cpu_baseline(nm, frame, sensor):
    """The numpy oracle's map_update + reset_local_map of one frame into the same map (1 core)."""
    from oracle import pin_oracle as O
    c = lambda t: t.detach().cpu().numpy()  # noqa: E731
    st = O.empty_map(float(nm.resolution), nm.buffer_size, c(nm.travel_dist), float(nm.diff_travel_dist_local))
    st.table = c(nm.buffer_pt_index).astype(np.int64)
    st.points, st.orientations = c(nm.neural_points), c(nm.point_orientations)
    st.ts_create, st.ts_update = c(nm.point_ts_create), c(nm.point_ts_update)
    st.certainties, st.geo_features = c(nm.point_certainties), c(nm.geo_features)
    f = c(frame)
    t0 = time.perf_counter()
    O.map_update(st, f, 0)
    O.reset_local_map(st, c(sensor), 0, float(nm.local_map_radius))
    el = time.perf_counter() - t0
    return {"value": 1.0 / el, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": "one 131072-point frame into the 1M-point map (oracle map_update + reset_local_map)"}


SLAM_FRAMES = 16           # configs[0]: timed frames after frame 0


def slam_frame_leg(args, dev, world, rank):
    """BASELINE configs[0] on the GPU: pin_slam.py's whole per-frame loop (:96-257) -- voxel
    down-sample + crop, the tracker's registration (run_demo.yaml: up to 20 iterations), travel
    distance, Mapper.process_frame (sampling, map update, pool), mapping(15) with the decoder
    training (frames < freeze_after_frame) -- over 64-beam x 1024-column scans of a synthetic
    street (pin_slam_amd.synthetic), run_demo.yaml settings, deskew off.  Frame 0 (the 15 x 40
    iteration warm-up of the empty map) is not timed; every later frame is, part by part
    (device-synchronised boundaries), the query index of the updated map (occupancy grid +
    compact records) as a part of its own."""
    from pin_slam_amd.synthetic import FrameLoop, Q_SCALE, lidar_scan, slam_poses, street_scene
    nsteps = SLAM_FRAMES
    cfg = P.Config(device=dev, reg_iter_n=20, track_on=True)     # config/lidar_slam/run_demo.yaml
    warm = int(cfg.pool_filter_freq)     # untimed: frame 0's 15 x 40 iterations .. the first pool filter
    rng = np.random.default_rng(21 + 1000 * rank)
    scene = street_scene(rng)
    poses = slam_poses(warm + nsteps)
    scans = [torch.from_numpy(lidar_scan(T, scene, rng).astype(np.float32) / np.float32(Q_SCALE)).to(dev)
             for T in poses]
    nm = P.NeuralPoints(cfg)
    torch.manual_seed(42)
    dec = P.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1).to(dev)
    tracker = P.Tracker(cfg, nm, dec)
    mapper = P.Mapper(cfg, None, nm, dec)
    loop = FrameLoop(cfg, nm, dec, tracker, mapper, build_index=True)
    # every frame hands the loop the next scan, preprocessed on a side stream while the device maps
    # (FrameLoop.prefetch): the scan's preprocessing does not depend on the map
    nxt = lambda k: scans[k + 1] if k + 1 < len(scans) else None   # noqa: E731
    for k in range(warm):
        loop.frame(scans[k], next_pts=nxt(k))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    parts, frame_s, valid = {}, [], 0
    for k in range(warm, warm + nsteps):
        stamps = []

        def mark(name):
            torch.cuda.synchronize()
            stamps.append((name, time.perf_counter()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        valid += int(loop.frame(scans[k], timer=mark, next_pts=nxt(k)))
        prev = t0
        for name, t in stamps:
            parts.setdefault(name, []).append(t - prev)
            prev = t
        frame_s.append(prev - t0)
    el, med = _frames_el(frame_s, nsteps, world, dev)
    err = max(float(np.linalg.norm(np.asarray(loop.odom_poses[k])[:3, 3] - poses[k][:3, 3]))
              for k in range(warm + nsteps))
    return {"metric": "SLAM frames/sec (pin_slam.py frame loop)", "value": nsteps * world / el, "unit": "frames/s",
            "ms_per_frame": el / nsteps * 1e3, "median_ms_per_frame": med * 1e3,
            "frame_ms": [round(t * 1e3, 3) for t in frame_s],
            "parts_mean_ms": {k: round(statistics.mean(v) * 1e3, 4) for k, v in parts.items()},
            "frames": nsteps, "valid_frames": valid, "max_pose_error_m": err, "map_points": nm.count(),
            "pool_samples": int(mapper.pool_sample_count), "scaling": "replicas", "timing": _FRAME_TIMING,
            "config": {"workload": "configs[0]: synthetic 64-beam street sequence (64K points/scan), run_demo.yaml "
                                   "settings (voxel 0.3, k 6, weighted_first, tracker iter_n 20, bs 16384, iters "
                                   "15, decoder trained), deskew off; the next scan preprocessed on a side stream "
                                   "during each frame's mapping (FrameLoop.prefetch)",
                       "timed_frames": f"{warm}..{warm + nsteps - 1}",
                       "note": f"frames 0..{warm - 1} are not timed (frame 0: 15 x 40 mapping iterations on the "
                               f"empty map; frame {warm - 1}: the first pool window filter, pool_filter_freq "
                               f"{warm}); the timed frames include the filter of frame {2 * warm - 1}"}}


def mapper_cpu_baseline(nm, dec, coord, label, full_rows=None):
    """One mapper iteration of the same workload in the PyTorch-CPU restatement
    (oracle/pin_torch_cpu.py: the batch + its 6 x N/10 numerical-gradient stencil rows,
    training-mode query, BCE + eikonal, backward, Adam on the [L+1, 8] features, decoder frozen),
    on this process's cores; one warm-up, median of 5.  full_rows: the batch is a sample of a
    full_rows batch (the per-neighbour iteration, ~8x the decoder work, is timed on a quarter
    batch to bound the CPU time); the rate is then scaled to a full iteration by the row ratio
    (the [L+1, 8] Adam, ~2 % of the CPU iteration, scaled with it: a slightly low baseline)."""
    import torch as _t
    from oracle import pin_torch_cpu as T
    threads = cpu_threads()
    old = _t.get_num_threads()
    _t.set_num_threads(threads)
    c = nm.config
    wf = bool(c.weighted_first)
    try:
        m = _torch_cpu_map(nm, wf, local=True)
        mlp = T.TorchMLP(dec.layers[0].weight.detach().cpu(), dec.layers[0].bias.detach().cpu(),
                         dec.lout.weight.detach().cpu(), dec.lout.bias.detach().cpu(), dec.sdf_scale)
        feats = _t.nn.Parameter(m.features.clone())
        cert = m.certainties.clone()
        ch, lh = coord.cpu(), label.cpu()
        sigma = float(c.logistic_gaussian_ratio * c.sigma_sigmoid_m)
        eps = float(c.voxel_size_m * c.num_grad_step_ratio)

        def one():
            opt = _t.optim.Adam([feats], lr=c.lr, betas=(0.9, 0.99), eps=c.adam_eps)
            T.mapping_iteration(m, mlp, feats, opt, ch, lh, sigma, c.weight_e, int(c.gradient_decimation), eps, cert)
        t = _timed_median(one)
    finally:
        _t.set_num_threads(old)
    scale = (full_rows or coord.shape[0]) / coord.shape[0]
    what = ("one full iteration" if scale == 1 else
            f"a {coord.shape[0]}-row sample of the {full_rows}-row iteration, rate scaled by {scale:g}")
    return {"value": 1.0 / (t * scale), "unit": "iters/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{what} ({coord.shape[0]} batch rows + stencil, {m.points.shape[0]}-point map, weighted_first "
                      f"{wf}): oracle/pin_torch_cpu.py (torch {_t.__version__} CPU, {threads} threads, autograd "
                      f"backward, torch.optim.Adam), one warm-up, median of 5 ({t:.2f} s each)"}


def _shard_info(mapper):
    """Owned / halo rows of this rank's slab and the halo exchange bytes per iteration."""
    p = getattr(mapper, "_partition", None)
    if p is None:
        return None
    halo = int(p.halo.numel())
    sent = sum(int(r.numel()) for r in p.send_rows.values())
    return {"mode": "space (owner-partitioned cells, halo exchange, shared quirk row)", "cells": list(p.shape),
            "owned_rows": int(p.owned.numel()), "halo_rows": halo, "exchange_bytes_per_iter": 2 * 32 * (halo + sent),
            "batch": "each rank draws its batch from its cell's pool samples, rows weighted so that the union is an "
                     "unbiased estimate of one reference batch (DESIGN.md section 6)"}


def _ar_buckets():
    from pin_slam_amd.mapper import _AR_BUCKETS
    return _AR_BUCKETS


def mapper_leg(args, dev, world, rank, wf=None, shard=None):
    """configs[3]: Mapper.mapping on a 4M-point map, 1M sampled queries per iteration per GPU
    (+ 6 x 100K numerical-gradient stencil rows), BCE + 0.5 eikonal, Adam on the features
    (decoder frozen, the steady state after freeze_after_frame).  W > 1 (weak scaling, 1M queries
    per rank): --mapper-shard space (default) -- every rank owns a slab of the map, samples its
    batches there and exchanges only halo gradient / feature rows with the neighbouring slabs
    (pin_slam_amd.sharding); dense -- every rank samples the whole map, the [L+1,8] feature
    gradient is reduce-scattered over RCCL, Adam steps each rank's 1/W of the rows and the rows
    are all-gathered every iteration (sharding.OwnerAdam)."""
    wf = (not args.nwf) if wf is None else wf
    nm, dec, pts = surface_map(MAPPER_SIDE, device=dev, buffer_size=int(5e7), nn_k=8, weighted_first=wf,
                               query_backend=args.backend, bs=MAPPER_BS)
    for p in dec.parameters():
        p.requires_grad_(False)
    coord, label, ts = surface_pool(pts, MAPPER_POOL, seed=11 + rank, device=dev)
    shard = (shard or args.mapper_shard) if world > 1 else "dense"
    mapper = P.Mapper(nm.config, None, nm, dec, group=dist.group.WORLD if world > 1 else None, shard=shard)
    L = int(nm.local_neural_points.shape[0])
    mapper.set_pool(coord, label, ts)
    torch.manual_seed(1234 + rank)
    backend = nm.backend()
    progress(f"mapper ({shard}, wf {wf}): map and pool built, warm-up")
    mapper.mapping(max(args.mapper_warmup, 1))
    progress("mapper: timed iterations")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    mapper.mapping(args.mapper_steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])
    bpi = mapper_bytes_per_iter(MAPPER_BS, L)
    ms = elapsed / args.mapper_steps * 1e3
    replicas_identical = None
    if world > 1:
        # every rank must end with the same map (the data-parallel step applies one update to every
        # replica): a checksum of the features and certainties, compared across ranks
        f = nm.geo_features.detach().double()
        ck = torch.stack([f.sum(), (f * f).sum(), f.abs().max(), nm.point_certainties.double().sum()]).to(dev)
        allck = [torch.zeros_like(ck) for _ in range(world)]
        if dist.get_backend() == "gloo":
            hk = [t.cpu() for t in allck]
            dist.all_gather(hk, ck.cpu())
            allck = hk
        else:
            dist.all_gather(allck, ck)
        replicas_identical = all(torch.equal(allck[0].cpu(), t.cpu()) for t in allck)
    res = {"metric": "mapper iters/sec", "value": args.mapper_steps / elapsed, "unit": "iters/s",
           "queries_per_sec": MAPPER_BS * world * args.mapper_steps / elapsed, "ms_per_iter": ms,
           "steps": args.mapper_steps, "warmup": args.mapper_warmup, "scaling": "weak",
           "replicas_identical": replicas_identical,
           "config": {"workload": "Mapper.mapping, 4M-point map, 1M queries/iter/GPU + numerical-gradient "
                                  "stencil (configs[3])", "map_points": int(pts.shape[0]),
                      "queries_per_iter_per_gpu": MAPPER_BS, "decoder": "frozen", "optimizer": "Adam on features",
                      "weighted_first": wf, "data_parallel": shard if world > 1 else None,
                      "grad_exchange": (f"{dist.get_backend()} reduce_scatter of the [L+1,8] f32 gradient "
                                        f"({4 * 8 * (L + 1) / 1e6:.0f} MB/iter) in {_ar_buckets()} row buckets, Adam "
                                        f"on this rank's 1/{world} of each bucket as soon as it lands, all_gather of "
                                        f"the stepped rows (sharding.OwnerAdam)") if world > 1 and shard == "dense"
                      else None,
                      "shard": (_shard_info(mapper) if world > 1 and shard == "space" else None),
                      "candidate_backend": backend, "timed": "mapping(K): K iterations + Adam state init + "
                                                             "assign_local_to_global"},
           "roofline": {"bound": "hbm", "achieved": bpi / (ms * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9,
                        "unit": "GB/s", "frac": bpi / (ms * 1e-3) / HBM_PEAK,
                        "scope": "whole iteration", "algorithmic_bytes_per_iter": bpi,
                        **mapper_traffic(wf)}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rows = MAPPER_BS if wf else MAPPER_BS // 4
        idx = torch.randint(0, MAPPER_POOL, (rows,), device=dev)
        res["cpu_baseline"] = mapper_cpu_baseline(nm, dec, coord[idx], label[idx], full_rows=MAPPER_BS)
    return res


def mapper_iter_kernels(wf):
    """The kernels one mapper iteration launches once each (gather, tile sort of the rows, forward,
    backward, loss reduction, Adam); their PMC bytes per launch summed are the iteration's
    traffic.  The forward instances carry weighted_first as their first template argument, the
    per-neighbour backward is k_train_backward_nwf_sorted; the others are shared by both decoding
    modes (same sizes)."""
    w = str(bool(wf)).lower()
    bwd = "k_train_backward<true," if wf else "k_train_backward_nwf_sorted"
    return ("k_train_gather_packed", "k_tile_rank<16, 16384>", "k_tile_place<2, 16384>",
            f"k_train_forward_grid<{w},", bwd, "k_loss_final", "k_adam_train")


def mapper_traffic(wf):
    """roofline.traffic of a mapper leg: the HBM bytes of one iteration's kernels from the committed
    PMC pass over the mapper legs (profiles/r06/mapper_traffic.json, tools/traffic.sh), with the
    per-kernel split."""
    path = os.path.join("profiles", "r06", "mapper_traffic.json")
    parts = {}
    kernels = mapper_iter_kernels(wf)
    for k in kernels:
        b = measured_traffic(k, path)
        if b is not None:
            parts[k] = b
    if len(parts) != len(kernels):
        return {"traffic": None, "traffic_source": path + " (missing)"}
    return {"traffic": sum(parts.values()), "traffic_source": path, "traffic_per_kernel": parts}


_T0 = time.perf_counter()


def progress(msg):
    """A progress line on stderr (rank 0): long multi-rank runs print as they go."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def _fresh_allocator():
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and local_rank >= ndev:
        raise SystemExit(f"LOCAL_RANK {local_rank} but only {ndev} visible GPU(s)")
    dev_index = local_rank % max(ndev, 1)
    torch.cuda.set_device(dev_index)
    dev = f"cuda:{dev_index}"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(dev))
        else:
            dist.init_process_group("gloo")
    wf = not args.nwf
    nm, dec, pts = surface_map(N_SIDE, device=dev, buffer_size=int(5e7), nn_k=8, weighted_first=wf,
                               query_backend=args.backend)
    q = surface_queries(pts, N_QUERY, seed=7 + rank, device=dev)
    # derived map state (occupancy grid + compact records) is built once per map version,
    # like the hash table itself; time it separately
    def index_build():
        torch.cuda.synchronize()
        tb = time.perf_counter()
        be = nm.backend()
        if be == "grid":
            nm.compact_records("global", True)
        torch.cuda.synchronize()
        return be, (time.perf_counter() - tb) * 1e3
    backend, build_cold_ms = index_build()        # first build: allocations, the brick box sized
    builds = []
    for _ in range(3):   # rebuilds after an insert (what a SLAM frame pays): every derived index dropped
        nm._cache.clear()
        builds.append(index_build()[1])
    build_ms = statistics.median(builds)

    def step(order="tile"):
        return P.query_sdf(nm, dec, q, query_locally=False, want_grad=True, want_certainty=False,
                           want_std=not wf, out_order=order)

    def window(order):
        for _ in range(args.warmup):
            step(order)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(order)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return time.perf_counter() - t0
    progress("headline")
    elapsed = window("tile")
    kern_ms, order_ms = time_kernel(nm, dec, q, wf, backend, args.steps, flags=1)
    elapsed_in = kern_in_ms = float("nan")
    if not args.no_input_order:
        elapsed_in = window("input")
        kern_in_ms, _ = time_kernel(nm, dec, q, wf, backend, args.steps, flags=0)
    t = torch.tensor([elapsed, kern_ms, order_ms, elapsed_in, kern_in_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms, order_ms, elapsed_in, kern_in_ms = (float(v) for v in t)
    total_q = N_QUERY * args.steps * world
    value = total_q / elapsed
    achieved = BYTES_PER_QUERY * N_QUERY / (kern_ms * 1e-3)
    # the launched instance: <WF, PGO, GRAD, FAT, MF> (grid) / <WF, PGO, GRAD, MF> (hash)
    from pin_slam_amd.query import _MLP_PACK
    kernel_full = query_kernel_name(backend, wf)
    kernel_name = kernel_full.split("<")[0]
    traffic = args.traffic_bytes if args.traffic_bytes is not None else measured_traffic(kernel_full)
    out = {
        "metric": "SDF+grad queries/sec over 1M-point map",
        "value": value,
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (decoder operands as f16 hi+lo pairs on the matrix cores, f32 accumulate)",
        "data": "synthetic",
        "config": {"workload": "SDF+analytic-grad, 1M-point surface map, 262144 queries/step/GPU (configs[1])",
                   "map_points": int(pts.shape[0]), "queries_per_step_per_gpu": N_QUERY, "Kc": int(nm.neighbor_K),
                   "nn_k": 8, "feature_dim": 8, "mlp": "11-64-1", "weighted_first": wf,
                   "buffer_size": int(nm.buffer_size), "parallelism": f"replicas x{world}",
                   "candidate_backend": backend, "map_index_build_ms": round(build_ms, 3),
                   "map_index_first_build_ms": round(build_cold_ms, 3)},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK,
                     "traffic": traffic,
                     "traffic_source": TRAFFIC_FILE + " (rocprofv3 --pmc FETCH_SIZE + WRITE_SIZE, "
                                      "FETCH x2 per MI355X_MICROARCH.md gfx950 note)",
                     "kernel": kernel_name, "kernel_ms": kern_ms,
                     "order_pass_ms": order_ms,
                     "algorithmic_bytes_per_query": BYTES_PER_QUERY,
                     # the three views of the same number: the kernel alone (frac, above);
                     # the whole step by BASELINE.md's formula, queries/s x 944 B / 8 TB/s (sort, launches
                     # and host time included); the HBM bytes the PMC counters saw per launch over the
                     # kernel's time (below 1 where neighbouring queries share lines in L2)
                     "frac_kernel": achieved / HBM_PEAK,
                     "frac_step": (value / world) * BYTES_PER_QUERY / HBM_PEAK,
                     "frac_pmc_traffic": (traffic / (kern_ms * 1e-3) / HBM_PEAK) if traffic else None},
        "mfma": mfma_evidence(kernel_full, wf, kern_ms) if _MLP_PACK else None,
        # the same step with the outputs scattered to each query's own index (query_sdf's default
        # for callers that index the outputs by query): same work, uncoalesced stores
        "input_order": None if args.no_input_order else {
            "value": total_q / elapsed_in, "unit": "queries/s", "ms_per_step": elapsed_in / args.steps * 1e3,
            "kernel_ms": kern_in_ms, "frac_kernel": BYTES_PER_QUERY * N_QUERY / (kern_in_ms * 1e-3) / HBM_PEAK},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("cpu baseline")
        out["cpu_baseline"] = cpu_baseline(nm, dec, q, wf)
    if wf and not args.no_nwf_leg:
        progress("per_neighbour")
        out["per_neighbour"] = nwf_leg(nm, dec, q, args, world, rank, backend)
    if not args.no_mesher:
        progress("mesher")
        out["mesher"] = mesher_leg(nm, dec, pts, args, dev, world, rank)
    del nm, dec, pts, q
    # every further leg builds its own workload: start each from an empty caching allocator, so a
    # leg's timed frames do not pay for releasing an earlier leg's cached blocks (the first timed
    # map_update frame took ~22 ms when the allocator freed the headline's blocks inside it)
    _fresh_allocator()
    if not args.no_tracker:
        progress("tracker")
        out["tracker"] = tracker_leg(args, dev, world, rank)
        _fresh_allocator()
    if not args.no_map_update:
        progress("map_update")
        out["map_update"] = map_leg(args, dev, world, rank)
        _fresh_allocator()
    if not args.no_process_frame:
        progress("process_frame")
        out["process_frame"] = process_frame_leg(args, dev, world, rank)
        _fresh_allocator()
    if not args.no_slam:
        progress("slam_frame")
        out["slam_frame"] = slam_frame_leg(args, dev, world, rank)
        _fresh_allocator()
    if not args.no_mapper:
        progress("mapper")
        out["mapper"] = mapper_leg(args, dev, world, rank)
        _fresh_allocator()
        if world > 1 and not args.no_mapper_alt:
            # both data-parallel designs in one line: the dense gradient all-reduce (north_star's
            # RCCL step) and the owner-partitioned cells with halo exchange
            alt = "space" if args.mapper_shard == "dense" else "dense"
            progress("mapper (other shard mode)")
            out["mapper_" + alt] = mapper_leg(args, dev, world, rank, shard=alt)
            _fresh_allocator()
    if not args.no_mapper and not args.no_mapper_nwf and not args.nwf:
        # per-neighbour decoding (weighted_first False: run_kitti / mulran / ncd_128 / livox .yaml)
        progress("mapper_nwf")
        out["mapper_nwf"] = mapper_leg(args, dev, world, rank, wf=False)
    # speed-up over the CPU baseline measured in the same run (BASELINE.md's CPU-baseline plan: "speed-up"
    # per config); at N > 1 no CPU baseline runs, and the headline is set against BASELINE.md's own
    # measurement of the reference (0.37M SDF+grad queries/s on 8 cores)
    if "cpu_baseline" in out:
        out["vs_baseline"] = value / out["cpu_baseline"]["value"]
        out["vs_baseline_basis"] = "value / cpu_baseline.value (same run)"
    else:
        out["vs_baseline"] = value / REF_CPU_QPS
        out["vs_baseline_basis"] = "value / 0.37M q/s (BASELINE.md: the reference on 8 CPU cores)"
    for leg in out.values():
        if isinstance(leg, dict) and isinstance(leg.get("cpu_baseline"), dict) and "value" in leg:
            leg["vs_baseline"] = leg["value"] / leg["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
