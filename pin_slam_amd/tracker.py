"""Drop-in ``Tracker`` (utils/tracker.py:19): point-to-implicit registration on the GPU.

Per Gauss-Newton / LM iteration the reference evaluates ``query_feature`` + ``Decoder.sdf``
+ autograd ``get_gradient`` on every source point, filters, weights and forms a 6x6 system
with torch ops (:176-496).  Here one iteration is:

0. ``pin_transform_points``: the source cloud under the current pose (``tracking`` only);
1. ``pin_query_sdf{,_grid}``: fused k-NN gather, IDW, decoder and closed-form dSDF/dq;
2. ``pin_reg_normal_eq``: validity mask, Geman-McClure weights and the f64 normal equations
   in one deterministic reduction;
3. ``pin_reg_solve``: the 6x6 f64 solve, expmap, T = dT T and the convergence measures of dT on
   the device; one asynchronous copy of a 55-double record (accumulators, status, dT) per
   iteration drives the control flow (the reference syncs on ``.item()``-style reads several
   times per iteration).

``tracking`` (:39-174: convergence, validity checks, fall-back to the initial guess) keeps the
pose on the device and runs the iterations through ``_RegLoop``: iteration i+1 is enqueued
before the host reads iteration i (stream order carries the pose), the cloud is tile-sorted once
per call and re-posed in tile order afterwards.  ``install()`` transplants it onto the reference
class.  Colour / photometric registration is out of scope (off in every lidar config).
"""
import ctypes
import math
import os

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from . import query as _query
from .query import mlp_view, order_workspace, query_sdf as fused_query_sdf
from .sharding import all_reduce


def transform_torch(points: torch.Tensor, transformation: torch.Tensor) -> torch.Tensor:
    """utils/tools.py:386-399: homogeneous [N,4] x T^T in the points' dtype."""
    homo = torch.cat([points, torch.ones(points.shape[0], 1, device=points.device, dtype=points.dtype)], dim=1)
    return torch.matmul(homo, transformation.to(points).T)[:, :3]


def skew(v):
    S = torch.zeros(3, 3, device=v.device, dtype=v.dtype)
    S[0, 1] = -v[2]
    S[0, 2] = v[1]
    S[1, 2] = -v[0]
    return S - S.T


def expmap(axis_angle: torch.Tensor) -> torch.Tensor:
    """utils/tracker.py:580-589 (Rodrigues)."""
    angle = axis_angle.norm()
    axis = axis_angle / angle
    eye = torch.eye(3, device=axis_angle.device, dtype=axis_angle.dtype)
    S = skew(axis)
    return eye + S * torch.sin(angle) + (S @ S) * (1.0 - torch.cos(angle))


def rotation_matrix_to_axis_angle(R: torch.Tensor):
    """utils/tracker.py:591-599: rotation angle (rad) of R."""
    return torch.acos((torch.trace(R) - 1) / 2)


def _expmap_np(axis_angle: np.ndarray) -> np.ndarray:
    """utils/tracker.py:580-589 (Rodrigues) in f64 on the host."""
    angle = np.linalg.norm(axis_angle)
    axis = axis_angle / angle
    K = np.array([[0.0, -axis[2], axis[1]], [axis[2], 0.0, -axis[0]], [-axis[1], axis[0], 0.0]])
    return np.eye(3) + K * np.sin(angle) + (K @ K) * (1.0 - np.cos(angle))


_T_PIN = {}


def _to_device(a: np.ndarray, device):
    """A small host array to the device through a per-device pinned staging buffer, without
    blocking the host (the caller's next _reg_accumulate read-back synchronises the stream before
    the buffer is written again)."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return torch.from_numpy(a).to(dev)
    key = (str(dev), a.shape, a.dtype.str)
    buf = _T_PIN.get(key)
    if buf is None:
        buf = _T_PIN[key] = torch.empty(a.shape, dtype=torch.from_numpy(a).dtype, pin_memory=True)
    buf.numpy()[...] = a
    return buf.to(dev, non_blocking=True)


def _solve(acc: np.ndarray, lm_lambda: float, require_cov: bool, require_eigen: bool, device):
    """Normal equations from the kernel accumulators -> (dT 4x4 f64, cov, eigenvalues).
    The weight normalisation w /= 2 mean(w) (utils/tracker.py:394) is the factor
    n / (2 sum w) on N and g.  The 6x6 algebra runs on the host in f64 (the reference's
    torch f64 ops on a 6x6); the results go to the device in one copy each."""
    s_w, s_r, s_wr2, cnt = acc[0], acc[1], acc[2], acc[3]
    scale = cnt / (2.0 * s_w)
    N = np.zeros((6, 6))
    k = 4
    for a in range(6):
        for b in range(a, 6):
            N[a, b] = N[b, a] = acc[k]
            k += 1
    N *= scale
    g = -acc[25:31] * scale
    N_old = N.copy()
    N = N + lm_lambda * np.diag(np.diag(N))
    t = np.linalg.inv(N) @ g
    T_np = np.eye(4)
    T_np[:3, :3] = _expmap_np(t[:3])
    T_np[:3, 3] = t[3:]
    T = _to_device(T_np, device)
    eig = None
    if require_eigen:
        eig = torch.from_numpy(np.linalg.eigvals(N_old[3:, 3:]).real.copy()).to(device)
    cov = None
    if require_cov:
        mse = s_wr2 / (2.0 * s_w)  # mean(w_norm * r^2)
        cov = torch.from_numpy(np.linalg.inv(N_old) * mse).to(device)
    return T, cov, eig


def implicit_reg(points, sdf_grad, sdf_residual, weight, lm_lambda=0.0, require_cov=False, require_eigen=False):
    """utils/tracker.py:468-520 on pre-filtered rows with given weights (HIP accumulation,
    f64 6x6 solve).  Returns (T, cov_mat, eigenvalues)."""
    _lib.require_device(points)
    p = points.detach().to(torch.float32).contiguous()
    g = sdf_grad.detach().to(torch.float32).contiguous()
    r = sdf_residual.detach().to(torch.float32).contiguous().view(-1)
    w = weight.detach().to(torch.float32).contiguous().view(-1)
    acc = _reg_accumulate(p, r, g, None, None, None, w, _lib.PinRegParams())
    # the caller's weights are already normalised: undo the kernel-side n/(2 sum w) factor
    a = acc.copy()
    a[4:] *= 2.0 * a[0] / a[3]
    T, cov, eig = _solve(a, lm_lambda, require_cov, require_eigen, points.device)
    if require_cov:
        cov = cov * (2.0 * a[0] / a[3])
    return T, cov, eig


_REG_BUF: dict = {}


_LOOP_BUF = {}


def _loop_buffers(dev, n):
    """The tracking loop's per-point buffers (sdf, grad, nn counts, std, posed points, sorted rows)
    and its two events, one set per (device, stream), grown by 1.25x when a cloud outgrows them:
    a tracking call then allocates nothing.  Calls on one stream are ordered and each ends with a
    host read of its last iteration, so the next call's writes never meet the previous one's."""
    s = _lib.stream(dev)
    key = (str(dev), s.value)
    lb = _LOOP_BUF.get(key)
    if lb is None or lb["cap"] < n:
        cap = max(int(n * 1.25), 1024)
        lb = dict(cap=cap, sdf=torch.empty(cap, dtype=torch.float32, device=dev),
                  grad=torch.empty((cap, 3), dtype=torch.float32, device=dev),
                  nn=torch.empty(cap, dtype=torch.int32, device=dev),
                  std=torch.empty(cap, dtype=torch.float32, device=dev),
                  cur=torch.empty((cap, 3), dtype=torch.float32, device=dev),
                  q4=torch.empty((cap, 4), dtype=torch.float32, device=dev),
                  events=(torch.cuda.Event(), torch.cuda.Event()))
        _LOOP_BUF[key] = lb
    return lb


def _reg_buffers(dev):
    """Buffers reused every step, one set per (device, stream): the reduction workspace (with
    pin_reg_step's last-block ticket), the accumulators + status record (one D2H copy), delta_T
    and two pose slots (the loop ping-pongs between them), and the pinned host mirrors.  Within a
    stream, launches are ordered and the host read in _register / _RegLoop.result synchronises, so
    reuse is safe; registrations on another stream (e.g. a loop-closure registration on a side
    stream) get their own set, so they never share the ticket counter or the partials."""
    s = _lib.stream(dev) if torch.device(dev).type == "cuda" else None
    key = (str(dev), s.value if s is not None else None)
    if key not in _REG_BUF:
        W = _lib.REG_WORKSPACE_DOUBLES
        n = W + _lib.REG_NACC + _lib.REG_NSTATUS + 16 * 3
        buf = torch.empty(n, dtype=torch.float64, device=dev)
        buf[W - 8:W].zero_()   # pin_reg_step's counter word (left zero by every call)
        host = torch.empty(_lib.REG_NACC + _lib.REG_NSTATUS, dtype=torch.float64, pin_memory=buf.is_cuda)
        host2 = torch.empty((2, _lib.REG_NACC + _lib.REG_NSTATUS + 16), dtype=torch.float64, pin_memory=buf.is_cuda)
        o = W + _lib.REG_NACC + _lib.REG_NSTATUS
        _REG_BUF[key] = dict(ws=buf[:W], acc_status=buf[W:o], acc_status_dT=buf[W:o + 16], acc=buf[W:W + _lib.REG_NACC],
                             status=buf[W + _lib.REG_NACC:o], dT=buf[o:o + 16].view(4, 4),
                             poses=(buf[o + 16:o + 32].view(4, 4), buf[o + 32:o + 48].view(4, 4)), host=host,
                             host2=host2, flip=0)
    return _REG_BUF[key]


def _reg_accumulate(points, sdf, grad, nn_count, sdf_std, label, weight, prm, valid_out=None):
    """pin_reg_normal_eq; the accumulators copied to the host (implicit_reg's pre-weighted form)."""
    b = _reg_buffers(points.device)
    _lib.call("pin_reg_normal_eq", _lib.ptr(points), _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn_count),
              _lib.ptr(sdf_std), _lib.ptr(label), _lib.ptr(weight), points.shape[0], prm, _lib.ptr(b["ws"]),
              _lib.ptr(b["acc"]), _lib.ptr(valid_out), _lib.stream())
    h = b["host"][:_lib.REG_NACC]
    h.copy_(b["acc"])
    return h.numpy().copy()


_LOOP_SORT_MIN = 16384   # tracking loops over at least this many points process them tile-sorted
_PIPELINE = os.environ.get("PIN_TRACK_PIPELINE", "1") != "0"   # 0: one _register call (and host read) per iteration


class _RegLoop:
    """One ``tracking`` call's registration iterations, bound once: the views, the outputs and the
    launch record (PinRegIter) are built in the constructor, so an iteration is ONE native call
    (pin_reg_iteration: pose, query, normal equations, solve, asynchronous copy of the 55-double
    record to pinned host memory) and one event record.

    - Tile order: where the grid backend serves the query and the cloud is large enough, iteration
      0 tile-sorts the posed cloud and later iterations re-pose the SORTED rows in place: the
      points move by the pose increment only, so the order stays a good locality order, and the
      sort's two launches are paid once per call.  The normal equations read the sorted rows.
    - Lookahead: iteration i + 1 is enqueued before the host waits for iteration i (its pose is
      iteration i's device output), so the GPU does not idle through the host's read and
      decision.  Poses ping-pong between two device slots and records between two pinned host
      slots: iteration i + 1 writes neither of iteration i's."""

    def __init__(self, tracker, src, labels, min_grad_norm, max_grad_norm, GM_dist, GM_grad, lm_lambda, init_pose):
        nm, cfg = tracker.neural_points, tracker.config
        self.n = n = src.shape[0]
        dev = src.device
        wf = bool(cfg.weighted_first)
        nn_k = int(cfg.query_nn_k)
        self.hv, self.pv = nm._views("local", True)
        self.mv = mlp_view(tracker.geo_decoder, packed=True)
        self.gv = nm.grid_view("local", True) if nm.backend() == "grid" else None
        sorted_ = self.gv is not None and n >= _LOOP_SORT_MIN and _query._TILE_QUERIES
        lb = _loop_buffers(dev, n)   # per-point outputs: reused views, nothing escapes the loop
        self.sdf = lb["sdf"][:n]
        self.grad = lb["grad"][:n]
        self.nn = lb["nn"][:n]
        self.std = None if wf else lb["std"][:n]
        self.cur = lb["cur"][:n]
        self.q4 = lb["q4"][:n] if sorted_ else None
        self.ws = order_workspace(n, dev) if sorted_ else None
        self.src, self.labels = src, labels   # kept alive with the launch record
        prm = _lib.PinRegParams(min_nn_count=nn_k, min_grad_norm=float(min_grad_norm),
                                max_grad_norm=float(max_grad_norm),
                                max_sdf_std=float(cfg.surface_sample_range_m * cfg.max_sdf_std_ratio),
                                gm_dist=float(GM_dist) if GM_dist is not None else 0.0,
                                gm_grad=float(GM_grad) if GM_grad is not None else 0.0,
                                div_grad_norm=int(bool(getattr(cfg, "reg_dist_div_grad_norm", False))),
                                q4_points=int(sorted_))
        b = self.b = _reg_buffers(dev)
        self.pose0 = init_pose.contiguous()
        self.events = lb["events"]
        d = lambda t: t.data_ptr() if t is not None else None   # noqa: E731
        self.rec = [_lib.PinRegIter(src=d(src), n=n, labels=d(labels), cur=d(self.cur), q4=d(self.q4),
                                    order_ws=d(self.ws), sdf=d(self.sdf), grad=d(self.grad), nn_count=d(self.nn),
                                    sdf_std=d(self.std), reg_ws=d(b["ws"]), acc_status_dt=d(b["acc_status_dT"]),
                                    host_out=b["host2"][k].data_ptr(), nn_k=nn_k, weighted_first=int(wf),
                                    lm_lambda=float(lm_lambda), prm=prm) for k in range(2)]
        self.a_grid = self.gv.ref() if self.gv is not None else None
        self.a_hash = None if self.gv is not None else self.hv.ref()
        self.a_pose = (_lib.ptr(b["poses"][0]), _lib.ptr(b["poses"][1]))
        self.a_pose0 = _lib.ptr(self.pose0)

    def pose(self, i):
        """The device pose after iteration i."""
        return self.b["poses"][i % 2]

    def enqueue(self, i):
        pose_in = self.a_pose0 if i == 0 else self.a_pose[(i - 1) % 2]
        _lib.call("pin_reg_iteration", self.a_grid, self.a_hash, self.pv.ref(), self.mv.ref(),
                  ctypes.byref(self.rec[i % 2]), int(i == 0), pose_in, self.a_pose[i % 2], _lib.stream())
        self.events[i % 2].record()

    def result(self, i):
        """(accumulators [31], status [8], delta pose [4,4]) of iteration i, on the host (waits for it)."""
        self.events[i % 2].synchronize()
        h = self.b["host2"][i % 2].numpy()
        o = _lib.REG_NACC + _lib.REG_NSTATUS
        return h[:_lib.REG_NACC].copy(), h[_lib.REG_NACC:o].copy(), h[o:].reshape(4, 4).copy()


def transform_points(points: torch.Tensor, pose: torch.Tensor) -> torch.Tensor:
    """transform_torch (utils/tools.py:386-399) as one launch (pin_transform_points): f32 points
    [N,3] under a [4,4] pose (f64 on the device)."""
    p = points.detach().to(torch.float32).contiguous()
    _lib.require_device(p)
    T = pose.detach().to(device=p.device, dtype=torch.float64).contiguous()
    out = torch.empty_like(p)
    _lib.call("pin_transform_points", _lib.ptr(p), p.shape[0], _lib.ptr(T), _lib.ptr(out), _lib.stream())
    return out


class Tracker:

    def __init__(self, config, neural_points, geo_decoder, sem_decoder=None, color_decoder=None, group=None):
        """group (a torch.distributed group of W > 1 ranks, optional): every registration step
        splits the source points into W contiguous chunks, each rank queries its chunk and the
        31 normal-equation accumulators are SUM all-reduced before the solve (one
        exchange step); every rank then takes the same pose."""
        self.group = group
        self.config = config
        self.silence = config.silence
        self.neural_points = neural_points
        self.geo_decoder = geo_decoder
        self.sem_decoder = sem_decoder
        self.color_decoder = color_decoder
        self.device = config.device
        self.dtype = config.dtype
        self.sdf_scale = config.logistic_gaussian_ratio * config.sigma_sigmoid_m

    # ------------------------------------------------------------------ utils/tracker.py:39-174
    def tracking(self, source_points, init_pose=None, source_colors=None, source_normals=None,
                 source_semantics=None, source_sdf=None, cur_ts=None, loop_reg: bool = False,
                 vis_result: bool = False):
        """The registration loop with the pose kept on the device: per iteration one transform
        launch, the fused query, the normal equations and their solve (pin_reg_solve, which also
        applies T = dT T and measures dT for the convergence test), then ONE host read of a
        39-double record that drives the reference's control flow (:92-159)."""
        cfg = self.config
        dev = torch.device(self.device) if not torch.is_tensor(source_points) else source_points.device
        T = torch.eye(4, dtype=torch.float64, device=dev) if init_pose is None else \
            init_pose.to(device=dev, dtype=torch.float64)
        cov_mat = None
        min_grad_norm = cfg.reg_min_grad_norm
        max_grad_norm = cfg.reg_max_grad_norm
        cur_GM_dist_m = cfg.reg_GM_dist_m if cfg.reg_GM_dist_m > 0 else None
        cur_GM_grad = cfg.reg_GM_grad if cfg.reg_GM_grad > 0 else None
        lm_lambda = cfg.reg_lm_lambda
        iter_n = cfg.reg_iter_n
        term_thre_deg = cfg.reg_term_thre_deg
        term_thre_m = cfg.reg_term_thre_m
        max_valid_final_sdf_residual_cm = cfg.surface_sample_range_m * 0.5 * 100.0
        min_valid_ratio = 0.2
        if loop_reg:
            max_valid_final_sdf_residual_cm = cfg.surface_sample_range_m * 0.6 * 100.0
            min_valid_ratio = 0.15
        max_increment_sdf_residual_ratio = 1.1
        eigenvalue_ratio_thre = 0.01
        min_valid_points = 30
        converged = False
        valid_flag = True
        last_sdf_residual_cm = 1e5
        source_point_count = source_points.shape[0]
        src = source_points.detach().to(torch.float32).contiguous()
        labels = None if source_sdf is None else source_sdf.detach().to(torch.float32).contiguous()
        weight_point_cloud = None
        eigenvalues = None
        sdf_residual_cm = 0.0
        valid_point_count = 0
        loop = None
        if _PIPELINE and self._shard_range(source_point_count)[2] == 1 and dev.type == "cuda" and source_normals is None:
            loop = _RegLoop(self, src, labels, min_grad_norm, max_grad_norm, cur_GM_dist_m, cur_GM_grad, lm_lambda, T)
            loop.enqueue(0)
        launched = 0
        self.last_iterations = 0
        self.last_status = "ok"   # or the reference's failure message (its prints stay under silence)
        for i in range(iter_n):
            want_stats = vis_result and converged
            if loop is not None:
                # one iteration ahead of the host: i + 1 runs while the host reads i, unless i is
                # known to be the last (converged at i - 1, or the iteration budget)
                if i + 1 < iter_n and not converged and launched < i + 1:
                    loop.enqueue(i + 1)
                    launched = i + 1
                acc, st, dT = loop.result(i)
                T = loop.pose(i)                                              # :115, T = dT @ T
                r = dict(eig=None, cov=None)
                if want_stats and st[4] > 0:
                    _, r["cov"], r["eig"] = _solve(acc, lm_lambda, True, True, dev)
            else:
                cur_points = transform_points(src, T)
                r = self._register(cur_points, source_normals, labels, min_grad_norm, max_grad_norm, cur_GM_dist_m,
                                   cur_GM_grad, lm_lambda, want_stats, pose_in=T)
                T = r["pose"]                                                 # :115, T = dT @ T
                st = r["status"]
                dT = r["delta"]
            self.last_iterations = i + 1
            self._iteration_done(i, dT, st)
            valid_point_count = int(st[0])
            sdf_residual_cm = float(st[1]) if st[4] > 0 else 0.0
            eigenvalues = r["eig"]
            cov_mat = r["cov"]
            if (sdf_residual_cm - last_sdf_residual_cm) / last_sdf_residual_cm > max_increment_sdf_residual_ratio:
                if not self.silence:
                    print("(Warning) registration failed: wrong optimization")
                valid_flag = False
                self.last_status = "wrong optimization"
            else:
                last_sdf_residual_cm = sdf_residual_cm
            if valid_point_count < min_valid_points or 1.0 * valid_point_count / source_point_count < min_valid_ratio:
                if not self.silence:
                    print("(Warning) registration failed: not enough valid points")
                valid_flag = False
                self.last_status = "not enough valid points"
            if not valid_flag or converged:
                break
            rot_angle_deg, tran_m = float(st[2]), float(st[3])                # :132-133, from the solve
            if abs(rot_angle_deg) < term_thre_deg and tran_m < term_thre_m or i == iter_n - 2:
                converged = True
        T = T.clone()    # the loop's pose lives in a reused slot
        if sdf_residual_cm > max_valid_final_sdf_residual_cm:
            if not self.silence:
                print("(Warning) registration failed: too large final residual")
            valid_flag = False
            self.last_status = "too large final residual"
        if eigenvalues is not None:
            min_eigenvalue = torch.min(eigenvalues).item()
            if cfg.eigenvalue_check and min_eigenvalue < valid_point_count * eigenvalue_ratio_thre:
                if not self.silence:
                    print("(Warning) registration failed: eigenvalue check failed")
                valid_flag = False
                self.last_status = "eigenvalue check failed"
        if cov_mat is not None:
            cov_mat = cov_mat.detach().cpu().numpy()
        # diagnostics of the last call (not part of the reference's return): the optimised pose
        # before a failed check replaces it with the initial guess, and the final residual
        self.last_pose, self.last_residual_cm = T, sdf_residual_cm
        if not valid_flag:
            T = init_pose
            cov_mat = None
        return T, cov_mat, weight_point_cloud, valid_flag

    def _iteration_done(self, i, delta, status):
        """Called once per registration iteration of ``tracking`` with its delta pose (host
        ndarray or device tensor [4,4]) and status record; a no-op (a hook for tests/tools)."""

    # ------------------------------------------------------------------ utils/tracker.py:176-275
    def query_source_points(self, coord, ts, bs, query_sdf=True, query_sdf_grad=True, query_color=False,
                            query_color_grad=False, query_sem=False, query_mask=True, query_certainty=True,
                            query_locally=True, mask_min_nn_count: int = 4):
        """Returns (sdf_pred, sdf_grad, color_pred, color_grad, sem_pred, mc_mask, certainty, sdf_std).
        One fused launch covers all points (the reference's bs batching is a memory bound, not a
        semantic one)."""
        if query_color or query_color_grad or query_sem:
            raise NotImplementedError("colour / semantic heads are out of scope")
        sdf, grad, nn, cert, std = fused_query_sdf(self.neural_points, self.geo_decoder, coord, query_locally=query_locally,
                                             want_grad=query_sdf_grad, want_std=True, want_certainty=query_certainty)
        mc_mask = nn >= mask_min_nn_count if query_mask else None
        if not query_sdf:
            sdf, std = None, None
        return sdf, grad, None, None, None, mc_mask, cert, std

    # ------------------------------------------------------------------ utils/tracker.py:277-452
    def _shard_range(self, n):
        """(lo, hi, world) of this rank's chunk of n source points; (0, n, 1) unsharded."""
        group = getattr(self, "group", None)
        if group is None or not dist.is_available() or not dist.is_initialized():
            return 0, n, 1
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        return n * rank // world, n * (rank + 1) // world, world

    def _register(self, pts, normals, labels, min_grad_norm, max_grad_norm, GM_dist, GM_grad, lm_lambda,
                  want_stats, pose_in=None, valid_out=None):
        """query + normal equations + solve of one registration step, all stream-ordered, then one
        host read of accumulators + status.  Returns dict(delta (device f64 [4,4]), pose (dT @
        pose_in, device), status (host [8]), acc (host [31]), cov, eig)."""
        if normals is not None:
            raise NotImplementedError("normal-consistency weights are not used by any reference config")
        cfg = self.config
        lo, hi, world = self._shard_range(pts.shape[0])
        if world > 1:   # this rank's chunk; the accumulators are summed over the ranks below
            pts = pts[lo:hi]
            labels = labels[lo:hi] if labels is not None else None
            valid_out = valid_out[lo:hi] if valid_out is not None else None
        # outputs in tile order where the batch is tile-sorted: the normal equations are a sum over the
        # points, so they read the sorted rows (q4) instead of un-permuting (PIN_QUERY_OUT_TILE)
        sdf, grad, nn, _, std, q4 = fused_query_sdf(self.neural_points, self.geo_decoder, pts, query_locally=True,
                                                    want_grad=True, want_std=not cfg.weighted_first,
                                                    want_certainty=False, out_order="tile")
        max_sdf_std = cfg.surface_sample_range_m * cfg.max_sdf_std_ratio
        prm = _lib.PinRegParams(min_nn_count=int(cfg.query_nn_k), min_grad_norm=float(min_grad_norm),
                                max_grad_norm=float(max_grad_norm), max_sdf_std=float(max_sdf_std),
                                gm_dist=float(GM_dist) if GM_dist is not None else 0.0,
                                gm_grad=float(GM_grad) if GM_grad is not None else 0.0,
                                div_grad_norm=int(bool(getattr(cfg, "reg_dist_div_grad_norm", False))),
                                q4_points=int(q4 is not None))
        if cfg.weighted_first:
            std = None  # reference: sdf_std stays 0 < max_sdf_std
        b = _reg_buffers(pts.device)
        s = _lib.stream()
        _lib.call("pin_reg_normal_eq", _lib.ptr(pts if q4 is None else q4), _lib.ptr(sdf), _lib.ptr(grad), _lib.ptr(nn),
                  _lib.ptr(std),
                  _lib.ptr(labels), None, pts.shape[0], ctypes.byref(prm), _lib.ptr(b["ws"]), _lib.ptr(b["acc"]),
                  _lib.ptr(valid_out), s)
        if world > 1:
            all_reduce(b["acc"], group=getattr(self, "group", None))   # 31 doubles: a sharded step's one exchange
        pose_out = None
        if pose_in is not None:
            b["flip"] ^= 1
            pose_out = b["poses"][b["flip"]]
            pin = pose_in if pose_in.is_contiguous() else pose_in.contiguous()
        _lib.call("pin_reg_solve", _lib.ptr(b["acc"]), float(lm_lambda), _lib.ptr(pin) if pose_in is not None else None,
                  _lib.ptr(b["dT"]), _lib.ptr(pose_out), _lib.ptr(b["status"]), s)
        host = b["host"]
        host.copy_(b["acc_status"])          # the step's one synchronisation
        h = host.numpy()
        acc, status = h[:_lib.REG_NACC].copy(), h[_lib.REG_NACC:].copy()
        cov = eig = None
        if want_stats and status[4] > 0:
            _, cov, eig = _solve(acc, lm_lambda, True, True, pts.device)
        return dict(delta=b["dT"], pose=pose_out, status=status, acc=acc, cov=cov, eig=eig)

    def registration_step(self, points, normals, sdf_labels, colors, cur_ts, min_grad_norm, max_grad_norm,
                          GM_dist=None, GM_grad=None, lm_lambda=0.0, vis_weight_pc=False):
        """utils/tracker.py:277-452 -> (delta_T, cov_mat, eigenvalues, None, valid_points,
        sdf_residual_cm, None).  valid_points keeps the source order."""
        if colors is not None and getattr(self.config, "photometric_loss_on", False):
            raise NotImplementedError("photometric registration is out of scope")
        pts = points.detach().to(torch.float32).contiguous()
        labels = sdf_labels.detach().to(torch.float32).contiguous() if sdf_labels is not None else None
        valid = torch.empty(pts.shape[0], dtype=torch.uint8, device=pts.device)
        r = self._register(pts, normals, labels, min_grad_norm, max_grad_norm, GM_dist, GM_grad, lm_lambda,
                           vis_weight_pc, valid_out=valid)
        lo, hi, world = self._shard_range(pts.shape[0])
        if world > 1:   # every rank's chunk of the validity mask, for the valid points of the whole cloud
            n = pts.shape[0]
            m = max(n * (k + 1) // world - n * k // world for k in range(world))
            mine = torch.zeros(m, dtype=torch.uint8, device=pts.device)
            mine[:hi - lo] = valid[lo:hi]
            group = getattr(self, "group", None)
            host = dist.get_backend(group) == "gloo" and mine.is_cuda
            src = mine.cpu() if host else mine
            parts = [torch.empty_like(src) for _ in range(world)]
            dist.all_gather(parts, src, group=group)
            for k, part in enumerate(parts):
                a, z = n * k // world, n * (k + 1) // world
                valid[a:z] = part[:z - a].to(valid.device)
        cnt = int(r["status"][0])
        # the count is on the host already: gather the valid rows without another sync
        valid_points = points[torch.nonzero_static(valid, size=cnt).squeeze(1)]
        if cnt < 10:
            T = torch.eye(4, device=points.device, dtype=torch.float64)
            return T, None, None, None, valid_points, 0.0, 0.0
        return r["delta"].clone(), r["cov"], r["eig"], None, valid_points, float(r["status"][1]), None
