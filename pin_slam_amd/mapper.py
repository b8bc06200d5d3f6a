"""Drop-in for the training path of utils/mapper.py:Mapper.

``mapping(iter_count)`` (utils/mapper.py:425-593) runs each iteration as three HIP launches
(+ the Adam launches) instead of the reference's autograd graph:

  pin_train_forward   batch rows + numerical-gradient stencil rows, training-mode
                      query_feature (certainty / ts side effects) + Decoder.sdf
  pin_train_backward  BCE + eikonal gradients, decoder backward, feature-gradient scatter,
                      decoder-parameter gradients (only while the decoder is trainable)
  pin_adam_step       torch.optim.Adam (fresh state per mapping() call, tools.py:89-116)

and finishes with ``assign_local_to_global`` (neural_points.py:315-324) like the reference.

Data parallel: with a process group of W > 1 ranks, every rank draws
its own batch, the per-rank gradients are scaled by 1/W inside the backward and SUM
all-reduced (RCCL over xGMI on ROCm), so every rank applies the same Adam step to its replica
of the map.  Certainty deltas (SUM) and ts_update (MAX) are reconciled once at the end of
mapping(): nothing inside an iteration reads them.

``sdf`` and ``get_numerical_gradient`` mirror utils/mapper.py:670-733 on the autograd-capable
drop-in query_feature for callers outside the fused loop.
"""
import ctypes
import os
import warnings

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .data_sampler import DataSampler
from .query import _MLP_PACK, _TILE_MIN, _TILE_QUERIES, mlp_view, mlp_view_repacked, query_sdf, query_sort
from .sharding import OwnerAdam, all_reduce

# weighted_first with a training decoder: decode each row in the backward on the matrix cores
# (PIN_TRAIN_ROW_DECODE=0: the f32 VALU decoder backward, for A/B runs)
_ROW_DECODE = os.environ.get("PIN_TRAIN_ROW_DECODE", "1") != "0"
# training batches from this many rows (batch + stencil) up are tile-sorted before the forward
_TRAIN_TILE_MIN = int(os.environ.get("PIN_TRAIN_TILE_MIN", str(_TILE_MIN)))
# batches below this many rows (batch + stencil) scatter their feature terms into this many replicas
# of the gradient, summed after the backward: a SLAM frame's 26K rows put up to ~65 (row, neighbour)
# pairs on one point, whose memory-side float atomics serialise on its address line
_REPLICA_ROWS = int(os.environ.get("PIN_TRAIN_REPLICA_ROWS", str(1 << 18)))
_REPLICAS = int(os.environ.get("PIN_TRAIN_REPLICAS", "8"))
# batches below this many rows run the forward with two lanes per row (PIN_TRAIN_PAIR)
_PAIR_ROWS = int(os.environ.get("PIN_TRAIN_PAIR_ROWS", str(1 << 17)))
# per-neighbour decoding, frozen decoder: the backward's input gradients from the forward's ReLU
# masks (PIN_TRAIN_DX); PIN_TRAIN_NWF_MASK=0 re-decodes each neighbour in the backward (A/B runs)
_NWF_MASK = os.environ.get("PIN_TRAIN_NWF_MASK", "1") != "0"
# the sample pool also kept as one 32-B record per sample for the batch gather (pin_pool_pack)
_PACK_POOL = os.environ.get("PIN_PACK_POOL", "1") != "0"
# deterministic mode (Mapper(deterministic=True) / config.deterministic): the feature-gradient
# terms and the certainty side effect are summed as 64-bit fixed-point integers
# (PinTrainState.grad_fixed / cert_fixed), the rows tile-sorted stably -- a mapping() call is then
# a function of its inputs and draws, bitwise.  Shifts: the feature gradients in two parts, 2^-50
# (8.9e-16, range +-8192) for terms >= 2^-38 and 2^-90 for smaller ones (fixed_add, pin_train.hip);
# 2^-32 (2.3e-10) and +-2^30 for a call's certainty sums
FIXED_SHIFT = 50
CERT_SHIFT = 32
# the dense loop draws get_batch's rows on the device (pin_train_gather_packed_draw: no draw
# launches) unless _randint is replaced on the instance (the tests' replay hook) or
# Mapper.device_draws is False; PIN_DEVICE_DRAWS=0 turns it off everywhere.  The draws are NOT the
# reference's numbers: its get_batch calls torch.randint on the device (utils/mapper.py:683-711),
# these are SplitMix64 of (seed, iteration, row) -- the same distribution (history rows uniform
# over the pool, new rows uniform over new_idx; test_device_batch_draws), another stream.  The
# seed comes from the device's torch generator (its seed and Philox offset, the offset then
# advanced as the reference's two randint draws per iteration would), so torch.manual_seed still
# fixes a run, no host sync is needed and the CPU generator is left alone (_device_seed).
_DEVICE_DRAWS = os.environ.get("PIN_DEVICE_DRAWS", "1") != "0"
# data-parallel dense loop: the feature gradient reduce-scattered in this many row buckets, each
# rank's piece of a bucket stepped by Adam as soon as it lands and all-gathered (_owner_adam)
_AR_BUCKETS = int(os.environ.get("PIN_AR_BUCKETS", "4"))


def _deterministic_default(config):
    """The mode of a Mapper built without deterministic=: config.deterministic, else the
    PIN_DETERMINISTIC environment switch (also for the reference's Mapper after install())."""
    d = getattr(config, "deterministic", None)
    return os.environ.get("PIN_DETERMINISTIC", "0") == "1" if d is None else bool(d)


def _viewed_elsewhere(t: torch.Tensor) -> bool:
    """True if any tensor other than ``t`` shares t's storage (a view kept by a caller).  A view
    holds its base's storage through its TensorImpl, not through a Python reference to ``t``, so
    the storage's use count is what sees it: 1 for t itself + 1 for the temporary handle here."""
    use_count = getattr(torch._C, "_storage_Use_Count", None)
    if use_count is None:
        return True     # cannot tell: never reuse
    return use_count(t.untyped_storage()._cdata) > 2


def transform_batch_torch(points: torch.Tensor, transformation: torch.Tensor) -> torch.Tensor:
    """utils/tools.py:401-407."""
    points = torch.matmul(transformation[:, :3, :3].to(points), points.unsqueeze(-1)) + \
        transformation[:, :3, 3:].to(points)
    return points.squeeze(-1)


class _TrainBuffers:
    """Per-row buffers of one iteration, reused across iterations and mapping() calls."""

    def __init__(self):
        self.key = None

    def eik(self, rows, nn_k, wf):
        """Analytic-eikonal buffers (PinTrainState.eik_coef / eik_vec), allocated on first use."""
        key = (rows, nn_k, wf, str(self.sdf.device))
        if getattr(self, "_eik_key", None) != key:
            dev = self.sdf.device
            self.eik_coef = torch.empty((rows, nn_k), dtype=torch.float32, device=dev)
            self.eik_vec = torch.empty((rows, 20 if wf else 4), dtype=torch.float32, device=dev)
            self._eik_key = key
        return self.eik_coef, self.eik_vec

    def replicas(self, n_floats, device):
        """Zeroed scratch of n_floats for PinTrainState.grad_replicas (pin_train_backward re-zeroes
        it after every use); re-allocated when too small or more than 4x too large."""
        return self._zeroed("grad_replicas", n_floats, torch.float32, device)

    def fixed(self, n, device):
        """Zeroed int64 scratch for PinTrainState.grad_fixed (the deterministic mode's fixed-point
        replicas, coarse and fine parts; the consumer re-zeroes it)."""
        return self._zeroed("grad_fixed", n, torch.int64, device)

    def cert_fixed(self, n, device):
        """Zeroed int64 scratch for PinTrainState.cert_fixed (folded and re-zeroed by
        pin_fixed_accumulate at the end of the plan)."""
        return self._zeroed("cert_fix", n, torch.int64, device)

    def _zeroed(self, name, n, dtype, device):
        buf = getattr(self, name, None)
        want = max(int(n), 1 << 16)
        if (buf is None or buf.numel() < n or buf.numel() > 4 * want or buf.dtype != dtype
                or buf.device != torch.device(device)):
            buf = torch.zeros((want,), dtype=dtype, device=device)
            setattr(self, name, buf)
        return buf

    def draw_shapes(self, n_hist, new_sel, n_new, device):
        """Placeholder index tensors of a device-drawn batch's sizes (the launch plan is sized from
        them; the draw kernel never reads them)."""
        key = (n_hist, n_new, str(device))
        if getattr(self, "_draw_key", None) != key:
            self._draw_idx = torch.empty((n_hist,), dtype=torch.int64, device=device)
            self._draw_new = torch.empty((n_new,), dtype=torch.int64, device=device)
            self._draw_key = key
        return self._draw_idx, (None if new_sel is None else (new_sel, self._draw_new))

    def get(self, rows, nn_k, wf, device):
        key = (rows, nn_k, wf, str(device))
        if key != self.key:
            D = _lib.FEATURE_DIM + 3
            self.ids = torch.empty((rows, nn_k), dtype=torch.int32, device=device)
            self.weights = torch.empty((rows, nn_k), dtype=torch.float32, device=device)
            self.x = torch.empty((rows, D) if wf else (rows, nn_k, 3), dtype=torch.float32, device=device)
            self.sdf = torch.empty((rows,), dtype=torch.float32, device=device)
            self.rows = torch.empty((rows, 3), dtype=torch.float32, device=device)
            self.rows4 = torch.empty((rows, 4), dtype=torch.float32, device=device)
            self.label = torch.empty((rows,), dtype=torch.float32, device=device)
            self.ts = torch.empty((rows,), dtype=torch.int64, device=device)
            # pin_train_backward's partials: a loss double per wave and a decoder-gradient partial
            # per block, sized for the smallest training block (one wave)
            nblk = (rows + 63) // 64
            self.workspace = torch.empty((nblk * 8 + nblk * _lib.MLP_PART_FLOATS * 4,), dtype=torch.uint8,
                                         device=device)
            self.loss = torch.zeros((1,), dtype=torch.float64, device=device)
            self.wrow = torch.empty((rows,), dtype=torch.float32, device=device)
            # bit 0: a batch index outside the pool (pin_train_gather clamps it); read per mapping()
            self.gather_error = torch.zeros((1,), dtype=torch.int32, device=device)
            self.key = key
        return self


class _StepPlan:
    """The launches of one training iteration (Mapper._step_plan); run() takes the batch's draw."""
    packed = None
    det = False
    fix = None        # deterministic mode, gradient folded by the Adam launch: the fixed-point replicas
    nfix = 0
    cert_fix = None

    def run(self, index, index_new, draw=None):
        """draw (n_hist, new_idx or None, seed, counter): the batch drawn on the device
        (pin_train_gather_packed_draw) instead of from the index tensors."""
        b = self.b
        if draw is not None:
            n_hist, new_sel, seed, ctr = draw
            _lib.check("pin_train_gather_packed_draw", self.f_draw(
                self.packed_ptr, self.packed_rows, n_hist, None if new_sel is None else new_sel.data_ptr(),
                0 if new_sel is None else new_sel.shape[0], seed, ctr, *self.gather_tail))
        elif not self.index_mode:
            _lib.call("pin_train_rows", _lib.ptr(self.q), self.gather_tail[0], self.gather_tail[1], self.s)
        elif self.packed is not None and index_new is not None:
            new_sel, draw = index_new
            _lib.check("pin_train_gather_packed_split", self.f_split(
                self.packed_ptr, self.packed_rows, index.data_ptr(), index.shape[0], new_sel.data_ptr(),
                new_sel.shape[0], draw.data_ptr(), *self.gather_tail))
        elif self.packed is not None:
            _lib.call("pin_train_gather_packed", _lib.ptr(self.packed), int(self.packed.shape[0]), _lib.ptr(index),
                      *self.gather_tail)
        else:
            q, sdf_label, ts, wpool = self.pools
            _lib.call("pin_train_gather", _lib.ptr(q), _lib.ptr(sdf_label), _lib.ptr(ts), _lib.ptr(wpool),
                      int(q.shape[0]), _lib.ptr(index), *self.gather_tail)
        if self.tiled:
            # process the rows tile by tile (pin_query_sort over the batch + stencil coordinates;
            # the deterministic mode keeps the input order inside a tile)
            query_sort(self.gv, b.rows, out=b.rows4, stable=self.det)
        self.mapper._order = b.rows4 if self.tiled else None
        _lib.check("pin_train_forward", self.f_fwd(*self.fwd_args))
        _lib.check("pin_train_backward", self.f_bwd(*self.bwd_args))

    def finish(self):
        """After the last run: the side effects went through raw pointers -- invalidate the caches
        built on them; the loss / sdf of the last iteration."""
        nm = self.mapper.neural_points
        if self.cert_fix is not None:   # the deterministic mode's certainty sums, folded in once
            cert = nm.local_point_certainties
            _lib.call("pin_fixed_accumulate", _lib.ptr(self.cert_fix), 1, cert.numel(), CERT_SHIFT, 1, _lib.ptr(cert),
                      self.s)
        nm.mark_modified(nm.local_point_certainties, nm.local_point_ts_update if self.ts64 is not None else None)
        self.mapper.last_loss = self.b.loss
        self.mapper.last_sdf = self.b.sdf[: self.n]


class Mapper:
    """utils/mapper.py:Mapper -- constructor signature, pools and training entry points."""

    def __init__(self, config, dataset, neural_points, geo_mlp, sem_mlp=None, color_mlp=None, group=None,
                 shard="dense", slab_layout="auto", deterministic=None):
        self.config = config
        self.silence = config.silence
        self.dataset = dataset
        self.neural_points = neural_points
        self.geo_mlp = geo_mlp
        self.sem_mlp = sem_mlp
        self.color_mlp = color_mlp
        self.device = config.device
        self.dtype = config.dtype
        self.used_poses = None
        self.lose_track = False
        # utils/mapper.py:50-54
        self.require_gradient = False
        if config.ekional_loss_on or getattr(config, "proj_correction_on", False) or \
                getattr(config, "consistency_loss_on", False):
            self.require_gradient = True
        if config.numerical_grad and not getattr(config, "proj_correction_on", False) and \
                not getattr(config, "consistency_loss_on", False):
            self.require_gradient = False
        self.total_iter = 0
        self.sdf_scale = config.logistic_gaussian_ratio * config.sigma_sigmoid_m
        self.sampler = DataSampler(config)
        self.ray_sample_count = 1 + config.surface_sample_n + config.free_behind_n + config.free_front_n
        self.new_idx = None
        self.ba_done_flag = False
        self.train_less = False
        dev, dt = self.device, self.dtype
        self.coord_pool = torch.empty((0, 3), device=dev, dtype=dt)
        self.global_coord_pool = torch.empty((0, 3), device=dev, dtype=dt)
        self.sdf_label_pool = torch.empty((0,), device=dev, dtype=dt)
        self.color_pool = None
        self.sem_label_pool = None
        self.normal_label_pool = None
        self.weight_pool = torch.empty((0,), device=dev, dtype=dt)
        self.time_pool = torch.empty((0,), device=dev, dtype=torch.long)
        self.pool_sample_count = 0
        self.group = group
        # data-parallel mode with a group of W > 1: "dense" (every rank samples the whole pool,
        # SUM all-reduce of the [L+1,8] gradient) or "space" (owner-partitioned slabs, halo
        # exchange only: pin_slam_amd.sharding); slab_layout "auto" (2-D cells where the map is
        # wide in both axes) or "1d" (slabs along the longer axis)
        if shard not in ("dense", "space"):
            raise ValueError("shard must be 'dense' or 'space'")
        self.shard = shard
        self.slab_layout = slab_layout
        self.last_loss = None        # device f64 tensor: loss of the last iteration
        # deterministic accumulation (FIXED_SHIFT above); default: config.deterministic, else the
        # PIN_DETERMINISTIC environment switch, else off
        self.deterministic = _deterministic_default(config) if deterministic is None else bool(deterministic)
        self._buf = _TrainBuffers()
        self._adam_t = 0

    # ---------------------------------------------------------------- data pool
    def dynamic_filter(self, points_torch, type_2_on: bool = False):
        """utils/mapper.py:79-108.  Strategy 1: measurements in confidently free space are dynamic.
        Strategy 2 (type_2_on): also dynamic where the SDF's analytic gradient is flat
        (|grad| <= 0.3) at a certain point (certainty >= 0.5) -- the reference's get_gradient of
        sdf_pred w.r.t. the points, here the fused kernel's closed-form gradient.  One fused query
        (local map, SDF + certainty [+ gradient]) instead of query_feature + sdf + autograd."""
        sdf, grad, _, cert, _ = query_sdf(self.neural_points, self.geo_mlp, points_torch, query_locally=True,
                                          want_grad=bool(type_2_on), want_certainty=True)
        c = self.config
        static_mask = (cert < c.dynamic_certainty_thre) | (sdf < c.dynamic_sdf_ratio_thre * c.voxel_size_m)
        if type_2_on:
            min_grad_norm, certainty_thre = 0.3, 0.5            # utils/mapper.py:101-102
            static_mask = static_mask & ((grad.norm(dim=-1) > min_grad_norm) | (cert < certainty_thre))
        return static_mask

    def _used_poses(self):
        """utils/mapper.py:205-211."""
        ds, c = self.dataset, self.config
        if ds is None:
            return self.used_poses
        if getattr(c, "pgo_on", False):
            return self._poses_dev(ds.pgo_poses)
        if getattr(c, "track_on", False):
            return self._poses_dev(ds.odom_poses)
        if getattr(ds, "gt_pose_provided", False):
            return self._poses_dev(ds.gt_poses)
        return self.used_poses

    def _poses_dev(self, poses):
        """torch.tensor(np.array(poses), f64) on the device, copied from pinned memory without
        waiting (a pageable copy drains the stream: one host wait per frame for a few KB)."""
        a = torch.from_numpy(np.array(poses, dtype=np.float64))
        if torch.device(self.device).type != "cuda":
            return a.to(self.device)
        return a.pin_memory().to(self.device, non_blocking=True)

    def process_frame(self, point_cloud_torch, frame_label_torch, cur_pose_torch, frame_id: int,
                      filter_dynamic: bool = False, draws=None):
        """utils/mapper.py:110-321: sample the frame's rays (one fused launch, samples in the sensor
        and the world frame), grow the neural-point map with the near-surface samples, append to
        the data pool, window-filter the pool every pool_filter_freq frames and mark the new,
        uncertain near-surface samples (query_certainty) for get_batch.  ``draws`` replays given
        sampler draws (tests)."""
        c = self.config
        frame_origin = cur_pose_torch[:3, 3]
        frame_orientation = cur_pose_torch[:3, :3]
        frame_point = point_cloud_torch[:, :3]
        self.static_mask = torch.ones(frame_point.shape[0], dtype=torch.bool, device=self.device)
        if filter_dynamic:                                                               # :124-131
            from .tracker import transform_torch
            self.static_mask = self.dynamic_filter(transform_torch(frame_point, cur_pose_torch))
            frame_point = frame_point[self.static_mask]
        frame_color = None
        if getattr(c, "color_on", False):
            frame_color = point_cloud_torch[:, 3:]
            if filter_dynamic:
                frame_color = frame_color[self.static_mask]
        if frame_label_torch is not None and filter_dynamic:
            frame_label_torch = frame_label_torch[self.static_mask]
        coord, sdf_label, normal_label, sem_label, color_label, weight, global_coord = self.sampler.sample(
            frame_point, None, frame_label_torch, frame_color, pose=cur_pose_torch, draws=draws)   # :149-151
        self.cur_sample_count = sdf_label.shape[0]
        self.pool_sample_count = self.sdf_label_pool.shape[0]
        sig_before = self._pool_signature() if self.global_coord_pool is not None else None
        # :185-188 first (the reference appends after the map update; the pools do not depend on
        # it): the appends are device copies with no host read, so they run while the host works
        # through the update's launches and count reads.  Appended into growable buffers (same
        # contents as the reference's torch.cat, without reallocating and copying the whole pool
        # every frame)
        self.coord_pool = self._pool_append("coord", self.coord_pool, coord)
        self.weight_pool = self._pool_append("weight", self.weight_pool, weight)
        self.sdf_label_pool = self._pool_append("sdf_label", self.sdf_label_pool, sdf_label)
        m_new, fid = coord.shape[0], int(frame_id)
        self.time_pool = self._pool_append("time", self.time_pool, None,
                                           fill=(m_new, torch.long, lambda v: v.fill_(fid)))
        time_repeat = self.time_pool[self.time_pool.shape[0] - m_new:]   # torch.full((m,), frame_id)
        self.sem_label_pool = None if sem_label is None else (
            sem_label if self.sem_label_pool is None else self._pool_append(
                "sem", self.sem_label_pool, sem_label.to(self.sem_label_pool.dtype)))
        self.color_pool = None if color_label is None else (
            color_label if self.color_pool is None else self._pool_append("color", self.color_pool, color_label))
        if getattr(c, "from_sample_points", True):                                       # :163-171
            if getattr(c, "from_all_samples", False):
                update_points = coord
            else:   # transform of the selected rows == the selected rows of the transform (row-wise)
                update_points = global_coord[torch.abs(sdf_label) < c.surface_sample_range_m * c.map_surface_ratio, :]
        else:
            from .tracker import transform_torch
            update_points = transform_torch(frame_point, cur_pose_torch)
        if getattr(c, "prune_map_on", False):                                            # :174-176
            if self.neural_points.prune_map(c.max_prune_certainty):
                self.neural_points.recreate_hash(None, None, True, True, frame_id)
        self.neural_points.update(update_points, frame_origin, frame_orientation, frame_id)   # :177
        self.normal_label_pool = None
        self.used_poses = self._used_poses()                                             # :205-211
        if self.ba_done_flag:                                                            # :214-217
            self.global_coord_pool = transform_batch_torch(self.coord_pool, self.used_poses[self.time_pool])
            self.ba_done_flag = False
        else:
            self.global_coord_pool = self._pool_append("global_coord", self.global_coord_pool, global_coord)
        # the packed records follow the pools: the new samples packed and appended (a stale or
        # missing packed pool is left for _packed_pool to rebuild in one pass)
        track = _PACK_POOL and self.__dict__.get("_pool_packed") is not None and sig_before is not None \
            and self.__dict__.get("_pool_packed_sig") == sig_before and self._pools_fusable()
        if track:
            self._pool_packed = self._pool_append(
                "packed", self._pool_packed, None,
                fill=(m_new, torch.float32, lambda v: self._pack(global_coord, sdf_label, time_repeat, weight, out=v)))
        if (frame_id + 1) % int(c.pool_filter_freq) == 0:                                # :226-262
            # the sphere test, the kept-row list and both counts in one pass (pin_pool_window),
            # one host read for the counts; the origin keeps the pose's dtype (torch promotes the
            # f32 pool against an f64 pose)
            pool = self.global_coord_pool
            n_pool = pool.shape[0]
            origin = frame_origin.detach()
            f64 = origin.dtype == torch.float64
            origin = origin.to(device=pool.device, dtype=torch.float64 if f64 else torch.float32).contiguous()
            keep_all, counts, ws, mask_buf = self._window_buffers(n_pool, pool.device)
            tail_start = n_pool - self.cur_sample_count if self.cur_sample_count > 0 else 0   # [-0:] is all
            _lib.call("pin_pool_window", _lib.ptr(pool.contiguous()), n_pool, _lib.ptr(origin), int(f64),
                      float(c.window_radius) ** 2, tail_start, _lib.ptr(keep_all), _lib.ptr(counts),
                      _lib.ptr(ws), _lib.stream())
            pool_sample_count, cur_kept = (int(v) for v in counts.cpu().tolist())
            keep = keep_all[:pool_sample_count]
            if pool_sample_count > c.pool_capacity:
                # the reference's random discards over the kept rows (:241-245), then the mask's rows
                discard_count = pool_sample_count - int(c.pool_capacity)
                discarded_index = self._randint(pool_sample_count, discard_count)
                filter_mask = mask_buf[:n_pool]
                filter_mask.zero_()
                filter_mask[keep] = True
                filter_mask[keep[discarded_index]] = False
                keep = torch.nonzero(filter_mask).squeeze(1)
                cur_kept = int(filter_mask[-self.cur_sample_count:].sum().item())
            # every pool compacted by the kept-row list in one launch (pin_gather_rows)
            names = ["coord", "global_coord", "sdf_label", "weight", "time"] + (["packed"] if track else []) + \
                (["sem"] if sem_label is not None else []) + (["color"] if color_label is not None else [])
            attrs = {"coord": "coord_pool", "global_coord": "global_coord_pool", "sdf_label": "sdf_label_pool",
                     "weight": "weight_pool", "time": "time_pool", "packed": "_pool_packed",
                     "sem": "sem_label_pool", "color": "color_pool"}
            outs = self._pool_compact_many([(nm_, getattr(self, attrs[nm_])) for nm_ in names], keep)
            for nm_, out in zip(names, outs):
                setattr(self, attrs[nm_], out)
            # :256-259 -- the kept rows of this frame's samples (filter_mask[-cur:]: all rows when
            # cur is 0) and of the whole pool
            self.cur_sample_count = cur_kept
            self.pool_sample_count = int(keep.shape[0])
        else:
            self.cur_sample_count = coord.shape[0]
            self.pool_sample_count = self.coord_pool.shape[0]
        if track:
            self._pool_packed_sig = self._pool_signature()
        if int(getattr(c, "bs_new_sample", 0)) > 0:                                      # :269-304
            cur = self.global_coord_pool[-self.cur_sample_count:]
            cur_label = self.sdf_label_pool[-self.cur_sample_count:]
            nm = self.neural_points
            nm.set_search_neighborhood(num_nei_cells=1, search_alpha=0.0)
            cert = nm.query_certainty(cur) if cur.shape[0] > 0 else torch.zeros(0, device=self.device)
            nm.set_search_neighborhood(num_nei_cells=c.num_nei_cells, search_alpha=c.search_alpha)
            self.new_idx = torch.where((cert < c.new_certainty_thre) &
                                       (torch.abs(cur_label) < c.surface_sample_range_m * 3.0))[0]
            self.new_idx += (self.pool_sample_count - self.cur_sample_count)
            new_sample_count = self.new_idx.shape[0]
            self.train_less = bool(getattr(c, "adaptive_mode", False) and
                                   new_sample_count / max(self.cur_sample_count, 1) < c.new_sample_ratio_thre)

    def _window_buffers(self, n, device):
        """The window filter's kept-row list, counts and workspace for a pool of n rows: sized with
        the pool buffers (_pool_append) so that the filter allocates nothing in steady state (a
        first-time workspace allocation inside the filter frame took ~20 ms at 11M rows)."""
        wb = self.__dict__.get("_window_bufs")
        if wb is None or wb[0].shape[0] < n or wb[0].device != torch.device(device):
            rows = max(int(n), 1)
            wb = (torch.empty((rows,), dtype=torch.int64, device=device),
                  torch.empty((2,), dtype=torch.int64, device=device),
                  torch.empty((int(_lib.fn("pin_pool_window_workspace_bytes")(rows)),), dtype=torch.uint8,
                              device=device),
                  torch.empty((rows,), dtype=torch.bool, device=device))   # the capacity discards' mask
            self._window_bufs = wb
        return wb

    def _pool_rows_hint(self, m):
        """Rows a pool buffer is first sized for: the window filter keeps at most pool_capacity
        samples and up to pool_filter_freq frames of m samples arrive between two filters, so
        buffers of this size never grow in steady state (a few hundred MB of HBM per pool)."""
        c = getattr(self, "config", None)
        if c is None:
            return 0
        return int(getattr(c, "pool_capacity", 0)) + int(getattr(c, "pool_filter_freq", 1)) * m * 5 // 4

    def _pool_append(self, name, cur, new, fill=None):
        """torch.cat((cur, new)) as a prefix view of a buffer sized once for the steady-state pool
        (grown by 1.5x if ever full); cur must be the previous return value to be appended in
        place (anything else is copied once).  fill=(m, dtype, fn) instead of new: m rows of that
        dtype, written by fn(view of the appended rows) (no temporary and copy)."""
        bufs = self.__dict__.setdefault("_pool_bufs", {})
        buf, last = bufs.get(name, (None, -1))
        n = cur.shape[0]
        m = new.shape[0] if fill is None else int(fill[0])
        dt = torch.promote_types(cur.dtype, new.dtype if fill is None else fill[1])   # torch.cat's promotion
        dev = new.device if fill is None else cur.device
        # in place only when cur IS the view returned last time: a shorter prefix view (a
        # truncated pool) still references the rows past it, so it gets a fresh buffer
        in_place = (buf is not None and n == last and buf.dtype == dt and buf.shape[1:] == cur.shape[1:]
                    and buf.shape[0] >= n + m and (n == 0 or cur.data_ptr() == buf.data_ptr())
                    and cur.is_contiguous())
        if not in_place:
            rows = max(int((n + m) * 1.5), 1024, self._pool_rows_hint(m))
            nb = torch.empty((rows,) + tuple(cur.shape[1:]), dtype=dt, device=dev)
            nb[:n] = cur
            buf = nb
            # the window filter's compaction target, sized alike now rather than at the first
            # filter (a first-time allocation of every pool there stalled that frame ~150 ms)
            spares = self.__dict__.setdefault("_pool_spare", {})
            sp = spares.get(name)
            if sp is None or sp.shape[0] < rows or sp.dtype != dt or sp.shape[1:] != nb.shape[1:]:
                spares[name] = torch.empty_like(nb)
            if name == "global_coord" and dev.type == "cuda":   # the window filter's buffers, sized alike
                self._window_buffers(rows, dev)
        if fill is None:
            buf[n:n + m] = new
        elif m > 0:
            fill[2](buf[n:n + m])
        bufs[name] = (buf, n + m)
        return buf[:n + m]

    def _pool_compact_many(self, pools, keep):
        """_pool_compact of several pools by one kept-row list: the targets taken as
        _pool_compact takes them, then every row copy in one pin_gather_rows launch.  pools:
        [(name, tensor)]; returns the compacted views in that order."""
        k = keep.shape[0]
        keep = keep.contiguous()
        outs, arrays = [], []
        # every source the launches read stays referenced until they are queued: a contiguous()
        # copy of a non-contiguous pool held only by the loop variable would go back to the caching
        # allocator at the next iteration, which could hand its block to the next spare before the
        # gather has read it
        srcs = []
        for name, cur in pools:
            out = self._pool_compact_target(name, cur, k)
            outs.append(out)
            if k > 0 and cur.numel() > 0:
                cur = cur.contiguous()
                srcs.append(cur)
                arrays.append(_lib.PinRowArray(cur.data_ptr(), out.data_ptr(),
                                               cur.numel() // cur.shape[0] * cur.element_size()))
        for i in range(0, len(arrays), _lib.ROW_ARRAYS_MAX):
            chunk = arrays[i:i + _lib.ROW_ARRAYS_MAX]
            arr = (_lib.PinRowArray * len(chunk))(*chunk)
            _lib.call("pin_gather_rows", arr, len(chunk), _lib.ptr(keep), k, _lib.stream())
        del srcs   # the launches are queued (stream order keeps a freed block from reuse before them)
        return outs

    def _pool_compact(self, name, cur, keep):
        """One pool compacted by the kept-row list (_pool_compact_many of one pool)."""
        return self._pool_compact_many([(name, cur)], keep)[0]

    def _pool_compact_target(self, name, cur, k):
        """cur.index_select(0, keep) written into the pool's spare buffer (kept per pool and
        swapped with the live one), so the window filter allocates nothing in steady state; the
        result is the pool's new live prefix view, which _pool_append then extends in place.
        The spare is the live buffer of the previous filter: a pool tensor a caller kept from
        before that filter is a view of it, so a spare whose storage has any view besides the
        spare itself is left alone (a fresh buffer is taken) and the kept tensor stays valid."""
        bufs = self.__dict__.setdefault("_pool_bufs", {})
        spares = self.__dict__.setdefault("_pool_spare", {})
        spare = spares.pop(name, None)
        if (spare is None or _viewed_elsewhere(spare) or spare.dtype != cur.dtype
                or spare.shape[1:] != cur.shape[1:] or spare.shape[0] < k or spare.device != cur.device):
            live = bufs.get(name, (None, -1))[0]
            rows = max(k, live.shape[0] if live is not None else 0)
            spare = torch.empty((rows,) + tuple(cur.shape[1:]), dtype=cur.dtype, device=cur.device)
        out = spare[:k]
        old = bufs.get(name, (None, -1))[0]
        if old is not None and old.data_ptr() != spare.data_ptr():
            spares[name] = old          # the previous live buffer becomes the spare
        bufs[name] = (spare, k)
        return out

    def set_pool(self, coord, sdf_label, ts, weight=None, global_coord=None):
        """Install a training-sample pool (the output of Mapper.process_frame, utils/mapper.py:110-321)."""
        self.coord_pool = coord
        self.global_coord_pool = coord if global_coord is None else global_coord
        self.sdf_label_pool = sdf_label
        self.time_pool = ts
        self.weight_pool = torch.ones_like(sdf_label) if weight is None else weight
        self.pool_sample_count = int(sdf_label.shape[0])

    def _pool_signature(self):
        pools = (self.global_coord_pool, self.sdf_label_pool, self.time_pool, self.weight_pool)
        return tuple((id(t), t.data_ptr(), t._version, t.shape[0]) if t is not None else None for t in pools)

    @staticmethod
    def _pack(coord, label, ts, weight, out=None):
        """pin_pool_pack of [n] samples -> [n, 8] f32 records (out: written in place)."""
        n = label.shape[0]
        out = torch.empty((n, 8), dtype=torch.float32, device=label.device) if out is None else out
        # converted copies held in locals until the launch is queued: a temporary freed inside the
        # argument list could be handed by the caching allocator to the next conversion, whose
        # queued write would land before the pack kernel reads it
        w = None if weight is None else weight.detach().to(torch.float32).contiguous()
        c = coord.contiguous()
        lb = label.contiguous()
        t64 = None if ts is None else ts.to(torch.int64).contiguous()
        _lib.call("pin_pool_pack", _lib.ptr(c), _lib.ptr(lb), _lib.ptr(t64), _lib.ptr(w), n, _lib.ptr(out),
                  _lib.stream())
        return out

    def _packed_pool(self):
        """The pools (global coordinates, labels, ts, weights) as one 32-B record per sample, for the
        batch gather.  process_frame keeps it current incrementally (new samples packed on append,
        the window filter's compaction applied to it too); any other change to the pools (set_pool,
        the bundle-adjustment re-transform, a caller's assignment) is detected by the pools'
        identity / version / length and the records are rebuilt in one pass."""
        sig = self._pool_signature()
        pk = self.__dict__.get("_pool_packed")
        if pk is not None and self.__dict__.get("_pool_packed_sig") == sig:
            return pk
        if not self._pools_fusable():
            return None
        n = self.sdf_label_pool.shape[0]
        if self.global_coord_pool.shape[0] != n or (self.time_pool is not None and self.time_pool.shape[0] != n):
            return None
        weight = self.weight_pool if (self.weight_pool is not None and self.weight_pool.shape[0] == n) else None
        bufs = self.__dict__.setdefault("_pool_bufs", {})
        buf = bufs.get("packed", (None, -1))[0]
        if buf is None or buf.shape[0] < n:
            buf = torch.empty((max(n, self._pool_rows_hint(0)), 8), dtype=torch.float32, device=self.device)
        pk = self._pack(self.global_coord_pool, self.sdf_label_pool, self.time_pool, weight, out=buf[:n])
        bufs["packed"] = (buf, n)
        self._pool_packed, self._pool_packed_sig = pk, sig
        return pk

    def _device_seed(self, iters):
        """A 62-bit seed for one mapping() call's device draws from the device's torch generator:
        its initial seed and Philox offset, the offset advanced by 8 per iteration (two randint
        draws of <= 4 values per thread each, as get_batch's would consume).  Falls back to the CPU
        generator where the device generator has no offset API."""
        dev = torch.device(self.device)
        try:
            gen = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
            off = int(gen.get_offset())
            gen.set_offset(off + 8 * max(int(iters), 1))
            x = (int(gen.initial_seed()) * 0x9E3779B97F4A7C15 + off + 1) & ((1 << 64) - 1)
            x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
            x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
            return (x ^ (x >> 31)) >> 2
        except (AttributeError, RuntimeError, IndexError):
            return int(torch.randint(0, 1 << 62, (1,)).item())

    def _randint(self, high, n):
        """torch.randint(0, high, (n,)) on the mapper's device: every draw of get_batch goes through
        here (tests replay the reference's recorded draws by replacing it on the instance)."""
        return torch.randint(0, high, (n,), device=self.device)

    def _new_sample_mode(self):
        """get_batch draws half new / half history samples (utils/mapper.py:325)."""
        stop = getattr(self.dataset, "stop_status", False) if self.dataset is not None else False
        return (int(getattr(self.config, "bs_new_sample", 0)) > 0 and self.new_idx is not None
                and not self.lose_track and not stop)

    def _batch_index(self, rows=None, new_idx=None):
        """The pool rows of one batch: get_batch's sampling (utils/mapper.py:323-350), same draws.
        rows / new_idx: the pool rows (and new samples) to draw from instead of the whole pool
        (a spatially sharded rank's slab).  self._n_new_rows: rows at the end that are new samples."""
        index_history, new_sel, index_new = self._batch_parts(rows, new_idx)
        if new_sel is None:
            return index_history
        return torch.cat((index_history, new_sel[index_new]), dim=0)

    def _batch_parts(self, rows=None, new_idx=None):
        """_batch_index's two draws kept apart: (history rows, new_idx or None, draw into new_idx or
        None); the batch is history rows followed by new_idx[draw] (the gather concatenates)."""
        bs = int(self.config.bs)
        bs_new_sample = int(getattr(self.config, "bs_new_sample", 0))
        count = self.pool_sample_count if rows is None else rows.shape[0]
        pick = (lambda i: i) if rows is None else (lambda i: rows[i])   # noqa: E731
        new_idx = self.new_idx if rows is None else new_idx
        self._n_new_rows = 0
        if self._new_sample_mode() and new_idx is not None:
            new_idx_count = new_idx.shape[0]
            if new_idx_count > 0:
                bs_new = min(new_idx_count, bs_new_sample)
                bs_history = bs - bs_new
                index_history = pick(self._randint(count, bs_history))
                index_new_batch = self._randint(new_idx_count, bs_new)
                self._n_new_rows = bs_new
                return index_history, new_idx, index_new_batch
        return pick(self._randint(count, bs)), None, None

    def _batch_sizes(self):
        """_batch_parts' sizes without its draws: (history rows, new_idx or None, new-sample rows)
        -- the device-drawn batch of the dense loop (pin_train_gather_packed_draw)."""
        bs = int(self.config.bs)
        bs_new_sample = int(getattr(self.config, "bs_new_sample", 0))
        self._n_new_rows = 0
        if self._new_sample_mode() and self.new_idx is not None:
            new_idx_count = self.new_idx.shape[0]
            if new_idx_count > 0:
                bs_new = min(new_idx_count, bs_new_sample)
                self._n_new_rows = bs_new
                return bs - bs_new, self.new_idx.to(torch.int64).contiguous(), bs_new
        return bs, None, 0

    def get_batch(self, global_coord=False):
        """utils/mapper.py:323-361."""
        index = self._batch_index()
        coord = self.global_coord_pool[index, :] if global_coord else self.coord_pool[index, :]
        sdf_label = self.sdf_label_pool[index]
        ts = self.time_pool[index]
        weight = self.weight_pool[index]
        sem_label = self.sem_label_pool[index] if self.sem_label_pool is not None else None
        color_label = self.color_pool[index] if self.color_pool is not None else None
        normal_label = self.normal_label_pool[index, :] if self.normal_label_pool is not None else None
        return coord, sdf_label, ts, normal_label, sem_label, color_label, weight

    # ---------------------------------------------------------------- training
    def _check_supported(self):
        c = self.config
        if c.main_loss_type != "bce":
            raise NotImplementedError("fused mapping implements main_loss_type 'bce' (utils/loss.py:40-47)")
        if getattr(c, "semantic_on", False) or getattr(c, "color_on", False):
            raise NotImplementedError("fused mapping implements the geometric decoder only")
        if getattr(c, "proj_correction_on", False) or getattr(c, "consistency_loss_on", False):
            raise NotImplementedError("proj_correction / consistency losses are not on the fused path")
        if c.ekional_loss_on and c.weight_e > 0:
            if getattr(c, "ekional_add_to", "all") != "all":
                raise NotImplementedError("fused mapping implements ekional_add_to 'all'")
        # utils/tools.py:89-116: the fused step is Adam without L2 (the reference's defaults)
        if not getattr(c, "opt_adam", True):
            raise NotImplementedError("fused mapping implements the Adam optimizer only (opt_adam True)")
        if float(getattr(c, "weight_decay", 0.0)) != 0.0:
            raise NotImplementedError("fused mapping implements Adam with weight_decay 0")

    def _world(self):
        """Ranks of the data-parallel group; 1 without an explicit group (an initialised default
        group alone does not make a mapper data-parallel: replicas mapping their own data, like
        bench.py's whole-frame leg, must not exchange gradients)."""
        group = getattr(self, "group", None)
        if group is None or group is False or not dist.is_available() or not dist.is_initialized():
            return 1
        return dist.get_world_size(group)

    def mapping(self, iter_count):
        """utils/mapper.py:425-593 (iteration body :443-575)."""
        self.check_deferred()
        if self.train_less:
            iter_count = max(1, iter_count - 5)
        self._check_supported()
        nm = self.neural_points
        feats = nm.local_geo_features
        _lib.require_device(feats.data)
        mlp_params = [p for p in self.geo_mlp.parameters() if p.requires_grad]
        train_mlp = len(mlp_params) > 0
        if train_mlp and len(mlp_params) != 4:
            raise NotImplementedError("fused mapping trains the whole 11->64->1 decoder or none of it")
        world = self._world()
        dev = feats.device
        # fresh optimiser state per call (utils/tools.py:89-116 via mapper.py:441)
        fdata = feats.data
        # gradient and moments (and the decoder's) zeroed in one fill; the dense fused loop's first
        # Adam step takes the moments as zero (PinAdamStep.zero_grad bit 1), so only the gradients
        # are filled there
        fused = (not self.ba_done_flag and "get_batch" not in self.__dict__ and self._pools_fusable())
        dense_loop = fused and (world <= 1 or getattr(self, "shard", "dense") != "space")
        nf, nmg = fdata.numel(), (_lib.MLP_GRAD_SIZE if train_mlp else 0)
        owner = None
        if dense_loop:
            grads = torch.zeros((nf + nmg,), dtype=torch.float32, device=dev)
            # data-parallel: reduce-scatter -> Adam on this rank's rows -> all-gather (OwnerAdam),
            # so the feature moments cover only this rank's rows
            if world > 1:
                owner = OwnerAdam(nf, getattr(self, "group", None), _AR_BUCKETS)
            nfm = owner.moments_size() if owner is not None else nf
            moments = torch.empty((2 * nfm + 2 * nmg,), dtype=torch.float32, device=dev)
            f_grad, f_m, f_v = grads[:nf].view_as(fdata), moments[:nfm], moments[nfm:2 * nfm]
            if owner is None:
                f_m, f_v = f_m.view_as(fdata), f_v.view_as(fdata)
            m_grad = m_m = m_v = None
            if train_mlp:
                m_grad, m_m, m_v = grads[nf:], moments[2 * nfm:2 * nfm + nmg], moments[2 * nfm + nmg:]
        else:
            state = torch.zeros((3 * nf + 3 * nmg,), dtype=torch.float32, device=dev)
            f_grad, f_m, f_v = (state[k * nf:(k + 1) * nf].view_as(fdata) for k in range(3))
            m_grad = m_m = m_v = None
            if train_mlp:
                m_grad, m_m, m_v = (state[3 * nf + k * nmg:3 * nf + (k + 1) * nmg] for k in range(3))
        cert_before = nm.local_point_certainties.clone() if world > 1 else None
        self._adam_t = 0
        # get_batch's gathers fused into the row build (pin_train_gather) when the pools allow it;
        # a get_batch replaced on the instance (tests, callers) is honoured
        fused = (not self.ba_done_flag and "get_batch" not in self.__dict__ and self._pools_fusable())
        part, slab_rows, slab_new, scales = self._slab_partition(world, fused)
        packed = self._packed_pool() if fused and _PACK_POOL else None
        # the dense fused loop builds its launch plan once (views, structs, buffers) and then only
        # draws and launches (gather, forward, backward, one Adam step that also sums the gradient
        # replicas and re-packs a training decoder); the version bumps of the raw-pointer writes
        # (features, decoder, certainty / ts) are applied once after the loop -- nothing inside
        # it reads them
        plan = None
        if fused and part is None:
            plan = self._dense_loop(iter_count, world, fdata, f_grad, f_m, f_v, mlp_params, m_grad, m_m, m_v, packed,
                                    owner, grads)
        for _ in range(iter_count if plan is None else 0):
            if fused:
                index = self._batch_index(slab_rows, slab_new)
                scale_h, scale_n = scales(int(index.shape[0]) - self._n_new_rows, self._n_new_rows)
                self.train_step(self.global_coord_pool, self.sdf_label_pool, self.time_pool, f_grad, m_grad,
                                world, index=index, reduce=False, scale=scale_h, n_tail=self._n_new_rows,
                                scale_tail=scale_n, weight=self.weight_pool, packed=packed)
            else:
                coord, sdf_label, ts, _, _, _, weight = self.get_batch(global_coord=not self.ba_done_flag)
                if self.ba_done_flag:
                    coord = transform_batch_torch(coord, self.used_poses[ts])
                self.train_step(coord, sdf_label, ts, f_grad, m_grad, world, weight=weight)
            if part is not None:
                part.exchange_gradients(f_grad)                   # halo rows -> owners
                if m_grad is not None:
                    all_reduce(m_grad, group=getattr(self, "group", None))
            self._adam(fdata, f_grad, f_m, f_v, mlp_params, m_grad, m_m, m_v, partition=part)
            if part is not None:
                part.exchange_features(fdata)                     # owners -> halo copies
            self.total_iter += 1
        if plan is not None:
            plan.finish()
            nm.mark_modified(feats)
            for p in mlp_params:
                torch.autograd.graph.increment_version(p)
            if mlp_params and plan.mv.struct.packed:   # the loop's Adam launches re-packed the image
                mlp_view_repacked(self.geo_mlp, plan.mv.struct.packed)
            self.total_iter += iter_count
        if part is not None:
            part.reconcile_side_effects(cert_before, nm.local_point_certainties, nm.local_point_ts_update)
            part.gather_owned(fdata, nm.local_point_certainties, nm.local_point_ts_update)
            nm.mark_modified(feats, nm.local_point_certainties, nm.local_point_ts_update)
        elif world > 1:
            cert = nm.local_point_certainties
            cert_delta = cert - cert_before
            sync_side_effects(cert_delta, nm.local_point_ts_update, getattr(self, "group", None))
            cert.copy_(cert_before + cert_delta)
        nm.assign_local_to_global()
        if fused and iter_count > 0:
            if getattr(self, "defer_checks", False):
                # the flag leaves with an asynchronous copy; the next call reads it (its event has
                # completed by then), so the host does not wait here for the whole call's kernels
                flag = self.__dict__.get("_gather_flag_host")
                if flag is None:
                    flag = self._gather_flag_host = torch.zeros((1,), dtype=self._buf.gather_error.dtype,
                                                                pin_memory=True)
                flag.copy_(self._buf.gather_error.view(-1)[:1], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                self._pending_gather_check = ev
            elif int(self._buf.gather_error.item()):
                self._buf.gather_error.zero_()
                raise IndexError("mapping(): a batch index fell outside the sample pool")

    def check_deferred(self):
        """The device-side batch check of the last mapping() call made with defer_checks (raises
        what that call would have raised)."""
        ev = self.__dict__.pop("_pending_gather_check", None)
        if ev is not None:
            ev.synchronize()
            if int(self._gather_flag_host[0]):
                self._buf.gather_error.zero_()
                raise IndexError("mapping(): a batch index fell outside the sample pool")

    def _dense_loop(self, iter_count, world, fdata, f_grad, f_m, f_v, mlp_params, m_grad, m_m, m_v, packed,
                    owner=None, grads=None):
        """The iterations of a dense fused mapping() call (utils/mapper.py:443-575): per iteration
        the batch draw (_batch_parts), the gather, forward and backward of a launch plan built
        once (_step_plan) and one pin_adam_step_train launch (the gradient replicas summed, a
        training decoder stepped and re-packed).  The version bumps of the raw-pointer writes are
        the caller's, after the loop -- nothing inside it reads them.  Returns the plan (None
        for no iterations)."""
        c = self.config
        plan = None
        segs = None
        adam = _lib.fn("pin_adam_step_train")
        s = _lib.stream()
        # get_batch's draws on the device: one seed per call from torch's (seeded) CPU generator,
        # the iteration counter per iteration; the tests' replay hook (_randint on the instance)
        # keeps the host draws
        dev_draw = (_DEVICE_DRAWS and packed is not None and getattr(self, "device_draws", True)
                    and "_randint" not in self.__dict__ and getattr(type(self), "_randint", None) is Mapper._randint)
        seed = self._device_seed(iter_count) if dev_draw else 0
        for it in range(iter_count):
            draw = None
            if dev_draw:
                n_hist, new_sel, n_new = self._batch_sizes()
                idx, idx_new = self._buf.draw_shapes(n_hist, new_sel, n_new, fdata.device)
                draw = (n_hist, new_sel, seed, it)
            else:
                index, new_sel, index_new = self._batch_parts()
                idx, idx_new = self._step_index(self.global_coord_pool, index,
                                                None if new_sel is None else (new_sel, index_new), packed)
            n = idx.shape[0] + (0 if idx_new is None else idx_new[1].shape[0])
            if plan is None or plan.n != n:
                plan = self._step_plan(self.global_coord_pool, self.sdf_label_pool, self.time_pool, f_grad, m_grad,
                                       world, idx, None, 0, 0.0, self.weight_pool, packed, idx_new, fused_adam=True)
                if m_grad is not None and segs is None:
                    segs = self._adam_segments(mlp_params, m_grad)
                mv = plan.mv if (segs is not None and plan.mv.struct.packed) else None
                # pin_adam_step_train's arguments but the per-step scalars
                head = (_lib.ptr(fdata), _lib.ptr(f_grad), _lib.ptr(f_m), _lib.ptr(f_v), fdata.numel(),
                        _lib.ptr(plan.rep), _REPLICAS if plan.rep is not None else plan.nfix,
                        _lib.ptr(plan.fix), FIXED_SHIFT,
                        segs[0] if segs else None, segs[1] if segs else None, len(mlp_params) if segs else 0,
                        _lib.ptr(m_grad), _lib.ptr(m_m), _lib.ptr(m_v), mv.ref() if mv else None,
                        ctypes.c_void_p(mv.struct.packed) if mv else None)
            plan.run(idx, idx_new, draw)
            self._adam_t += 1
            # the first step of the call's fresh optimiser: the moments are taken as zero (mapping()
            # leaves them unfilled for this loop)
            st = adam_scalars(c.lr, self._adam_t, c.adam_eps, zero_grad=3 if self._adam_t == 1 else 1)
            if world > 1:
                self._owner_adam(owner, fdata, grads, f_m, f_v, m_grad, head, st, s)
            else:
                _lib.check("pin_adam_step_train", adam(*head, ctypes.byref(st), s))
        return plan

    def _owner_adam(self, owner, fdata, grads, f_m, f_v, m_grad, head, st, s):
        """The data-parallel step of the dense loop (the reference's
        optimizer.step(), utils/mapper.py:570-572): the ranks' gradients (scaled by 1/W in the
        backward) reduce-scattered in row buckets, pin_adam_step on this rank's piece of each
        bucket as soon as that bucket lands, the stepped piece all-gathered while the later
        buckets are still on the wire (sharding.OwnerAdam).  The decoder's 833 gradients travel
        with the few feature rows that do not fill a bucket in one all-reduce; every rank steps
        (and re-packs) the decoder with one block of pin_adam_step_train."""
        step = _lib.fn("pin_adam_step")

        def adam(p, g, m, v):
            _lib.check("pin_adam_step", step(_lib.ptr(p), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), p.numel(),
                                             ctypes.byref(st), s))

        def decoder():
            if m_grad is not None:
                dec_args = (None, None, None, None, 0, None, 0, None, 0) + head[9:]
                _lib.check("pin_adam_step_train", _lib.fn("pin_adam_step_train")(*dec_args, ctypes.byref(st), s))
        owner.step(fdata.view(-1), grads, f_m, f_v, adam, decoder)

    def _slab_partition(self, world, fused):
        """shard="space" set-up of one mapping() call: (partition, the slab's pool rows, the slab's
        new samples, scales) -- or four Nones for the dense path.  Every rank takes the same
        decision (the counts are all-reduced before any rank leaves the set-up): a slab without
        pool samples makes the call fall back to dense, with a warning.  The global2local
        fill-quirk row (local row 1) is a shared row of the partition, not a fallback.

        scales(bs_hist_r, bs_new_r) -> (history-row scale, new-row scale).  A rank draws its batch
        from its slab only, so its rows are weighted to keep the union an unbiased estimate of the
        reference's single-process batch (utils/mapper.py:323-350: bs_hist rows uniform over the
        pool of N samples, bs_new rows uniform over the n new samples):
            scale_h = (bs_hist / bs_hist_r) (N_r / N),   scale_n = (bs_new / bs_new_r) (n_r / n)
        with N_r / n_r the slab's pool / new sample counts (a flat 1/W would over-weight the samples
        of sparsely sampled slabs).  A stencil group takes the scale of its base row."""
        if world <= 1 or getattr(self, "shard", "dense") != "space":
            return None, None, None, None
        group = getattr(self, "group", None)
        nm = self.neural_points
        if not fused:
            raise NotImplementedError("shard='space' samples device pools through the fused batch path")
        from .sharding import SlabPartition, query_reach, slab_batch_plan
        part = SlabPartition(nm.local_neural_points, query_reach(nm, self.config), group,
                             layout=getattr(self, "slab_layout", "auto"))
        plan = slab_batch_plan(part, self.global_coord_pool[: self.pool_sample_count], self.new_idx,
                               int(self.config.bs), int(getattr(self.config, "bs_new_sample", 0)),
                               self._new_sample_mode())
        if plan is None:
            warnings.warn("shard='space': a slab holds no pool samples; this mapping() call uses the dense "
                          "gradient all-reduce")
            return None, None, None, None
        self._partition = part
        return (part,) + plan

    def _pools_fusable(self):
        c, l, t = self.global_coord_pool, self.sdf_label_pool, self.time_pool
        return (c is not None and c.is_cuda and c.dtype == torch.float32 and c.is_contiguous() and c.dim() == 2
                and l is not None and l.dtype == torch.float32 and l.is_contiguous()
                and (t is None or (t.dtype == torch.int64 and t.is_contiguous())))

    def train_step(self, coord, sdf_label, ts, grad_features, mlp_grad=None, world=1, index=None, reduce=True,
                   scale=None, n_tail=0, scale_tail=0.0, weight=None, packed=None, index_new=None):
        """Forward + backward of one iteration: grad_features [L+1,8] (+ mlp_grad [833]) += dL/d*,
        SUM all-reduced over the group when world > 1 and reduce.  Returns the device loss tensor.
        index ([N] int64): coord / sdf_label / ts are then the sample pools and the batch is their
        rows `index` (get_batch's gathers done by pin_train_gather).
        scale: loss / gradient factor (default 1/world); the last n_tail batch rows (and the
        stencil groups based on them) take scale_tail instead (slab sharding's new-sample rows).
        weight: the batch rows' sample weights (the weight pool with index), used as |weight| by the
        BCE term when loss_weight_on (utils/mapper.py:514-516).
        packed: the same pools as one 32-B record per sample (_packed_pool), gathered instead.
        index_new: (new_idx, draw) -- the batch continues with rows new_idx[draw] after index
        (get_batch's new samples, _batch_parts), concatenated by the packed gather itself."""
        index, index_new = self._step_index(coord, index, index_new, packed)
        plan = self._step_plan(coord, sdf_label, ts, grad_features, mlp_grad, world, index, scale, n_tail,
                               scale_tail, weight, packed, index_new)
        plan.run(index, index_new)
        plan.finish()
        if world > 1 and reduce:
            allreduce_gradients([grad_features, mlp_grad], getattr(self, "group", None))
        return plan.b.loss

    @staticmethod
    def _step_index(coord, index, index_new, packed):
        """The batch's pool rows as the gathers take them (int64 on the pool's device)."""
        if index is None:
            return None, None
        index = index.to(device=coord.device, dtype=torch.int64).contiguous()
        if index_new is not None:
            new_sel, draw = (t.to(device=coord.device, dtype=torch.int64).contiguous() for t in index_new)
            if packed is None:    # the unpacked gather takes one index
                return torch.cat((index, new_sel[draw]), dim=0), None
            index_new = (new_sel, draw)
        return index, index_new

    def _step_plan(self, coord, sdf_label, ts, grad_features, mlp_grad, world, index, scale, n_tail, scale_tail,
                   weight, packed, index_new, fused_adam=False):
        """Everything of one training iteration that does not depend on the batch's draw: the
        configuration structs, the views, the per-row buffers and the launch arguments.  It stays
        valid while the map, the pools and the batch size stay as they are -- a whole mapping()
        call, whose iterations then only launch (_StepPlan.run).  fused_adam: the caller steps with
        pin_adam_step_train, which also sums the gradient replicas and re-packs the decoder."""
        c = self.config
        nm = self.neural_points
        weighted = bool(getattr(c, "loss_weight_on", False)) and weight is not None
        P = _StepPlan()
        P.mapper = self
        P.wrow = None
        P.rep = None
        if index is None:
            q = coord.detach().to(torch.float32).contiguous()
            _lib.require_device(q)
            P.label = sdf_label.detach().to(torch.float32).contiguous()
            P.ts64 = ts.to(device=q.device, dtype=torch.int64).contiguous() if ts is not None else None
            n = q.shape[0]
            if weighted:
                P.wrow = weight.detach().to(device=q.device, dtype=torch.float32).abs().contiguous()
        else:
            q = coord
            _lib.require_device(q)
            n = index.shape[0] + (0 if index_new is None else index_new[1].shape[0])
        if grad_features is not None and (grad_features.shape[1] != 8 or not grad_features.is_contiguous()):
            raise ValueError("grad_features must be a contiguous [L+1, 8] float32 tensor")
        dec = int(c.gradient_decimation)
        eik = bool(c.ekional_loss_on and c.weight_e > 0)
        # numerical_grad off: the eikonal term on the analytic gradient of every batch row, its
        # double backward in closed form (PIN_TRAIN_EIK, utils/mapper.py:50-54, :481-482)
        analytic = eik and not bool(c.numerical_grad)
        nd = (n + dec - 1) // dec if (eik and not analytic) else 0
        nn_k = int(c.query_nn_k)
        wf = bool(c.weighted_first)
        rows = n + 6 * nd
        if not hasattr(self, "_buf"):    # methods transplanted onto the reference class
            self._buf = _TrainBuffers()
        b = P.b = self._buf.get(rows, nn_k, wf, q.device)
        P.n, P.rows = n, rows
        cfg = _lib.PinTrainCfg(n_main=n, n_stencil=nd, decimation=dec, nn_k=nn_k, weighted_first=int(wf),
                               eps=float(np.float32(c.voxel_size_m * c.num_grad_step_ratio)),
                               sigma=float(np.float32(self.sdf_scale)), weight_e=float(np.float32(c.weight_e)),
                               grad_scale=float(np.float32(1.0 / world if scale is None else scale)), flags=0,
                               n_tail=int(n_tail), grad_scale_tail=float(np.float32(scale_tail)))
        hv, pv = nm._views("local", True)
        s = P.s = _lib.stream()
        grid = nm.backend() == "grid"
        gv = P.gv = nm.grid_view("local", False) if grid else None
        # every row of the iteration (batch + stencil) materialised once: the tile sort and the
        # forward read it; the row build / gather takes flags 0, the training kernels their own
        cfg_rows = P.cfg_rows = cfg
        rows_xyz = b.rows
        if index is None:
            P.q = q
        else:
            P.label = b.label
            P.ts64 = b.ts if ts is not None else None
            P.wrow = b.wrow if weighted else None
            if packed is None:
                P.pools = (q, sdf_label, ts, weight.detach().to(torch.float32).contiguous() if weighted else None)
            P.packed = packed
            if packed is not None:
                P.packed_ptr, P.packed_rows = packed.data_ptr(), int(packed.shape[0])
        P.gather_tail = (ctypes.byref(cfg_rows), _lib.ptr(rows_xyz), _lib.ptr(P.label), _lib.ptr(P.ts64),
                         _lib.ptr(P.wrow), _lib.ptr(b.gather_error), s)
        P.index_mode = index is not None
        cfg = P.cfg = _lib.PinTrainCfg.from_buffer_copy(cfg_rows)
        cfg.flags = _lib.PIN_TRAIN_ROWS
        P.tiled = grid and _TILE_QUERIES and rows >= _TRAIN_TILE_MIN
        det = P.det = bool(getattr(self, "deterministic", None) if hasattr(self, "deterministic")
                           else _deterministic_default(c))
        st = P.st = _lib.PinTrainState(ids=b.ids.data_ptr(), weights=b.weights.data_ptr(), x=b.x.data_ptr(),
                                       sdf=b.sdf.data_ptr(), certainties=nm.local_point_certainties.data_ptr(),
                                       ts_update=nm.local_point_ts_update.data_ptr() if P.ts64 is not None else None,
                                       order=None, sorted_rows=b.rows4.data_ptr() if P.tiled else None,
                                       row_weight=_lib.ptr(P.wrow), row_ts=_lib.ptr(P.ts64))
        # replicas for small batches on small maps: every replica is read and re-zeroed in full per
        # iteration (L+1 rows x 32 B each), which pays only while the map is not much larger than
        # the batch's (row, neighbour) pairs
        use_rep = (grad_features is not None and rows < _REPLICA_ROWS and _REPLICAS > 1
                   and grad_features.shape[0] == pv.features.shape[0]
                   and grad_features.shape[0] <= 2 * rows * nn_k)
        # the Adam launch sums the replicas -- unless the gradient is all-reduced before it
        defer = bool(fused_adam) and world == 1
        if det and grad_features is not None:
            if grad_features.shape[0] != pv.features.shape[0]:
                raise ValueError("deterministic mapping needs grad_features of the local map's [L+1, 8] shape")
            nrep = _REPLICAS if use_rep else 1
            fix = b.fixed(2 * nrep * grad_features.numel(), q.device)   # coarse and fine parts
            st.grad_fixed, st.fixed_shift = fix.data_ptr(), FIXED_SHIFT
            st.replicas, st.replica_mode = nrep, int(defer)
            P.fix, P.nfix = (fix if defer else None), nrep
        elif use_rep:
            rep = b.replicas(_REPLICAS * grad_features.numel(), q.device)
            st.grad_replicas, st.replicas, st.replica_mode = rep.data_ptr(), _REPLICAS, int(defer)
            P.rep = rep if defer else None
        if det:
            cf = P.cert_fix = b.cert_fixed(nm.local_point_certainties.numel(), q.device)
            st.cert_fixed, st.cert_shift = cf.data_ptr(), CERT_SHIFT
        # frozen decoder (PIN_TRAIN_DX): weighted_first -- decode on the matrix cores and keep
        # dsdf/dx for the backward instead of re-evaluating the decoder there; per-neighbour -- keep
        # each neighbour's ReLU masks from the forward's decode, from which the backward's
        # matrix-core GEMM2 gives its input gradient (no feature re-gather, no hidden layer)
        dx = mlp_grad is None and _MLP_PACK and not analytic and (wf or _NWF_MASK)
        # per-neighbour decoding: the backward takes each neighbour's dsdf/dx from the matrix cores;
        # weighted_first with a training decoder: the backward decodes each row there once (input
        # gradient + ReLU masks of the decoder-parameter products)
        mv = P.mv = mlp_view(self.geo_mlp,
                             packed=_MLP_PACK and (mlp_grad is None or (wf and not analytic and _ROW_DECODE)))
        if rows < _PAIR_ROWS:
            cfg.flags |= _lib.PIN_TRAIN_PAIR
        if dx:
            cfg.flags |= _lib.PIN_TRAIN_DX
        if analytic:
            cfg.flags |= _lib.PIN_TRAIN_EIK
            ec, ev = b.eik(rows, nn_k, wf)
            st.eik_coef, st.eik_vec = ec.data_ptr(), ev.data_ptr()
        if pv.features.data_ptr() != nm.local_geo_features.data_ptr():
            raise RuntimeError("local_geo_features must be a contiguous float32 tensor")
        P.fwd_args = ((None, gv.ref()) if grid else (hv.ref(), None)) + (
            pv.ref(), mv.ref(), _lib.ptr(rows_xyz), _lib.ptr(P.ts64), ctypes.byref(cfg), ctypes.byref(st), s)
        P.bwd_args = (pv.ref(), mv.ref(), _lib.ptr(P.label), ctypes.byref(cfg), ctypes.byref(st),
                      _lib.ptr(grad_features), _lib.ptr(mlp_grad), _lib.ptr(b.workspace), _lib.ptr(b.loss), s)
        P.keep = (hv, pv, gv, mv, grad_features, mlp_grad)
        P.f_fwd, P.f_bwd = _lib.fn("pin_train_forward"), _lib.fn("pin_train_backward")
        P.f_split = _lib.fn("pin_train_gather_packed_split")
        P.f_draw = _lib.fn("pin_train_gather_packed_draw")
        return P

    def _adam(self, fdata, f_grad, f_m, f_v, mlp_params, m_grad, m_m, m_v, step=None, partition=None):
        """torch.optim.Adam(betas=(0.9, 0.99), eps=adam_eps) step (utils/tools.py:111-112); with a
        slab partition only the owned feature rows (their halo copies are refreshed after)."""
        c = self.config
        self._adam_t = (getattr(self, "_adam_t", 0) + 1) if step is None else step
        st = adam_scalars(c.lr, self._adam_t, c.adam_eps)
        s = _lib.stream()
        segs = None
        if m_grad is not None:
            # the pointer / size arrays cached on the parameters' storage
            skey = (tuple(p.data.data_ptr() for p in mlp_params), m_grad.numel())
            hit = self.__dict__.get("_adam_segs")
            if hit is None or hit[0] != skey:
                hit = (skey, self._adam_segments(mlp_params, m_grad))
                self._adam_segs = hit
            segs = hit[1]
        if partition is None and segs is not None:
            # the features and the decoder's four tensors in one launch (same scalars)
            _lib.call("pin_adam_step_segments", _lib.ptr(fdata), _lib.ptr(f_grad), _lib.ptr(f_m), _lib.ptr(f_v),
                      fdata.numel(), segs[0], segs[1], len(mlp_params), _lib.ptr(m_grad), _lib.ptr(m_m),
                      _lib.ptr(m_v), ctypes.byref(st), s)
        elif partition is None:
            _lib.call("pin_adam_step", _lib.ptr(fdata), _lib.ptr(f_grad), _lib.ptr(f_m), _lib.ptr(f_v),
                      fdata.numel(), ctypes.byref(st), s)
        else:
            _lib.call("pin_adam_rows", _lib.ptr(fdata), _lib.ptr(f_grad), _lib.ptr(f_m), _lib.ptr(f_v),
                      _lib.ptr(partition.adam_rows), partition.adam_rows.numel(), ctypes.byref(st), s)
            partition.zero_halo(f_grad)
        if m_grad is not None and partition is not None:   # the decoder's parameters in one launch of their own
            _lib.call("pin_adam_segments", segs[0], segs[1], len(mlp_params), _lib.ptr(m_grad), _lib.ptr(m_m),
                      _lib.ptr(m_v), ctypes.byref(st), s)
        feats = self.neural_points.local_geo_features
        self.neural_points.mark_modified(feats if feats.data_ptr() == fdata.data_ptr() else fdata)
        # the step wrote through raw pointers: bump the versions so views built on the parameters
        # (the matrix-core operand image of mlp_view) are rebuilt before the next use
        for p in mlp_params if m_grad is not None else ():
            torch.autograd.graph.increment_version(p)

    @staticmethod
    def _adam_segments(mlp_params, m_grad):
        """(pointer array, size array) of the decoder tensors, whose gradients / moments lie end to
        end in m_grad / m_m / m_v (pin_adam_segments' layout)."""
        for p in mlp_params:
            if not (p.data.is_contiguous() and p.data.dtype == torch.float32):
                raise RuntimeError("decoder parameters must be contiguous float32")
        n = len(mlp_params)
        ptrs = (ctypes.c_void_p * n)(*[p.data.data_ptr() for p in mlp_params])
        sizes = (ctypes.c_int64 * n)(*[p.numel() for p in mlp_params])
        if sum(sizes) != m_grad.numel():
            raise RuntimeError("decoder parameters do not match the gradient layout")
        return ptrs, sizes


    # ---------------------------------------------------------------- autograd helpers
    def sdf(self, x, get_std=False):
        """utils/mapper.py:670-681 on the drop-in query_feature (training mode, autograd-capable)."""
        geo_feature, _, weight_knn, _, _ = self.neural_points.query_feature(x)
        sdf_pred = self.geo_mlp.sdf(geo_feature)
        sdf_std = None
        if not self.config.weighted_first:
            sdf_pred_mean = torch.sum(sdf_pred * weight_knn, dim=1)
            if get_std:
                sdf_var = torch.sum((weight_knn * (sdf_pred - sdf_pred_mean.unsqueeze(-1)) ** 2), dim=1)
                sdf_std = torch.sqrt(sdf_var).squeeze(1)
            sdf_pred = sdf_pred_mean.squeeze(1)
        return sdf_pred, sdf_std

    def get_numerical_gradient(self, x, sdf_x=None, eps=0.02, two_side=True):
        """utils/mapper.py:683-733."""
        N = x.shape[0]
        ex = torch.tensor([eps, 0.0, 0.0], dtype=x.dtype, device=x.device)
        ey = torch.tensor([0.0, eps, 0.0], dtype=x.dtype, device=x.device)
        ez = torch.tensor([0.0, 0.0, eps], dtype=x.dtype, device=x.device)
        if two_side:
            pts = torch.cat((x + ex, x - ex, x + ey, x - ey, x + ez, x - ez), dim=0)
            s = self.sdf(pts)[0].unsqueeze(-1)
            gx = (s[:N] - s[N:2 * N]) / (2 * eps)
            gy = (s[2 * N:3 * N] - s[3 * N:4 * N]) / (2 * eps)
            gz = (s[4 * N:5 * N] - s[5 * N:]) / (2 * eps)
        else:
            pts = torch.cat((x + ex, x + ey, x + ez), dim=0)
            s = self.sdf(pts)[0].unsqueeze(-1)
            sx = sdf_x.unsqueeze(-1)
            gx = (s[:N] - sx) / eps
            gy = (s[N:2 * N] - sx) / eps
            gz = (s[2 * N:] - sx) / eps
        return torch.cat([gx, gy, gz], dim=1)


def allreduce_gradients(grads, group=None):
    """SUM all-reduce of the per-rank gradients (already scaled by 1/world in the backward, so
    the sum is the gradient of the mean loss over the union of the ranks' batches).  A [L+1,16]
    accumulator exchanges only its gradient lanes 0..7 (packed, 128 MB at 4M points)."""
    for g in grads:
        if g is None:
            continue
        if g.dim() == 2 and g.shape[1] == 16:
            packed = g[:, :8].contiguous()
            all_reduce(packed, group=group)
            g[:, :8].copy_(packed)
        else:
            all_reduce(g, group=group)


def sync_side_effects(cert_delta, ts_update, group=None):
    """Training-mode side effects of a data-parallel mapping() call: the ranks' certainty deltas
    add up (scatter_add_, neural_points.py:640) and ts_update takes the max (:644)."""
    all_reduce(cert_delta, group=group)
    all_reduce(ts_update, op=dist.ReduceOp.MAX, group=group)


def adam_scalars(lr, step, eps, beta1=0.9, beta2=0.99, zero_grad=True, grad_stride=8) -> "_lib.PinAdamStep":
    """Scalars torch.optim.Adam (single-tensor) derives per step, cast to float32 as its kernels do."""
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    return _lib.PinAdamStep(neg_step_size=float(np.float32(-(lr / bc1))), one_minus_beta1=float(np.float32(1 - beta1)),
                            beta2=float(np.float32(beta2)), one_minus_beta2=float(np.float32(1 - beta2)),
                            bias_correction2_sqrt=float(np.float32(bc2 ** 0.5)), eps=float(np.float32(eps)),
                            zero_grad=int(zero_grad), grad_stride=int(grad_stride))
