"""Drop-in ``NeuralPoints`` (model/neural_points.py:18) backed by the gfx950 kernels.

Same constructor, attributes and methods as the reference class, so
``pin_slam.py``, ``Tracker``, ``Mapper`` and ``Mesher`` run unchanged.  What is
different inside:

* ``buffer_pt_index`` is int32 (200 MB instead of 400 MB at the default
  5e7 slots; fits the 256 MiB Infinity Cache).  Only this class reads it.
* queries run in HIP (``query_feature``, ``radius_neighborhood_search``,
  ``query_certainty``) against per-point candidate *records*
  (x, y, z, id) that fold the travel-distance filter and ``global2local`` into
  one 16-byte gather; records are rebuilt when any tensor they depend on is
  replaced or modified in place (tracked with ``Tensor._version``).
* map maintenance (update / local map / rehash / prune / adjust) runs as
  stream-ordered torch ops on the device plus the hash-rebuild kernel.

Reference quirk kept for parity: ``reset_local_map`` builds ``global2local``
with ``torch.full_like(<bool mask>, -1).long()`` (neural_points.py:301), which
is all ONES, so a point outside the local map that survives the time filter is
read as local point 1.  ``strict_global2local=True`` in the config gives -1
instead (not the reference's behaviour).
"""
import ctypes
import math
import os
import weakref

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .query import QueryFeatureFn, hash_view, points_view

PRIMES = (73856093, 19349669, 83492791)


def neighbor_offsets(num_nei_cells: int, search_alpha: float, device=None) -> torch.Tensor:
    """Integer cell offsets inside the (c + alpha) sphere, in meshgrid 'ij' order
    (model/neural_points.py:430-439)."""
    r = torch.arange(-num_nei_cells, num_nei_cells + 1, dtype=torch.int64, device=device)
    grid = torch.stack(torch.meshgrid(r, r, r, indexing="ij"), -1).reshape(-1, 3)
    keep = (grid * grid).sum(-1) < (num_nei_cells + search_alpha) ** 2
    return grid[keep]


def voxel_down_sample(points: torch.Tensor, voxel_size: float) -> torch.Tensor:
    """Index of one point per voxel: the one closest to the voxel centre after quantising
    the distance to 1000 levels, lowest index on ties (semantics of utils/tools.py:409-442,
    including its flattened-voxel key built with the single extent grid.max())."""
    n = points.shape[0]
    cell = torch.floor(points / voxel_size)
    centre = (cell + 0.5) * voxel_size
    d = ((points - centre) ** 2).sum(1) ** 0.5
    q = (d / d.max() * 999).long()
    c = cell.long() - torch.floor(points.min(dim=0)[0] / voxel_size).long()
    ext = c.max()
    key = c[:, 0] + c[:, 1] * ext + c[:, 2] * ext * ext
    uniq, inv = torch.unique(key, return_inverse=True)
    scale = 10 ** len(str(n - 1))
    packed = torch.arange(n, device=points.device) + q * scale
    best = torch.empty(uniq.shape, dtype=torch.int64, device=points.device)
    best.scatter_reduce_(0, inv, packed, reduce="amin", include_self=False)
    return best % scale


def voxel_down_sample_min_value(points: torch.Tensor, voxel_size: float, value: torch.Tensor) -> torch.Tensor:
    """One point per voxel with the minimum (quantised) value (utils/tools.py:444-477)."""
    n = points.shape[0]
    c = torch.floor(points / voxel_size).long() - torch.floor(points.min(dim=0)[0] / voxel_size).long()
    v = (value / value.max() * 999).long()
    ext = c.max()
    key = c[:, 0] + c[:, 1] * ext + c[:, 2] * ext * ext
    uniq, inv = torch.unique(key, return_inverse=True)
    scale = 10 ** len(str(n - 1))
    packed = torch.arange(n, device=points.device) + v * scale
    best = torch.empty(uniq.shape, dtype=torch.int64, device=points.device)
    best.scatter_reduce_(0, inv, packed, reduce="amin", include_self=False)
    return best % scale


def grid_window_collision_free(buffer_size: int, num_nei_cells: int) -> bool:
    """True iff no two cells whose difference d has |d_i| <= W collide in the hash, where W
    bounds how far (in cells) a neighbour cell can be from the voxel of a candidate that passes
    the distance test: W = c + ceil(sqrt(3) (c + 1)) + 1.  Then a table slot reached from a
    neighbour cell either holds the point whose own voxel it is, or a point too far away to be
    accepted -- which is what makes the occupancy grid exact (pin_grid.hip)."""
    W = num_nei_cells + math.ceil(math.sqrt(3) * (num_nei_cells + 1)) + 1
    r = np.arange(-W, W + 1, dtype=np.int64)
    d = np.stack(np.meshgrid(r, r, r, indexing="ij"), -1).reshape(-1, 3)
    d = d[(d != 0).any(1)]
    h = (d * np.array(PRIMES, dtype=np.int64)).sum(1)
    return not bool((np.mod(h, int(buffer_size)) == 0).any())


def hash_slots(points: torch.Tensor, resolution: float, buffer_size: int) -> torch.Tensor:
    """floor_mod(floor(p / res) . primes, B) (model/neural_points.py:214-216 with the
    negative-index wrap of the table lookup)."""
    g = torch.floor(points / resolution).to(torch.int64)
    h = (g * torch.tensor(PRIMES, dtype=torch.int64, device=points.device)).sum(-1)
    return torch.remainder(h, int(buffer_size))


def last_writer(slots: torch.Tensor) -> torch.Tensor:
    """Positions of the last occurrence of every distinct slot (CPU index_put order)."""
    perm = torch.argsort(slots, stable=True)
    s = slots[perm]
    last = torch.ones_like(s, dtype=torch.bool)
    last[:-1] = s[1:] != s[:-1]
    return perm[last]


def quat_multiply(q1: torch.Tensor, q2: torch.Tensor) -> torch.Tensor:
    w1, x1, y1, z1 = q1.unbind(-1)
    w2, x2, y2, z2 = q2.unbind(-1)
    return torch.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                        w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], -1)


def rotmat_to_quat(R: torch.Tensor) -> torch.Tensor:
    qw = torch.sqrt(1.0 + R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2]) / 2.0
    qx = (R[:, 2, 1] - R[:, 1, 2]) / (4 * qw)
    qy = (R[:, 0, 2] - R[:, 2, 0]) / (4 * qw)
    qz = (R[:, 1, 0] - R[:, 0, 1]) / (4 * qw)
    return torch.stack([qw, qx, qy, qz], -1)


class NeuralPoints(nn.Module):

    def __init__(self, config) -> None:
        super().__init__()
        self.config = config
        self.silence = getattr(config, "silence", True)
        if config.feature_dim != _lib.FEATURE_DIM:
            raise ValueError(f"pin_slam_amd supports feature_dim={_lib.FEATURE_DIM} (got {config.feature_dim})")
        if getattr(config, "pos_encoding_band", 0) > 0:
            raise NotImplementedError("positional encoding (pos_encoding_band > 0) is not on the accelerated path")
        if getattr(config, "color_on", False):
            raise NotImplementedError("colour features are out of scope (off in every lidar config)")
        if getattr(config, "layer_norm_on", False):
            raise NotImplementedError("layer_norm_on is not on the accelerated path")
        self.geo_feature_dim = config.feature_dim
        self.geo_feature_std = config.feature_std
        self.color_feature_dim = config.feature_dim
        self.color_feature_std = config.feature_std
        self.device = config.device
        self.dtype = config.dtype
        self.idx_dtype = torch.int64
        self.resolution = config.voxel_size_m
        self.buffer_size = int(config.buffer_size)
        if not 0 < self.buffer_size < 2 ** 31:
            raise ValueError("buffer_size must be < 2^31 (int32 hash table)")
        self.temporal_local_map_on = True
        self.local_map_radius = config.local_map_radius
        self.diff_travel_dist_local = config.local_map_radius * config.local_map_travel_dist_ratio
        self.diff_ts_local = config.diff_ts_local
        self.local_orientation = torch.eye(3, device=self.device)
        self.cur_ts = 0
        self.max_ts = 0
        self.travel_dist = None
        self.est_poses = None
        self.after_pgo = False
        self.strict_global2local = bool(getattr(config, "strict_global2local", False))
        self.primes = torch.tensor(PRIMES, dtype=self.idx_dtype, device=self.device)

        self.buffer_pt_index = torch.full((self.buffer_size,), -1, dtype=torch.int32, device=self.device)
        self.neural_points = torch.empty((0, 3), dtype=self.dtype, device=self.device)
        self.point_orientations = torch.empty((0, 4), dtype=self.dtype, device=self.device)
        self.geo_features = torch.zeros((1, self.geo_feature_dim), dtype=self.dtype, device=self.device)
        self.color_features = None
        self.point_ts_create = torch.empty((0,), device=self.device, dtype=torch.long)
        self.point_ts_update = torch.empty((0,), device=self.device, dtype=torch.long)
        self.point_certainties = torch.empty((0,), dtype=self.dtype, device=self.device)

        self.local_neural_points = torch.empty((0, 3), dtype=self.dtype, device=self.device)
        self.local_point_orientations = torch.empty((0, 4), dtype=self.dtype, device=self.device)
        self.local_geo_features = nn.Parameter()
        self.local_color_features = nn.Parameter()
        self.local_point_certainties = torch.empty((0,), dtype=self.dtype, device=self.device)
        self.local_point_ts_update = torch.empty((0,), device=self.device, dtype=torch.long)
        self.local_mask = None
        self.global2local = None

        self._cache = {}
        self.set_search_neighborhood(num_nei_cells=config.num_nei_cells, search_alpha=config.search_alpha)
        self.memory_footprint = []
        self.to(self.device)

    # ------------------------------------------------------------------ bookkeeping
    def is_empty(self):
        return self.neural_points.shape[0] == 0

    def count(self):
        return self.neural_points.shape[0]

    def local_count(self):
        return self.local_neural_points.shape[0]

    def print_memory(self):
        if not self.silence:
            print("# Global neural point: %d" % (self.count()))
            print("# Local  neural point: %d" % (self.local_count()))
        point_dim = self.config.feature_dim + 3 + 4
        cur_memory = self.count() * point_dim * 4 / 1024 / 1024
        print("Memory consumption: %f (MB)" % cur_memory)
        self.memory_footprint.append(cur_memory)

    # ------------------------------------------------------------------ neighbourhood
    def set_search_neighborhood(self, num_nei_cells: int = 1, search_alpha: float = 1.0):
        """model/neural_points.py:430-457."""
        self.neighbor_dx = neighbor_offsets(num_nei_cells, search_alpha, device=self.primes.device)
        self.neighbor_K = self.neighbor_dx.shape[0]
        self.max_valid_dist2 = 3 * ((num_nei_cells + 1) * self.resolution) ** 2
        dx_host = np.ascontiguousarray(self.neighbor_dx.cpu().numpy().astype(np.int32))
        self.neighbor_window = int(np.abs(dx_host).max()) if dx_host.size else 0
        self._cells_host = dx_host
        self._cells = None  # device tables built lazily (need the HIP runtime)
        self._offsets = None
        self._grid_exact = grid_window_collision_free(self.buffer_size, num_nei_cells)

    def _cell_table(self):
        if self._cells is None:
            cells = torch.empty(((self.neighbor_K + 15) // 16 * 16,), dtype=torch.int32, device=self.device)
            _lib.require_device(cells)
            _lib.call("pin_neighbor_cells", self._cells_host.ctypes.data_as(_lib.c_void_p), int(self.neighbor_K),
                      self.buffer_size, _lib.ptr(cells), _lib.stream())
            self._cells = cells
        return self._cells

    def _offset_table(self):
        """Packed (dx+128) | (dy+128)<<8 | (dz+128)<<16 per neighbour cell, reference order."""
        if self._offsets is None:
            dx = self._cells_host.astype(np.int64)
            packed = (dx[:, 0] + 128) | ((dx[:, 1] + 128) << 8) | ((dx[:, 2] + 128) << 16)
            pad = np.zeros((self.neighbor_K + 15) // 16 * 16, dtype=np.int32)
            pad[:self.neighbor_K] = packed
            self._offsets = torch.from_numpy(pad).to(self.device)
        return self._offsets

    # ------------------------------------------------------------------ derived-state cache
    def _cached(self, name, deps, scalars, build):
        """Value of ``build()`` cached under ``name`` until a dependency tensor is replaced or
        modified in place (identity + ``Tensor._version``) or a scalar in ``scalars`` changes."""
        hit = self._cache.get(name)
        if hit is not None:
            val, refs, vers, key = hit
            if key == scalars and len(refs) == len(deps) and all(
                    (r() is d) and (d is None or d._version == v) for r, d, v in zip(refs, deps, vers)):
                return val
        val = build()
        refs = tuple(weakref.ref(d) if d is not None else (lambda: None) for d in deps)
        vers = tuple(d._version if d is not None else None for d in deps)
        self._cache[name] = (val, refs, vers, scalars)
        return val

    # ------------------------------------------------------------------ candidate records
    def _deps(self, mode):
        if mode == "global":
            return (self.neural_points,)
        if mode == "global_tf":
            return (self.neural_points, self.point_ts_create, self.travel_dist)
        return (self.neural_points, self.point_ts_create, self.travel_dist, self.global2local,
                self.local_neural_points)

    def records(self, mode: str) -> torch.Tensor:
        """[M,4] f32 candidate records for ``mode`` in {"global", "global_tf", "local"}."""
        return self._cached("records:" + mode, self._deps(mode),
                            (self.cur_ts, float(self.diff_travel_dist_local)), lambda: self._build_records(mode))

    def _build_records(self, mode):
        pts = self.neural_points.contiguous()
        _lib.require_device(pts)
        M = pts.shape[0]
        if M == 0:
            # empty map: one rejected placeholder record (id -1), so the kernels' clamped gathers
            # stay in bounds and every candidate is rejected (the reference raises IndexError here)
            rec = torch.zeros((1, 4), dtype=torch.float32, device=pts.device)
            rec[0, 3] = torch.tensor([-1], dtype=torch.int32).view(torch.float32)[0]
            return rec
        rec = torch.empty((M, 4), dtype=torch.float32, device=pts.device)
        local = mode != "global"
        td = self.travel_dist
        ts = self.point_ts_create.contiguous() if local else None
        if td is not None and local:
            td = td.to(device=pts.device, dtype=torch.float32).contiguous()
            if not 0 <= self.cur_ts < td.shape[0]:
                raise IndexError("travel_dist has no entry for cur_ts=%d" % self.cur_ts)
        else:
            td = None
        g2l = self.global2local.contiguous() if (mode == "local" and self.global2local is not None) else None
        lpos = self.local_neural_points.contiguous() if mode == "local" else None
        _lib.call("pin_build_records", _lib.ptr(pts), M, int(local), _lib.ptr(g2l), _lib.ptr(ts), _lib.ptr(td),
                  int(td.shape[0]) if td is not None else 0, int(self.cur_ts),
                  float(np.float32(self.diff_travel_dist_local)), _lib.ptr(lpos),
                  int(lpos.shape[0]) if lpos is not None else 0, _lib.ptr(rec), _lib.stream())
        return rec

    # ------------------------------------------------------------------ occupancy grid
    MAX_GRID_BRICKS = 1 << 26

    def backend(self) -> str:
        """"grid" when the occupancy grid reproduces the hash probes exactly, else "hash"."""
        want = getattr(self.config, "query_backend", "auto")
        if want == "hash" or self.count() == 0 or not self._grid_exact:
            return "hash"
        occ = self.occupancy()
        if occ is None:
            if want == "grid":
                raise RuntimeError("occupancy grid not exact for this map (displaced table entries or box too big)")
            return "hash"
        return "grid"

    def occupancy(self):
        """(bricks [nb,4] u32, PinGridDims, n_occ) or None when the table holds entries that are
        not at their point's own voxel slot (then only the hash path is exact)."""
        return self._cached("occupancy", (self.neural_points, self.buffer_pt_index),
                            (float(self.resolution), self.buffer_size), self._build_occupancy)

    def _build_occupancy(self):
        pts = self.neural_points.contiguous()
        _lib.require_device(pts)
        res = float(np.float32(self.resolution))
        bounds = torch.empty(6, dtype=torch.int64, device=pts.device)
        _lib.call("pin_cell_bounds", _lib.ptr(pts), pts.shape[0], res, _lib.ptr(bounds), _lib.stream())
        b = bounds.cpu().tolist()
        lo, hi = b[:3], b[3:]
        ext = [(h - l + 1 + 3) // 4 for l, h in zip(lo, hi)]
        nb = ext[0] * ext[1] * ext[2]
        if nb > self.MAX_GRID_BRICKS:
            return None
        dims = _lib.PinGridDims(ox=lo[0], oy=lo[1], oz=lo[2], nbx=ext[0], nby=ext[1], nbz=ext[2], reserved=0)
        bricks = torch.empty((nb, 4), dtype=torch.int32, device=pts.device)
        counters = torch.empty(2, dtype=torch.int64, device=pts.device)
        ws = torch.empty(((nb + 4095) // 4096 * 4 + 16,), dtype=torch.uint8, device=pts.device)
        _lib.call("pin_grid_mark", _lib.ptr(pts), pts.shape[0], res, _lib.ptr(self.buffer_pt_index), self.buffer_size,
                  ctypes.byref(dims), _lib.ptr(bricks), _lib.ptr(counters), _lib.ptr(ws), _lib.stream())
        marked, occupied = counters.cpu().tolist()
        if marked != occupied:
            return None
        return bricks, dims, int(marked)

    def compact_records(self, mode: str, fat: bool):
        """(crec [n_occ,4] f32, cfeat [n_occ,8] or None, ccert [n_occ] or None, cgid [n_occ] i32) in
        brick order for a query mode (features / certainties copied only when ``fat``)."""
        occ = self.occupancy()
        local = mode == "local"
        feats = (self.local_geo_features if local else self.geo_features) if fat else None
        cert = (self.local_point_certainties if local else self.point_certainties) if fat else None
        rec = self.records(mode)
        deps = (self.neural_points, self.buffer_pt_index, rec, feats, cert)
        return self._cached(f"crec:{mode}:{int(fat)}", deps, (float(self.resolution),),
                            lambda: self._build_compact(occ, rec, feats, cert))

    def _build_compact(self, occ, rec, feats, cert):
        bricks, dims, n_occ = occ
        pts = self.neural_points.contiguous()
        n = max(n_occ, 1)
        crec = torch.zeros((n, 4), dtype=torch.float32, device=pts.device)
        cfeat = torch.zeros((n, 8), dtype=torch.float32, device=pts.device) if feats is not None else None
        ccert = torch.zeros((n,), dtype=torch.float32, device=pts.device) if feats is not None else None
        cgid = torch.full((n,), -1, dtype=torch.int32, device=pts.device)
        f = feats.detach().contiguous() if feats is not None else None
        c = cert.detach().contiguous() if cert is not None else None
        _lib.call("pin_grid_fill", _lib.ptr(pts), pts.shape[0], float(np.float32(self.resolution)),
                  _lib.ptr(self.buffer_pt_index), self.buffer_size, ctypes.byref(dims), _lib.ptr(bricks),
                  _lib.ptr(rec), _lib.ptr(f), _lib.ptr(c), _lib.ptr(crec), _lib.ptr(cfeat), _lib.ptr(ccert),
                  _lib.ptr(cgid), _lib.stream())
        return crec, cfeat, ccert, cgid

    def grid_view(self, mode: str, fat: bool):
        from .query import _View
        bricks, dims, n_occ = self.occupancy()
        crec, cfeat, ccert, cgid = self.compact_records(mode, fat)
        offs = self._offset_table()
        g = _lib.PinGrid(bricks=bricks.data_ptr(), dims=dims, crec=crec.data_ptr(), cgid=cgid.data_ptr(),
                         n_occ=n_occ, offsets=offs.data_ptr(), resolution=float(np.float32(self.resolution)),
                         num_cells=int(self.neighbor_K), max_valid_dist2=float(np.float32(self.max_valid_dist2)),
                         cfeat=cfeat.data_ptr() if cfeat is not None else None,
                         ccert=ccert.data_ptr() if ccert is not None else None, fat=int(fat), window=99 if os.environ.get("PIN_GRID_SCAN") == "cells" else self.neighbor_window,
                         reserved=0)
        return _View(g, (bricks, crec, cfeat, ccert, cgid, offs))

    # ------------------------------------------------------------------ map update
    def update(self, points: torch.Tensor, sensor_position: torch.Tensor, sensor_orientation: torch.Tensor, cur_ts):
        """model/neural_points.py:205-270: voxel down-sample, hash probe, insert new points
        (free slot, collision or stale), last-writer-wins slot assignment, padded features."""
        res = self.resolution
        sample_points = points[voxel_down_sample(points, res)]
        slots = hash_slots(sample_points, res, self.buffer_size)
        hash_idx = self.buffer_pt_index[slots].long()
        if not self.is_empty():
            d2 = ((self.neural_points[hash_idx] - sample_points) ** 2).sum(-1)
            dtd = self.travel_dist[cur_ts] - self.travel_dist[self.point_ts_update[hash_idx]]
            update_mask = (hash_idx == -1) | (d2 > 3 * res ** 2) | (dtd > self.diff_travel_dist_local)
        else:
            update_mask = torch.ones(hash_idx.shape, dtype=torch.bool, device=self.device)
        added = sample_points[update_mask]
        n_new = added.shape[0]
        M = self.count()
        cur_idx = hash_idx.clone()
        cur_idx[update_mask] = torch.arange(n_new, dtype=torch.int64, device=self.device) + M
        sel = last_writer(slots)
        self.buffer_pt_index[slots[sel]] = cur_idx[sel].to(torch.int32)
        self.neural_points = torch.cat((self.neural_points, added), 0)
        quat = torch.zeros((n_new, 4), dtype=self.dtype, device=self.device)
        quat[:, 0] = 1.0
        self.point_orientations = torch.cat((self.point_orientations, quat), 0)
        ts = torch.full((n_new,), int(cur_ts), device=self.device, dtype=torch.long)
        self.point_ts_create = torch.cat((self.point_ts_create, ts), 0)
        self.point_ts_update = torch.cat((self.point_ts_update, ts), 0)
        new_fts = self.geo_feature_std * torch.randn(n_new + 1, self.geo_feature_dim, device=self.device,
                                                     dtype=self.dtype)
        self.geo_features = torch.cat((self.geo_features[:-1], new_fts), 0)
        self.point_certainties = torch.cat(
            (self.point_certainties, torch.zeros(n_new, device=self.device, dtype=self.dtype)), 0)
        self.reset_local_map(sensor_position, sensor_orientation, cur_ts)

    def reset_local_map(self, sensor_position: torch.Tensor, sensor_orientation: torch.Tensor, cur_ts: int,
                        use_travel_dist: bool = True, diff_ts_local: int = 50):
        """model/neural_points.py:272-313."""
        self.cur_ts = cur_ts
        self.max_ts = max(self.max_ts, cur_ts)
        dist2sensor = ((self.neural_points - sensor_position) ** 2).sum(-1)
        if self.config.use_mid_ts:
            ts_used = ((self.point_ts_create + self.point_ts_update) / 2).long()
        else:
            ts_used = self.point_ts_create
        if use_travel_dist:
            dtd = torch.abs(self.travel_dist[cur_ts] - self.travel_dist[ts_used])
            mask = (dist2sensor < self.local_map_radius ** 2) & (dtd < self.diff_travel_dist_local)
        else:
            mask = (dist2sensor < self.local_map_radius ** 2) & (torch.abs(cur_ts - ts_used) < diff_ts_local)
        self.local_neural_points = self.neural_points[mask]
        self.local_point_orientations = self.point_orientations[mask]
        self.local_point_certainties = self.point_certainties[mask]
        self.local_point_ts_update = self.point_ts_update[mask]
        mask = torch.cat((mask, torch.ones(1, dtype=torch.bool, device=mask.device)))
        self.local_mask = mask
        fill = -1 if self.strict_global2local else 1  # see module docstring (reference quirk)
        g2l = torch.full(mask.shape, fill, dtype=torch.long, device=mask.device)
        li = torch.nonzero(mask).flatten()
        g2l[li] = torch.arange(li.shape[0], device=mask.device)
        g2l[-1] = -1
        self.global2local = g2l
        self.local_geo_features = nn.Parameter(self.geo_features[mask])
        self.local_orientation = sensor_orientation
        self._local_snapshot = self._snapshot()

    def _snapshot(self):
        """Identity + version of the position / orientation tensors right after reset_local_map:
        while both the global and the local copies are untouched, writing the local copy back
        (assign_local_to_global) is an exact no-op and is skipped, so derived indexes built over
        ``neural_points`` (records, occupancy grid) stay valid across mapping() calls."""
        ts = (self.neural_points, self.local_neural_points, self.point_orientations, self.local_point_orientations)
        return tuple((weakref.ref(t), t._version) for t in ts)

    def _unchanged_since_reset(self, idx):
        snap = getattr(self, "_local_snapshot", None)
        if snap is None:
            return False
        ts = (self.neural_points, self.local_neural_points, self.point_orientations, self.local_point_orientations)
        return all(snap[i][0]() is ts[i] and ts[i]._version == snap[i][1] for i in idx)

    def assign_local_to_global(self):
        """model/neural_points.py:315-324."""
        m = self.local_mask
        if not self._unchanged_since_reset((0, 1)):
            self.neural_points[m[:-1]] = self.local_neural_points
        if not self._unchanged_since_reset((2, 3)):
            self.point_orientations[m[:-1]] = self.local_point_orientations
        self._local_snapshot = self._snapshot()
        self.geo_features[m] = self.local_geo_features.data
        self.point_certainties[m[:-1]] = self.local_point_certainties
        self.point_ts_update[m[:-1]] = self.local_point_ts_update

    def prune_map(self, prune_certainty_thre):
        """model/neural_points.py:329-353."""
        dtd = torch.abs(self.travel_dist[self.cur_ts] - self.travel_dist[self.point_ts_update])
        prune = (dtd > self.diff_travel_dist_local) & (self.point_certainties < prune_certainty_thre)
        count = int(prune.sum().item())
        if count > 100:
            if not self.silence:
                print("# Prune neural points: ", count)
            keep = ~prune
            self.neural_points = self.neural_points[keep]
            self.point_orientations = self.point_orientations[keep]
            self.point_ts_create = self.point_ts_create[keep]
            self.point_ts_update = self.point_ts_update[keep]
            self.point_certainties = self.point_certainties[keep]
            self.geo_features = self.geo_features[torch.cat((keep, torch.ones(1, dtype=torch.bool,
                                                                               device=keep.device)))]
            return True
        return False

    def adjust_map(self, pose_diff_torch):
        """model/neural_points.py:355-370: move every point by the pose correction of its frame."""
        self.after_pgo = True
        if self.config.use_mid_ts:
            used_ts = ((self.point_ts_create + self.point_ts_update) / 2).long()
        else:
            used_ts = self.point_ts_create
        T = pose_diff_torch[used_ts]
        self.neural_points = (torch.matmul(T[:, :3, :3].to(self.neural_points),
                                           self.neural_points.unsqueeze(-1))
                              + T[:, :3, 3:].to(self.neural_points)).squeeze(-1)
        dq = rotmat_to_quat(pose_diff_torch[:, :3, :3])
        self.point_orientations = quat_multiply(dq[used_ts], self.point_orientations).to(self.dtype)

    def recreate_hash(self, sensor_position: torch.Tensor, sensor_orientation: torch.Tensor,
                      kept_points: bool = True, with_ts: bool = True, cur_ts=0):
        """model/neural_points.py:372-428."""
        res = self.resolution
        self.buffer_pt_index = torch.full((self.buffer_size,), -1, dtype=torch.int32, device=self.device)
        if with_ts:
            if self.config.use_mid_ts:
                ts_used = ((self.point_ts_create + self.point_ts_update) / 2).long()
            else:
                ts_used = self.point_ts_create
            sample_idx = voxel_down_sample_min_value(self.neural_points, res, torch.abs(ts_used - cur_ts).float())
        else:
            sample_idx = voxel_down_sample_min_value(self.neural_points, res, -self.point_certainties)
        if kept_points:
            slots = hash_slots(self.neural_points[sample_idx], res, self.buffer_size)
            sel = last_writer(slots)
            self.buffer_pt_index[slots[sel]] = sample_idx[sel].to(torch.int32)
        else:
            self.neural_points = self.neural_points[sample_idx]
            self.point_orientations = self.point_orientations[sample_idx]
            self.point_ts_create = self.point_ts_create[sample_idx]
            self.point_ts_update = self.point_ts_update[sample_idx]
            self.point_certainties = self.point_certainties[sample_idx]
            pad = torch.cat((sample_idx, torch.tensor([-1], device=sample_idx.device)))
            self.geo_features = self.geo_features[pad]
            self.rebuild_hash()
        if sensor_position is not None:
            self.reset_local_map(sensor_position, sensor_orientation, cur_ts)
        if not kept_points:
            self.print_memory()

    def rebuild_hash(self):
        """table[slot(p_i)] = i over all points, highest index wins (HIP kernel)."""
        self.buffer_pt_index.fill_(-1)
        pts = self.neural_points.contiguous()
        _lib.call("pin_hash_rebuild", _lib.ptr(pts), pts.shape[0], float(np.float32(self.resolution)),
                  _lib.ptr(self.buffer_pt_index), self.buffer_size, _lib.stream())

    def clear_temp(self, clean_more: bool = False):
        """model/neural_points.py:678-693."""
        self.buffer_pt_index = None
        self.local_neural_points = None
        self.local_point_orientations = None
        self.local_geo_features = nn.Parameter()
        self.local_color_features = nn.Parameter()
        self.local_point_certainties = None
        self.local_point_ts_update = None
        self.local_mask = None
        self.global2local = None
        self._cache = {}
        if clean_more:
            self.point_ts_create = None
            self.point_ts_update = None
            self.point_certainties = None

    # ------------------------------------------------------------------ queries
    def _views(self, mode: str, query_locally: bool):
        rec = self.records(mode)
        hv = hash_view(self)
        if query_locally:
            pv = points_view(rec, self.local_geo_features.data, self.local_neural_points,
                             self.local_point_orientations, self.local_point_certainties, self.after_pgo)
        else:
            pv = points_view(rec, self.geo_features, self.neural_points, self.point_orientations,
                             self.point_certainties, self.after_pgo)
        return hv, pv

    def radius_neighborhood_search(self, points: torch.Tensor, time_filtering: bool = False):
        """model/neural_points.py:459-509 -> (dist2 [N,K] f32, idx [N,K] int64 global)."""
        _lib.require_device(points)
        q = points.detach().to(torch.float32).contiguous()
        hv, pv = self._views("global_tf" if time_filtering else "global", False)
        n = q.shape[0]
        d2 = torch.empty((n, self.neighbor_K), dtype=torch.float32, device=q.device)
        idx = torch.empty((n, self.neighbor_K), dtype=torch.int64, device=q.device)
        _lib.call("pin_radius_search", hv.ref(), pv.ref(), _lib.ptr(q), n, _lib.ptr(d2), _lib.ptr(idx),
                  _lib.stream())
        return d2, idx

    def query_certainty(self, query_points: torch.Tensor):
        """model/neural_points.py:511-525."""
        _lib.require_device(query_points)
        q = query_points.detach().to(torch.float32).contiguous()
        hv, pv = self._views("global", False)
        out = torch.empty(q.shape[0], dtype=torch.float32, device=q.device)
        _lib.call("pin_query_certainty", hv.ref(), pv.ref(), _lib.ptr(q), q.shape[0], _lib.ptr(out), _lib.stream())
        return out

    def query_feature(self, query_points: torch.Tensor, query_ts: torch.Tensor = None, training_mode: bool = True,
                      query_locally: bool = True, query_geo_feature: bool = True, query_color_feature: bool = False):
        """model/neural_points.py:528-674.  Returns (geo_features_vector, None, weight_vector [N,k,1],
        nn_counts [N] int64, queried_certainty [N]); differentiable w.r.t. the query points and
        the (local) geo features through the HIP backward kernel."""
        if not query_geo_feature and not query_color_feature:
            raise SystemExit("you need to at least query one kind of feature")
        _lib.require_device(query_points)
        nn_k = int(self.config.query_nn_k)
        mode = "local" if query_locally else "global"
        hv, pv = self._views(mode, query_locally)
        feats = self.local_geo_features if query_locally else self.geo_features
        gv = self.grid_view(mode, False) if self.backend() == "grid" else None
        out = QueryFeatureFn.apply(query_points, feats, hv, pv, nn_k, bool(self.config.weighted_first), gv)
        geo_vec, weights, nn_counts, certainty, ids = out
        if training_mode:
            cert_t = self.local_point_certainties if query_locally else self.point_certainties
            ts_t, qts = None, None
            if query_locally and query_ts is not None:
                ts_t = self.local_point_ts_update
                qts = query_ts.to(device=ids.device, dtype=torch.int64).contiguous()
            _lib.call("pin_train_scatter", _lib.ptr(ids), _lib.ptr(weights.detach()), ids.shape[0], nn_k,
                      _lib.ptr(qts), _lib.ptr(cert_t), _lib.ptr(ts_t), _lib.stream())
        return geo_vec, None, weights.unsqueeze(-1), nn_counts, certainty

    def get_map_o3d_bbx(self):
        raise NotImplementedError("open3d visualisation helpers are out of scope")

    def get_neural_points_o3d(self, *args, **kwargs):
        raise NotImplementedError("open3d visualisation helpers are out of scope")
