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
* map maintenance (update / local map / rehash / prune / adjust) runs in the
  pin_map.hip kernels (voxel down-sample, insert, local-map selection,
  gathers/scatters); the only host syncs are the counts that size new tensors.

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
from .query import QueryFeatureFn, hash_view, points_view, tensor_key

PRIMES = (73856093, 19349669, 83492791)


def neighbor_columns(dx: np.ndarray):
    """The neighbour cells regrouped as (x, y) columns for the column scan of the grid kernels:
    entries (dx+128) | (dy+128)<<8 | (dz0+128)<<16 | nz<<24, one per run of consecutive cells with
    the same (dx, dy) and dz ascending by 1.  Visiting the columns in order visits the cells in
    the reference order (meshgrid 'ij', model/neural_points.py:430-439).  None when a column
    would repeat (not a ball) or a run exceeds 5 cells."""
    cols, seen = [], set()
    i = 0
    while i < len(dx):
        x, y, z0 = (int(v) for v in dx[i])
        j = i + 1
        while j < len(dx) and int(dx[j][0]) == x and int(dx[j][1]) == y and int(dx[j][2]) == z0 + (j - i):
            j += 1
        if (x, y) in seen or j - i > 5:
            return None
        seen.add((x, y))
        cols.append((x + 128) | ((y + 128) << 8) | ((z0 + 128) << 16) | ((j - i) << 24))
        i = j
    return cols


def neighbor_offsets(num_nei_cells: int, search_alpha: float, device=None) -> torch.Tensor:
    """Integer cell offsets inside the (c + alpha) sphere, in meshgrid 'ij' order
    (model/neural_points.py:430-439)."""
    r = torch.arange(-num_nei_cells, num_nei_cells + 1, dtype=torch.int64, device=device)
    grid = torch.stack(torch.meshgrid(r, r, r, indexing="ij"), -1).reshape(-1, 3)
    keep = (grid * grid).sum(-1) < (num_nei_cells + search_alpha) ** 2
    return grid[keep]


_MAP_WS = {}


def map_workspace(n: int, device) -> torch.Tensor:
    """Device workspace of the map-maintenance kernels for n elements (grown, reused per device
    and stream: the calls are stream-ordered, so reuse across calls on one stream is safe, and a
    call on another stream -- FrameLoop's next-scan preprocessing -- has a buffer of its own)."""
    need = _lib.map_workspace_bytes(max(int(n), 1))
    key = (str(device), _lib.stream(device).value)
    buf = _MAP_WS.get(key)
    if buf is None or buf.numel() < need:
        buf = torch.empty((need,), dtype=torch.uint8, device=device)
        _MAP_WS[key] = buf
    return buf


def _down_sample(points: torch.Tensor, voxel_size: float, value) -> torch.Tensor:
    p = points.detach().to(torch.float32).contiguous()
    _lib.require_device(p)
    n = p.shape[0]
    if n == 0:
        raise RuntimeError("voxel_down_sample: empty point cloud (the reference's min() raises too)")
    v = value.detach().to(device=p.device, dtype=torch.float32).contiguous() if value is not None else None
    out = torch.empty((n,), dtype=torch.int64, device=p.device)
    cnt = torch.empty((1,), dtype=torch.int64, device=p.device)
    _lib.call("pin_voxel_down_sample", _lib.ptr(p), n, float(np.float32(voxel_size)), _lib.ptr(v), _lib.ptr(out),
              _lib.ptr(cnt), _lib.ptr(map_workspace(n, p.device)), _lib.stream())
    return out[:int(cnt.item())]


def voxel_down_sample(points: torch.Tensor, voxel_size: float) -> torch.Tensor:
    """Index of one point per voxel: the one closest to the voxel centre after quantising the
    distance to 1000 levels, lowest index on ties, in ascending voxel-key order
    (utils/tools.py:409-442, including its flattened key built with the single extent
    grid.max()).  HIP: pin_voxel_down_sample."""
    return _down_sample(points, voxel_size, None)


def voxel_down_sample_min_value(points: torch.Tensor, voxel_size: float, value: torch.Tensor) -> torch.Tensor:
    """One point per voxel with the minimum quantised value (utils/tools.py:444-477)."""
    return _down_sample(points, voxel_size, value)


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


def _view_key(t):
    """View-cache key of a tensor the raw-pointer views read: identity and storage, plus the
    version when the view holds a converted copy instead of the tensor itself."""
    if t is None:
        return None
    d = t.data if isinstance(t, nn.Parameter) else t
    inplace = d.dtype == torch.float32 and d.is_contiguous()
    return (id(t), d.data_ptr(), None if inplace else d._version)


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
        self._trust_table()   # an empty table over no points

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
    _NBHD_FIELDS = ("neighbor_dx", "neighbor_K", "max_valid_dist2", "neighbor_window", "_cells_host", "_cells",
                    "_offsets", "_num_columns", "_grid_exact")

    def set_search_neighborhood(self, num_nei_cells: int = 1, search_alpha: float = 1.0):
        """model/neural_points.py:430-457.  Each neighbourhood's tables are built once and kept:
        Mapper.process_frame switches to the 1-cell neighbourhood and back every frame."""
        self._save_neighborhood()
        # the tables also depend on the resolution (max_valid_dist2), the table size (slot offsets,
        # grid exactness) and the device they live on
        key = (int(num_nei_cells), float(search_alpha), float(self.resolution), int(self.buffer_size),
               str(self.primes.device))
        self._nbhd_key = key
        hit = self.__dict__.setdefault("_nbhd_cache", {}).get(key)
        if hit is not None:
            self._set_plain(hit)
            return
        dx = neighbor_offsets(num_nei_cells, search_alpha)          # host, then one copy
        self.neighbor_dx = dx.to(self.primes.device)
        self.neighbor_K = dx.shape[0]
        self.max_valid_dist2 = 3 * ((num_nei_cells + 1) * self.resolution) ** 2
        dx_host = np.ascontiguousarray(dx.numpy().astype(np.int32))
        self.neighbor_window = int(np.abs(dx_host).max()) if dx_host.size else 0
        self._cells_host = dx_host
        self._cells = None  # device tables built lazily (need the HIP runtime)
        self._offsets = None
        self._num_columns = 0
        self._grid_exact = grid_window_collision_free(self.buffer_size, num_nei_cells)
        self._save_neighborhood()

    def _set_plain(self, fields):
        """Attribute writes without nn.Module.__setattr__'s registry checks (~3 us each, a dozen
        per frame) for names that are not parameters, buffers or submodules; others go through
        setattr as usual."""
        reg = (self._parameters, self._buffers, self._modules)
        d = self.__dict__
        for k, v in fields.items():
            if isinstance(v, (nn.Parameter, nn.Module)) or any(k in r for r in reg):
                setattr(self, k, v)
            else:
                d[k] = v

    def _save_neighborhood(self):
        key = self.__dict__.get("_nbhd_key")
        if key is not None:
            self.__dict__.setdefault("_nbhd_cache", {})[key] = {k: getattr(self, k) for k in self._NBHD_FIELDS
                                                                 if hasattr(self, k)}

    def _cell_table(self):
        if self._cells is None:
            cells = torch.empty(((self.neighbor_K + 15) // 16 * 16,), dtype=torch.int32, device=self.device)
            _lib.require_device(cells)
            _lib.call("pin_neighbor_cells", self._cells_host.ctypes.data_as(_lib.c_void_p), int(self.neighbor_K),
                      self.buffer_size, _lib.ptr(cells), _lib.stream())
            self._cells = cells
            self._save_neighborhood()
        return self._cells

    def _offset_table(self):
        """Packed (dx+128) | (dy+128)<<8 | (dz+128)<<16 per neighbour cell, reference order, padded
        to 16 entries, then the column table of PinGrid.num_columns (see neighbor_columns)."""
        if self._offsets is None:
            dx = self._cells_host.astype(np.int64)
            packed = (dx[:, 0] + 128) | ((dx[:, 1] + 128) << 8) | ((dx[:, 2] + 128) << 16)
            pad = np.zeros((self.neighbor_K + 15) // 16 * 16, dtype=np.int32)
            pad[:self.neighbor_K] = packed
            cols = neighbor_columns(dx) if self.neighbor_window <= 2 else None
            self._num_columns = 0 if cols is None else len(cols)
            if cols is not None:
                pad = np.concatenate([pad, np.asarray(cols, dtype=np.int64).astype(np.int32)])
            self._offsets = torch.from_numpy(pad).to(self.device)
            self._save_neighborhood()
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

    # margin of the brick box kept between builds (bricks per side, x/y and z): a moving sensor
    # grows the map by a few cells per frame, so most rebuilds fit the previous box
    GRID_BOX_MARGIN = (8, 8, 2)

    def _build_occupancy(self):
        """Occupancy bricks of the current points.  One host read per build in the common case:
        the cell bounds and the mark kernel's two counters land in one device buffer, the marking
        runs in the box kept from the previous build (exact bounds + GRID_BOX_MARGIN), and the box
        is re-sized (a second read) only when the points have left it."""
        pts = self.neural_points.contiguous()
        _lib.require_device(pts)
        res = float(np.float32(self.resolution))
        state = torch.empty(8, dtype=torch.int64, device=pts.device)    # bounds [6], marked, occupied
        _lib.call("pin_cell_bounds", _lib.ptr(pts), pts.shape[0], res, _lib.ptr(state), _lib.stream())
        box = self.__dict__.get("_grid_box")
        if box is not None:
            bricks, dims, ws = self._grid_mark(pts, res, box, state)
            b = state.cpu().tolist()
            if self._box_fits(box, b[:3], b[3:6]):
                return self._occupancy_result(bricks, dims, b[6], b[7])
        else:
            b = state.cpu().tolist()
        lo, hi = b[:3], b[3:6]
        m = self.GRID_BOX_MARGIN
        box_lo = [lo[a] - 4 * m[a] for a in range(3)]
        ext = [(hi[a] + 4 * m[a] - box_lo[a] + 1 + 3) // 4 for a in range(3)]
        if ext[0] * ext[1] * ext[2] > self.MAX_GRID_BRICKS:
            box_lo = list(lo)
            ext = [(h - l + 1 + 3) // 4 for l, h in zip(lo, hi)]
            if ext[0] * ext[1] * ext[2] > self.MAX_GRID_BRICKS:
                return None
        box = (tuple(box_lo), tuple(ext))
        self._grid_box = box
        bricks, dims, ws = self._grid_mark(pts, res, box, state)
        marked, occupied = state[6:8].cpu().tolist()
        return self._occupancy_result(bricks, dims, marked, occupied)

    # The table is "trusted" when this object wrote it from the current positions (insert,
    # kept-points re-hash, rebuild) and neither tensor changed since: every occupied slot then
    # holds a point of its own cell, and the exactness check needs no pass over the B slots.
    def _trust_table(self):
        pts, tab = self.neural_points, self.buffer_pt_index
        self._table_trust = None if tab is None else (weakref.ref(pts), pts._version, weakref.ref(tab), tab._version)

    def _table_trusted(self):
        t = self.__dict__.get("_table_trust")
        if t is None:
            return False
        pr, pv, tr, tv = t
        return pr() is self.neural_points and pv == self.neural_points._version and \
            tr() is self.buffer_pt_index and tv == self.buffer_pt_index._version

    @staticmethod
    def _box_fits(box, lo, hi):
        (ox, oy, oz), (ex, ey, ez) = box
        return all(lo[a] >= o and hi[a] < o + 4 * e for a, o, e in zip(range(3), (ox, oy, oz), (ex, ey, ez)))

    def _grid_mark(self, pts, res, box, state):
        (ox, oy, oz), (ex, ey, ez) = box
        nb = ex * ey * ez
        dims = _lib.PinGridDims(ox=ox, oy=oy, oz=oz, nbx=ex, nby=ey, nbz=ez, reserved=0)
        bricks = torch.empty((nb, 4), dtype=torch.int32, device=pts.device)
        ws = torch.empty(((nb + 4095) // 4096 * 4 + 16,), dtype=torch.uint8, device=pts.device)
        flags = _lib.PIN_GRID_TABLE_TRUSTED if self._table_trusted() else 0
        _lib.call("pin_grid_mark_ex", _lib.ptr(pts), pts.shape[0], res, _lib.ptr(self.buffer_pt_index),
                  self.buffer_size, ctypes.byref(dims), _lib.ptr(bricks), _lib.ptr(state[6:8]), _lib.ptr(ws), flags,
                  _lib.stream())
        return bricks, dims, ws

    @staticmethod
    def _occupancy_result(bricks, dims, marked, occupied):
        if marked != occupied:   # table entries away from their point's own slot: hash path only
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
        # pin_grid_fill writes every one of the n_occ entries exactly once (each marked point its
        # rank in the brick order; marked == occupied is what made the grid exact), so only an
        # empty grid's placeholder entry needs values
        alloc = (lambda shape, dt, v: torch.empty(shape, dtype=dt, device=pts.device)) if n_occ > 0 else \
            (lambda shape, dt, v: torch.full(shape, v, dtype=dt, device=pts.device))   # noqa: E731
        crec = alloc((n, 4), torch.float32, 0.0)
        cfeat = alloc((n, 8), torch.float32, 0.0) if feats is not None else None
        ccert = alloc((n,), torch.float32, 0.0) if feats is not None else None
        cgid = alloc((n,), torch.int32, -1)
        f = feats.detach().contiguous() if feats is not None else None
        c = cert.detach().contiguous() if cert is not None else None
        _lib.call("pin_grid_fill", _lib.ptr(pts), pts.shape[0], float(np.float32(self.resolution)),
                  _lib.ptr(self.buffer_pt_index), self.buffer_size, ctypes.byref(dims), _lib.ptr(bricks),
                  _lib.ptr(rec), _lib.ptr(f), _lib.ptr(c), _lib.ptr(crec), _lib.ptr(cfeat), _lib.ptr(ccert),
                  _lib.ptr(cgid), _lib.stream())
        return crec, cfeat, ccert, cgid

    def grid_view(self, mode: str, fat: bool):
        """PinGrid view of a query mode, reused while the occupancy grid, the compact records and the
        neighbourhood tables it points into are the same objects."""
        occ = self.occupancy()
        comp = self.compact_records(mode, fat)
        offs = self._offset_table()
        key = (id(occ), id(comp), id(offs), self.neighbor_window, self._num_columns, os.environ.get("PIN_GRID_SCAN"))
        hit = self.__dict__.setdefault("_grid_view_cache", {}).get((mode, bool(fat)))
        if hit is not None and hit[0] == key:
            return hit[1]
        v = self._grid_view(occ, comp, offs, fat)
        self._grid_view_cache[(mode, bool(fat))] = (key, v)
        return v

    def _grid_view(self, occ, comp, offs, fat):
        from .query import _View
        bricks, dims, n_occ = occ
        crec, cfeat, ccert, cgid = comp
        g = _lib.PinGrid(bricks=bricks.data_ptr(), dims=dims, crec=crec.data_ptr(), cgid=cgid.data_ptr(),
                         n_occ=n_occ, offsets=offs.data_ptr(), resolution=float(np.float32(self.resolution)),
                         num_cells=int(self.neighbor_K), max_valid_dist2=float(np.float32(self.max_valid_dist2)),
                         cfeat=cfeat.data_ptr() if cfeat is not None else None,
                         ccert=ccert.data_ptr() if ccert is not None else None, fat=int(fat), window=99 if os.environ.get("PIN_GRID_SCAN") == "cells" else self.neighbor_window,
                         num_columns=0 if os.environ.get("PIN_GRID_SCAN") == "bricks" else self._num_columns)
        return _View(g, (bricks, crec, cfeat, ccert, cgid, offs, occ, comp))

    # ------------------------------------------------------------------ map maintenance
    def _travel_dist_dev(self, device):
        if self.travel_dist is None:
            raise TypeError("NeuralPoints.travel_dist is not set (the reference indexes it here too)")
        return self._cached("travel_dist_f32", (self.travel_dist,), (str(device),),
                            lambda: self.travel_dist.detach().to(device=device, dtype=torch.float32).contiguous())

    def _map_arrays(self, local: bool = False, features: bool = True) -> _lib.PinMapArrays:
        """PinMapArrays over the global (or local) tensors; every one must be contiguous."""
        if local:
            ts = (None, self.local_point_orientations, None, self.local_point_ts_update, self.local_point_certainties,
                  self.local_geo_features.data if features else None)
            pos, count = self.local_neural_points, self.local_neural_points.shape[0]
        else:
            ts = (None, self.point_orientations, self.point_ts_create, self.point_ts_update, self.point_certainties,
                  self.geo_features.data if features else None)
            pos, count = self.neural_points, self.neural_points.shape[0]
        for t in (pos,) + ts[1:]:
            if t is not None and not t.is_contiguous():
                raise ValueError("pin_slam_amd: map tensors must be contiguous")
        ptr = lambda t: t.data_ptr() if t is not None and t.numel() else None  # noqa: E731
        return _lib.PinMapArrays(positions=ptr(pos), orientations=ptr(ts[1]), ts_create=ptr(ts[2]),
                                 ts_update=ptr(ts[3]), certainties=ptr(ts[4]), features=ptr(ts[5]), count=count,
                                 feature_dim=self.geo_feature_dim, reserved=0)

    def _select_global(self, rows: torch.Tensor, n: int):
        """Replace every per-point array by its rows ``rows[:n]`` (features keep the padding row)."""
        dev = self.neural_points.device
        F = self.geo_feature_dim
        out = dict(pos=torch.empty((n, 3), dtype=self.dtype, device=dev),
                   quat=torch.empty((n, 4), dtype=self.dtype, device=dev),
                   tc=torch.empty((n,), dtype=torch.long, device=dev), tu=torch.empty((n,), dtype=torch.long, device=dev),
                   cert=torch.empty((n,), dtype=self.dtype, device=dev),
                   feat=torch.empty((n + 1, F), dtype=self.dtype, device=dev))
        dst = _lib.PinMapArrays(positions=out["pos"].data_ptr(), orientations=out["quat"].data_ptr(),
                                ts_create=out["tc"].data_ptr(), ts_update=out["tu"].data_ptr(),
                                certainties=out["cert"].data_ptr(), features=out["feat"].data_ptr(), count=n,
                                feature_dim=F, reserved=0)
        src = self._map_arrays()
        _lib.call("pin_map_gather", ctypes.byref(src), _lib.ptr(rows), n, 1, ctypes.byref(dst), _lib.stream())
        self.neural_points, self.point_orientations = out["pos"], out["quat"]
        self.point_ts_create, self.point_ts_update = out["tc"], out["tu"]
        self.point_certainties, self.geo_features = out["cert"], out["feat"]

    def update(self, points: torch.Tensor, sensor_position: torch.Tensor, sensor_orientation: torch.Tensor, cur_ts):
        """model/neural_points.py:205-270: voxel down-sample, hash probe, insert new points
        (free slot, collision or stale), last-writer-wins slot assignment, padded features.
        HIP: pin_voxel_down_sample + pin_map_insert; one host sync for the number of new points."""
        res = self.resolution
        pts = points.detach().to(self.dtype).contiguous()
        _lib.require_device(pts)
        dev = pts.device
        sidx = voxel_down_sample(pts, res)
        n = sidx.shape[0]
        M = self.count()
        td = self._travel_dist_dev(dev) if M > 0 else None
        if td is not None and not 0 <= int(cur_ts) < td.shape[0]:
            raise IndexError("travel_dist has no entry for cur_ts=%d" % int(cur_ts))
        new_rows = torch.empty((max(n, 1),), dtype=torch.int64, device=dev)
        n_new = torch.empty((1,), dtype=torch.int64, device=dev)
        was_trusted = self._table_trusted()   # an insert keeps an exact table exact
        _lib.call("pin_map_insert", _lib.ptr(pts), _lib.ptr(sidx), n, float(np.float32(res)),
                  _lib.ptr(self.buffer_pt_index), self.buffer_size, _lib.ptr(self.neural_points) if M else None,
                  _lib.ptr(self.point_ts_update) if M else None, M, _lib.ptr(td), int(cur_ts),
                  float(np.float32(3 * res ** 2)), float(np.float32(self.diff_travel_dist_local)), _lib.ptr(new_rows),
                  _lib.ptr(n_new), _lib.ptr(map_workspace(n, dev)), _lib.stream())
        torch.autograd.graph.increment_version(self.buffer_pt_index)
        k = int(n_new.item())
        # the reference's torch.cat of each per-point array (:225-242), appended in place into
        # buffers with spare capacity (_append_rows): no per-frame copy of the whole map and no
        # allocator growth as the map grows (a growing torch.cat needed a fresh, larger block from
        # time to time -- a ~10 ms frame)
        self._set_plain(dict(neural_points=self._append_rows("neural_points", self.neural_points, pts[new_rows[:k]])))
        if was_trusted:
            self._trust_table()
        # the new rows' initial values written straight into the appended rows (no temporaries and
        # copies): identity quaternions, the frame's ts, zero certainty, and padded features drawn
        # as the reference draws them -- randn(k + 1, F) from the same generator, times the std
        std, ts_val = self.geo_feature_std, int(cur_ts)

        def quat(v):
            v.zero_()
            v[:, 0] = 1.0

        def feats(v):
            torch.randn(v.shape, out=v, dtype=self.dtype, device=dev)
            v.mul_(std)
        self._set_plain(dict(
            point_orientations=self._append_rows("point_orientations", self.point_orientations, None, fill=(k, quat)),
            point_ts_create=self._append_rows("point_ts_create", self.point_ts_create, None,
                                              fill=(k, lambda v: v.fill_(ts_val))),
            point_ts_update=self._append_rows("point_ts_update", self.point_ts_update, None,
                                              fill=(k, lambda v: v.fill_(ts_val))),
            geo_features=self._append_rows("geo_features", self.geo_features, None, replace_last=True,
                                           fill=(k + 1, feats)),
            point_certainties=self._append_rows("point_certainties", self.point_certainties, None,
                                                fill=(k, lambda v: v.zero_()))))
        self.reset_local_map(sensor_position, sensor_orientation, cur_ts)

    def _append_rows(self, name, cur, new, replace_last=False, fill=None):
        """torch.cat((cur, new)) -- or torch.cat((cur[:-1], new)) with replace_last (the padding
        feature row) -- as a prefix view of a buffer with spare rows, written in place when cur is
        the view this method returned last time (anything else, e.g. an array a caller assigned,
        is copied once into a new buffer with 1.25x the rows).  The rows of cur are not touched,
        except the padding row with replace_last, whose old tensor then gets a version bump.
        fill=(m, fn) instead of new: m rows of cur's dtype, written by fn(view of those rows)."""
        bufs = self.__dict__.setdefault("_row_bufs", {})
        buf, last = bufs.get(name, (None, None))
        n = cur.shape[0] - (1 if replace_last else 0)
        m = new.shape[0] if fill is None else int(fill[0])
        dt = cur.dtype if fill is not None else torch.promote_types(cur.dtype, new.dtype)
        dev = cur.device if fill is not None else new.device
        in_place = (buf is not None and last is not None and last() is cur and buf.dtype == dt
                    and buf.shape[1:] == cur.shape[1:] and buf.shape[0] >= n + m and cur.is_contiguous()
                    and (cur.shape[0] == 0 or cur.data_ptr() == buf.data_ptr()))
        if not in_place:
            rows = max(int((n + m) * 1.25), n + m, 1024)
            buf = torch.empty((rows,) + tuple(cur.shape[1:]), dtype=dt, device=dev)
            buf[:n] = cur[:n]
        elif replace_last:
            torch.autograd.graph.increment_version(cur)
        if fill is None:
            buf[n:n + m] = new
        elif m > 0:
            fill[1](buf[n:n + m])
        out = buf[:n + m]
        bufs[name] = (buf, weakref.ref(out))
        return out

    def reset_local_map(self, sensor_position: torch.Tensor, sensor_orientation: torch.Tensor, cur_ts: int,
                        use_travel_dist: bool = True, diff_ts_local: int = 50):
        """model/neural_points.py:272-313.  HIP: pin_local_map (mask, global2local, row list)
        + pin_map_gather of the local arrays; one host sync for the local count."""
        self.cur_ts = cur_ts
        self.max_ts = max(self.max_ts, cur_ts)
        dev = self.neural_points.device
        _lib.require_device(self.neural_points)
        M = self.count()
        sensor = torch.as_tensor(sensor_position).detach().to(dev).reshape(-1)[:3]
        f64 = sensor.dtype == torch.float64
        sensor = sensor.to(torch.float64 if f64 else torch.float32).contiguous()
        td = self._travel_dist_dev(dev) if (use_travel_dist and M > 0) else None
        if td is not None and not 0 <= int(cur_ts) < td.shape[0]:
            raise IndexError("travel_dist has no entry for cur_ts=%d" % int(cur_ts))
        mask = torch.empty((M + 1,), dtype=torch.uint8, device=dev)
        g2l = torch.empty((M + 1,), dtype=torch.int64, device=dev)
        rows = torch.empty((max(M, 1),), dtype=torch.int64, device=dev)
        cnt = torch.empty((1,), dtype=torch.int64, device=dev)
        fill = -1 if self.strict_global2local else 1  # see module docstring (reference quirk)
        src = self._map_arrays()
        _lib.call("pin_local_map", ctypes.byref(src), _lib.ptr(td), _lib.ptr(sensor), int(f64), int(cur_ts),
                  float(self.local_map_radius) ** 2, float(np.float32(self.diff_travel_dist_local)),
                  int(bool(self.config.use_mid_ts)), int(bool(use_travel_dist)), int(diff_ts_local), fill,
                  _lib.ptr(mask), _lib.ptr(g2l), _lib.ptr(rows), _lib.ptr(cnt), _lib.ptr(map_workspace(M, dev)),
                  _lib.stream())
        L = int(cnt.item())
        F = self.geo_feature_dim
        lpos = torch.empty((L, 3), dtype=self.dtype, device=dev)
        lquat = torch.empty((L, 4), dtype=self.dtype, device=dev)
        lcert = torch.empty((L,), dtype=self.dtype, device=dev)
        lts = torch.empty((L,), dtype=torch.long, device=dev)
        lfeat = torch.empty((L + 1, F), dtype=self.dtype, device=dev)
        dst = _lib.PinMapArrays(positions=lpos.data_ptr(), orientations=lquat.data_ptr(), ts_create=None,
                                ts_update=lts.data_ptr(), certainties=lcert.data_ptr(), features=lfeat.data_ptr(),
                                count=L, feature_dim=F, reserved=0)
        _lib.call("pin_map_gather", ctypes.byref(src), _lib.ptr(rows), L, 1, ctypes.byref(dst), _lib.stream())
        lmask = mask.view(torch.bool)
        self._set_plain(dict(local_neural_points=lpos, local_point_orientations=lquat, local_point_certainties=lcert,
                             local_point_ts_update=lts, local_mask=lmask, global2local=g2l,
                             local_orientation=sensor_orientation, _local_rows=(lmask, rows[:L])))
        self.local_geo_features = nn.Parameter(lfeat)
        self._local_snapshot = self._snapshot()

    # derived state rebuilt on demand: weak references, capacity buffers and views keyed on tensor
    # identity, none of which pickles (weakref) or means anything in another process
    _TRANSIENT = ("_cache", "_nbhd_cache", "_grid_box", "_table_trust", "_grid_view_cache", "_row_bufs",
                  "_local_snapshot", "_local_rows", "_view_cache")

    def __getstate__(self):
        """Pickling (the reference's save_implicit_map, utils/tools.py:224-238, torch.saves the
        NeuralPoints object itself): the map without its transient caches, and every array that is
        a prefix view of a capacity buffer (_append_rows) saved as its own rows only."""
        state = dict(self.__dict__)
        for k in self._TRANSIENT:
            state.pop(k, None)
        state["_cache"] = {}

        def own(t):
            if isinstance(t, torch.Tensor) and t.untyped_storage().nbytes() != t.numel() * t.element_size():
                c = t.detach().clone()
                return nn.Parameter(c, requires_grad=t.requires_grad) if isinstance(t, nn.Parameter) else c
            return t
        for k, v in list(state.items()):
            state[k] = own(v)
        for group in ("_parameters", "_buffers"):
            if group in state:
                state[group] = {k: own(v) for k, v in state[group].items()}
        return state

    def _snapshot(self):
        """Identity + version of the position / orientation tensors right after reset_local_map:
        while both the global and the local copies are untouched, writing the local copy back
        (assign_local_to_global) is an exact no-op and is skipped, so derived indexes built over
        ``neural_points`` (records, occupancy grid) stay valid across mapping() calls."""
        ts = (self.neural_points, self.local_neural_points, self.point_orientations, self.local_point_orientations)
        return tuple((weakref.ref(t), t._version) for t in ts)

    @staticmethod
    def mark_modified(*tensors):
        """Bump the version of tensors a kernel wrote through raw pointers (features by Adam,
        certainty / ts side effects), so the derived caches keyed on ``_version`` (the fat compact
        records) are rebuilt before the next query reads them."""
        for t in tensors:
            if t is not None and t.numel():
                torch.autograd.graph.increment_version(t)

    def _unchanged_since_reset(self, idx):
        snap = getattr(self, "_local_snapshot", None)
        if snap is None:
            return False
        ts = (self.neural_points, self.local_neural_points, self.point_orientations, self.local_point_orientations)
        return all(snap[i][0]() is ts[i] and ts[i]._version == snap[i][1] for i in idx)

    def _local_row_list(self):
        lr = getattr(self, "_local_rows", None)
        if lr is not None and lr[0] is self.local_mask:
            return lr[1]
        return torch.nonzero(self.local_mask[:-1]).flatten()

    def assign_local_to_global(self):
        """model/neural_points.py:315-324.  HIP: one pin_map_scatter over the local rows; the
        position / orientation write-back is skipped while it is an exact no-op."""
        rows = self._local_row_list()
        L = rows.shape[0]
        write_pos = not self._unchanged_since_reset((0, 1))
        write_quat = not self._unchanged_since_reset((2, 3))
        src = self._map_arrays(local=True)
        if not write_pos:
            src.positions = None
        if not write_quat:
            src.orientations = None
        dst = self._map_arrays()
        _lib.call("pin_map_scatter", ctypes.byref(src), _lib.ptr(rows), L, 1, ctypes.byref(dst), _lib.stream())
        changed = [self.geo_features, self.point_certainties, self.point_ts_update]
        changed += [self.neural_points] if write_pos else []
        changed += [self.point_orientations] if write_quat else []
        for t in changed:
            torch.autograd.graph.increment_version(t)
        self._local_snapshot = self._snapshot()

    def prune_map(self, prune_certainty_thre):
        """model/neural_points.py:329-353.  HIP: pin_prune_rows + pin_map_gather."""
        dev = self.neural_points.device
        M = self.count()
        td = self._travel_dist_dev(dev)
        keep = torch.empty((max(M, 1),), dtype=torch.int64, device=dev)
        cnt = torch.empty((1,), dtype=torch.int64, device=dev)
        src = self._map_arrays(features=False)
        _lib.call("pin_prune_rows", ctypes.byref(src), _lib.ptr(td), int(self.cur_ts),
                  float(np.float32(self.diff_travel_dist_local)), float(np.float32(prune_certainty_thre)),
                  _lib.ptr(keep), _lib.ptr(cnt), _lib.ptr(map_workspace(M, dev)), _lib.stream())
        kept = int(cnt.item())
        count = M - kept
        if count > 100:
            if not self.silence:
                print("# Prune neural points: ", count)
            self._select_global(keep, kept)
            return True
        return False

    def adjust_map(self, pose_diff_torch):
        """model/neural_points.py:355-370: move every point by the pose correction of its frame
        (new tensors, as the reference assigns new ones).  HIP: pin_map_adjust."""
        self.after_pgo = True
        dev = self.neural_points.device
        T = pose_diff_torch.detach().to(device=dev, dtype=torch.float32).contiguous()
        pos = self.neural_points.clone()
        quat = self.point_orientations.to(torch.float32).clone()
        arr = _lib.PinMapArrays(positions=pos.data_ptr() if pos.numel() else None,
                                orientations=quat.data_ptr() if quat.numel() else None,
                                ts_create=self.point_ts_create.data_ptr() if pos.numel() else None,
                                ts_update=self.point_ts_update.data_ptr() if pos.numel() else None,
                                certainties=None, features=None, count=pos.shape[0], feature_dim=0, reserved=0)
        _lib.call("pin_map_adjust", ctypes.byref(arr), _lib.ptr(T), T.shape[0], int(bool(self.config.use_mid_ts)),
                  _lib.stream())
        self.neural_points = pos
        self.point_orientations = quat.to(self.dtype)

    def recreate_hash(self, sensor_position: torch.Tensor, sensor_orientation: torch.Tensor,
                      kept_points: bool = True, with_ts: bool = True, cur_ts=0):
        """model/neural_points.py:372-428.  HIP: pin_voxel_down_sample (min-value form), then
        pin_hash_assign (kept points) or pin_map_gather + pin_hash_rebuild (merge)."""
        res = self.resolution
        dev = self.neural_points.device
        self.buffer_pt_index.fill_(-1)
        if with_ts:
            if self.config.use_mid_ts:
                ts_used = ((self.point_ts_create + self.point_ts_update) / 2).long()
            else:
                ts_used = self.point_ts_create
            value = torch.abs(ts_used - cur_ts).float()
        else:
            value = -self.point_certainties
        sample_idx = voxel_down_sample_min_value(self.neural_points, res, value)
        n = sample_idx.shape[0]
        # the reference's key divides by value.max() (utils/tools.py:459): at 0 the quantised values
        # are inf / NaN and the wrapped amin keys yield indices outside the map, which its
        # neural_points[sample_idx] rejects with IndexError (neural_points.py:397 / :407); the
        # kernels must never gather them
        if n and int(sample_idx.max()) >= self.count():
            raise IndexError("recreate_hash: the down-sample returned an index outside the map "
                             "(value.max() == 0 in voxel_down_sample_min_value, as in the reference)")
        if kept_points:
            pts = self.neural_points.contiguous()
            _lib.call("pin_hash_assign", _lib.ptr(pts), _lib.ptr(sample_idx), n, float(np.float32(res)),
                      _lib.ptr(self.buffer_pt_index), self.buffer_size, _lib.ptr(map_workspace(n, dev)),
                      _lib.stream())
            torch.autograd.graph.increment_version(self.buffer_pt_index)
            self._trust_table()
        else:
            self._select_global(sample_idx, n)
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
        torch.autograd.graph.increment_version(self.buffer_pt_index)
        self._trust_table()

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
        self._local_rows = None
        self._cache = {}
        if clean_more:
            self.point_ts_create = None
            self.point_ts_update = None
            self.point_certainties = None

    # ------------------------------------------------------------------ queries
    def _views(self, mode: str, query_locally: bool):
        """(PinHash view, PinPoints view) of a query mode, reused while every tensor they are built
        from is the same (see the key below) -- a query call then costs no view rebuild."""
        rec = self.records(mode)
        if query_locally:
            src = (self.local_geo_features, self.local_neural_points, self.local_point_orientations,
                   self.local_point_certainties)
        else:
            src = (self.geo_features, self.neural_points, self.point_orientations, self.point_certainties)
        # the local map's positions also as 16-B rows: the training forward (mapping, local rows)
        # reads every neighbour's position by id beside its feature rows (cached on the positions)
        p4 = None
        if query_locally and src[1] is not None and src[1].shape[0] > 0:
            pos = src[1]
            p4 = self._cached("positions4_local", (pos,), (),
                              lambda: torch.nn.functional.pad(pos.detach().to(torch.float32), (0, 1)).contiguous())
        # the views hold raw pointers: a tensor the kernels read in place keys the view by identity
        # and storage only (its content may change -- Adam writes the features every iteration
        # -- without a rebuild); one the view copies (not f32-contiguous) by its version too
        key = (mode, bool(query_locally), bool(self.after_pgo), tensor_key((rec, self.buffer_pt_index)),
               tuple(_view_key(t) for t in src), id(p4), float(self.resolution), int(self.buffer_size),
               int(self.neighbor_K), float(self.max_valid_dist2), id(self._cells))
        hit = self.__dict__.setdefault("_view_cache", {}).get((mode, bool(query_locally)))
        if hit is not None and hit[0] == key:
            return hit[1]
        hv = hash_view(self)
        f = src[0].data if isinstance(src[0], nn.Parameter) else src[0]
        pv = points_view(rec, f, src[1], src[2], src[3], self.after_pgo, positions4=p4)
        # the key is taken after hash_view, which may build the cell table
        key = key[:-1] + (id(self._cells),)
        self._view_cache[(mode, bool(query_locally))] = (key, (hv, pv))
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
            self.mark_modified(cert_t, ts_t)
        return geo_vec, None, weights.unsqueeze(-1), nn_counts, certainty

    def get_map_o3d_bbx(self):
        raise NotImplementedError("open3d visualisation helpers are out of scope")

    def get_neural_points_o3d(self, *args, **kwargs):
        raise NotImplementedError("open3d visualisation helpers are out of scope")
