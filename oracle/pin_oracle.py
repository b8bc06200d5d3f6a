"""CPU oracle: a numpy restatement of PIN-SLAM's neural-point query hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``pin_slam_amd`` may import this module;
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg use it, and only as the checker / the timed CPU baseline.

Pinned against the reference: ``tests/test_oracle_golden.py`` checks every
function here against ``tests/golden/*.npz``, which ``tests/golden/gen_golden.py``
produced by running the reference code itself (torch CPU) in the build container.

Semantics follow the reference file:line cited on each function.  Arithmetic is
float32 where the reference's discrete decisions depend on it (voxel floor, the
squared distance that gates validity and the k-NN order, ReLU masks) and the
same op order as the reference where practical; reductions may differ in the
last bits (the tests state their tolerances).
"""
from __future__ import annotations

import dataclasses
from typing import Optional

import numpy as np

PRIMES = np.array([73856093, 19349669, 83492791], dtype=np.int64)  # model/neural_points.py:69
IDW_EPS = 1e-15                                                    # model/neural_points.py:618
INVALID_DIST2 = 9e3                                                # model/neural_points.py:561


# ---------------------------------------------------------------- neighbourhood / hash
def neighbor_offsets(num_nei_cells: int, search_alpha: float) -> np.ndarray:
    """model/neural_points.py:430-453: integer offsets inside the (c+alpha) sphere, meshgrid 'ij' order."""
    d = np.arange(-num_nei_cells, num_nei_cells + 1, dtype=np.int64)
    gx, gy, gz = np.meshgrid(d, d, d, indexing="ij")
    dx = np.stack([gx, gy, gz], -1).reshape(-1, 3)
    dx2 = (dx ** 2).sum(-1)
    return dx[dx2 < (num_nei_cells + search_alpha) ** 2]


def max_valid_dist2(num_nei_cells: int, resolution: float) -> float:
    """model/neural_points.py:457."""
    return 3 * ((num_nei_cells + 1) * resolution) ** 2


def voxel_coords(points: np.ndarray, resolution: float) -> np.ndarray:
    """model/neural_points.py:465 / :214: f32 true division, floor, to int64."""
    res = np.float32(resolution)
    return np.floor(points.astype(np.float32) / res).astype(np.int64)


def hash_slots(cells: np.ndarray, buffer_size: int) -> np.ndarray:
    """model/neural_points.py:472 + the index wrap of :476: fmod keeps the dividend's
    sign; a negative remainder r indexes slot B + r (Python negative indexing)."""
    h = np.fmod((cells * PRIMES).sum(-1), np.int64(buffer_size))
    return np.where(h < 0, h + buffer_size, h)


# ---------------------------------------------------------------- map state
@dataclasses.dataclass
class MapState:
    """Plain-array snapshot of the NeuralPoints tensors the query path reads
    (model/neural_points.py:73-95, :293-311)."""
    resolution: float
    buffer_size: int
    table: np.ndarray                 # [B] int64, -1 = empty
    points: np.ndarray                # [M,3] f32
    orientations: np.ndarray          # [M,4] f32 (w,x,y,z)
    geo_features: np.ndarray          # [M+1,F] f32 (last row = padding)
    ts_create: np.ndarray             # [M] int64
    ts_update: np.ndarray             # [M] int64
    certainties: np.ndarray           # [M] f32
    travel_dist: np.ndarray           # [T] f32
    cur_ts: int
    diff_travel_dist_local: float
    local_mask: np.ndarray            # [M+1] bool
    global2local: np.ndarray          # [M+1] int64
    local_points: np.ndarray
    local_orientations: np.ndarray
    local_features: np.ndarray        # [L+1,F]
    local_certainties: np.ndarray
    local_ts_update: np.ndarray
    after_pgo: bool = False

    def copy(self) -> "MapState":
        return dataclasses.replace(self, **{f.name: (getattr(self, f.name).copy()
                                                      if isinstance(getattr(self, f.name), np.ndarray)
                                                      else getattr(self, f.name))
                                             for f in dataclasses.fields(self)})


def table_from_slots(buffer_size: int, slots: np.ndarray, vals: np.ndarray) -> np.ndarray:
    t = np.full(int(buffer_size), -1, dtype=np.int64)
    t[slots] = vals
    return t


def build_table(points: np.ndarray, resolution: float, buffer_size: int) -> np.ndarray:
    """Hash every point into a fresh table, last writer wins (neural_points.py:420-422)."""
    t = np.full(int(buffer_size), -1, dtype=np.int64)
    slots = hash_slots(voxel_coords(points, resolution), buffer_size)
    t[slots] = np.arange(points.shape[0], dtype=np.int64)
    return t


def reset_local_map(st: MapState, sensor_position: np.ndarray, cur_ts: int, local_map_radius: float,
                    use_mid_ts: bool = False) -> None:
    """model/neural_points.py:272-311 (travel-distance form)."""
    st.cur_ts = int(cur_ts)
    d2 = ((st.points - sensor_position.astype(np.float32)) ** 2).sum(-1)
    ts_used = _ts_used(st, use_mid_ts)
    dtd = np.abs(st.travel_dist[cur_ts] - st.travel_dist[ts_used])
    mask = (d2 < local_map_radius ** 2) & (dtd < st.diff_travel_dist_local)
    st.local_points = st.points[mask]
    st.local_orientations = st.orientations[mask]
    st.local_certainties = st.certainties[mask]
    st.local_ts_update = st.ts_update[mask]
    mask = np.concatenate([mask, [True]])
    st.local_mask = mask
    # reference quirk (neural_points.py:301): non-local points map to local index 1
    g2l = np.full(mask.shape[0], 1, dtype=np.int64)
    li = np.nonzero(mask)[0]
    g2l[li] = np.arange(li.shape[0])
    g2l[-1] = -1
    st.global2local = g2l
    st.local_features = st.geo_features[mask].copy()


def assign_local_to_global(st: MapState) -> None:
    """model/neural_points.py:315-324."""
    m = st.local_mask
    st.points[m[:-1]] = st.local_points
    st.orientations[m[:-1]] = st.local_orientations
    st.geo_features[m] = st.local_features
    st.certainties[m[:-1]] = st.local_certainties
    st.ts_update[m[:-1]] = st.local_ts_update


# ---------------------------------------------------------------- search
def radius_neighborhood_search(st: MapState, q: np.ndarray, neighbor_dx: np.ndarray, maxd2: float,
                               time_filtering: bool = False):
    """model/neural_points.py:459-509 -> (dist2 [N,Kc] f32, idx [N,Kc] int64 global)."""
    q = q.astype(np.float32)
    g = voxel_coords(q, st.resolution)
    cells = g[:, None, :] + neighbor_dx[None]
    idx = st.table[hash_slots(cells, st.buffer_size)].copy()
    if time_filtering:
        dtd = np.abs(st.travel_dist[st.cur_ts] - st.travel_dist[st.ts_create[idx]])
        idx[~(dtd < st.diff_travel_dist_local)] = -1
    diff = st.points[idx] - q[:, None, :]
    dist2 = (diff * diff).sum(-1, dtype=np.float32)
    dist2[idx == -1] = np.float32(maxd2)
    idx[dist2 > np.float32(maxd2)] = -1
    return dist2, idx


def quat_rotate_passive(quat: np.ndarray, v: np.ndarray) -> np.ndarray:
    """utils/tools.py:316-323: p' = q* p q (rotation by the conjugate)."""
    w = quat[..., :1]
    u = -quat[..., 1:]
    t = 2.0 * np.cross(u, v)
    return v + w * t + np.cross(u, t)


def quat_to_rotmat(quat: np.ndarray) -> np.ndarray:
    """Active rotation matrix R(q); the passive form above is R(q)^T v."""
    w, x, y, z = [quat[..., i].astype(np.float64) for i in range(4)]
    R = np.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1)
    return R.reshape(quat.shape[:-1] + (3, 3))


@dataclasses.dataclass
class Query:
    feat: np.ndarray          # [N,F+3] (weighted_first) or [N,k,F+3]
    weights: np.ndarray       # [N,k] f32
    nn_counts: np.ndarray     # [N] int64
    certainty: np.ndarray     # [N] f32
    idx: np.ndarray           # [N,k] int64 (local or global index, -1 invalid)
    dist2: np.ndarray         # [N,k] f32
    vec: np.ndarray           # [N,k,3] f32 (after optional rotation, zero for invalid)
    nbr_points: np.ndarray    # [N,k,3] f32 neighbour positions read through the (local) index
    nbr_gpoints: np.ndarray   # [N,k,3] f32 positions of the GLOBAL candidate the distance came from
    nbr_quat: np.ndarray      # [N,k,4]
    nbr_feat: np.ndarray      # [N,k,F]


def ref_sort_row(vals, stats=None, raw=False) -> list:
    """The column order torch's CPU sort(stable=False) leaves one row in: libstdc++ std::sort
    (introsort -- median-of-three quicksort down to runs of 16, heapsort past 2 floor(log2 n)
    levels, then an insertion sort) with a plain less-than on the values (aten SortingKernel), as
    the reference's k-NN sort runs it (model/neural_points.py:562).  Equal values end up in an
    order that depends on the whole row, which is what this restatement reproduces."""
    k = list(vals) if raw else [float(v) for v in vals]   # raw: keys compared as given (adversary tests)
    g = list(range(len(k)))
    n = len(k)

    def swap(a, b):
        k[a], k[b] = k[b], k[a]
        g[a], g[b] = g[b], g[a]

    def adjust_heap(f, h, ln, vk, vg):          # __adjust_heap + __push_heap
        top, c = h, h
        while c < (ln - 1) // 2:
            c = 2 * (c + 1)
            if k[f + c] < k[f + c - 1]:
                c -= 1
            k[f + h], g[f + h] = k[f + c], g[f + c]
            h = c
        if ln % 2 == 0 and c == (ln - 2) // 2:
            c = 2 * (c + 1)
            k[f + h], g[f + h] = k[f + c - 1], g[f + c - 1]
            h = c - 1
        parent = (h - 1) // 2
        while h > top and k[f + parent] < vk:
            k[f + h], g[f + h] = k[f + parent], g[f + parent]
            h = parent
            parent = (h - 1) // 2
        k[f + h], g[f + h] = vk, vg

    def heap_sort(f, l):                         # __partial_sort(first, last, last)
        if stats is not None:
            stats["heap"] = stats.get("heap", 0) + 1
        ln = l - f
        if ln >= 2:
            parent = (ln - 2) // 2
            while True:
                adjust_heap(f, parent, ln, k[f + parent], g[f + parent])
                if parent == 0:
                    break
                parent -= 1
        while l - f > 1:
            l -= 1
            vk, vg = k[l], g[l]
            k[l], g[l] = k[f], g[f]
            adjust_heap(f, 0, l - f, vk, vg)

    def linear_insert(i):                        # __unguarded_linear_insert
        vk, vg = k[i], g[i]
        j = i - 1
        while vk < k[j]:
            k[i], g[i] = k[j], g[j]
            i, j = j, j - 1
        k[i], g[i] = vk, vg

    def insertion_sort(f, l):
        for i in range(f + 1, l):
            if k[i] < k[f]:
                vk, vg = k[i], g[i]
                k[f + 1:i + 1], g[f + 1:i + 1] = k[f:i], g[f:i]
                k[f], g[f] = vk, vg
            else:
                linear_insert(i)

    def introsort_loop(f, l, depth):
        while l - f > 16:
            if depth == 0:
                heap_sort(f, l)
                return
            depth -= 1
            a, b, c = f + 1, f + (l - f) // 2, l - 1      # __move_median_to_first
            if k[a] < k[b]:
                swap(f, b) if k[b] < k[c] else (swap(f, c) if k[a] < k[c] else swap(f, a))
            elif k[a] < k[c]:
                swap(f, a)
            elif k[b] < k[c]:
                swap(f, c)
            else:
                swap(f, b)
            lo, hi = f + 1, l                              # __unguarded_partition
            while True:
                while k[lo] < k[f]:
                    lo += 1
                hi -= 1
                while k[f] < k[hi]:
                    hi -= 1
                if not lo < hi:
                    break
                swap(lo, hi)
                lo += 1
            introsort_loop(lo, l, depth)
            l = lo

    if n > 1:
        introsort_loop(0, n, 2 * (n.bit_length() - 1))
        if n > 16:
            insertion_sort(0, 16)
            for i in range(16, n):
                linear_insert(i)
        else:
            insertion_sort(0, n)
    return g


def ref_sort_order(d2: np.ndarray) -> np.ndarray:
    """np.argsort(d2, axis=1) in the reference's order (ref_sort_row): rows whose valid
    distances are all distinct take a stable argsort (any sort agrees there up to the order of
    the 9e3 entries, which hold no neighbour); rows with equal valid distances are redone."""
    order = np.argsort(d2, axis=1, kind="stable")
    s = np.take_along_axis(d2, order, 1)
    tied = ((s[:, 1:] == s[:, :-1]) & (s[:, 1:] < INVALID_DIST2)).any(1)
    for r in np.nonzero(tied)[0]:
        order[r] = ref_sort_row(d2[r])
    return order


def query_feature(st: MapState, q: np.ndarray, nn_k: int, neighbor_dx: np.ndarray, maxd2: float,
                  weighted_first: bool = True, training_mode: bool = False, query_locally: bool = True,
                  query_ts: Optional[np.ndarray] = None, time_filtering: bool = True) -> Query:
    """model/neural_points.py:528-674.  Training-mode side effects update ``st`` in place."""
    q = q.astype(np.float32)
    N = q.shape[0]
    d2, idx = radius_neighborhood_search(st, q, neighbor_dx, maxd2, time_filtering and query_locally)
    gidx = idx
    if query_locally:
        # NB neural_points.py:301 builds global2local with full_like(<bool mask>, -1).long(),
        # i.e. every non-local point maps to local index 1 (not -1).  The fixture arrays carry
        # that exact table; distances (and their gradient) still come from the global point.
        idx = st.global2local[idx]
    nn_counts = (idx >= 0).sum(-1).astype(np.int64)
    d2 = d2.copy()
    d2[idx == -1] = np.float32(INVALID_DIST2)
    order = ref_sort_order(d2)   # torch.sort(dists2, dim=1): the reference's order of equal distances
    d2 = np.take_along_axis(d2, order, 1)[:, :nn_k]
    idx = np.take_along_axis(idx, order, 1)[:, :nn_k]
    gidx = np.take_along_axis(gidx, order, 1)[:, :nn_k]
    nbr_gpts = st.points[gidx]
    valid = idx >= 0
    if query_locally:
        feats_src, pts_src, quat_src, cert_src = (st.local_features, st.local_points,
                                                  st.local_orientations, st.local_certainties)
    else:
        feats_src, pts_src, quat_src, cert_src = (st.geo_features, st.points, st.orientations, st.certainties)
    F = feats_src.shape[1]
    nbr_feat = np.zeros((N, nn_k, F), np.float32)
    nbr_feat[valid] = feats_src[idx[valid]]
    nbr_pts = pts_src[idx]
    nbr_quat = quat_src[idx]
    certainty = cert_src[idx].copy()
    vec = (q[:, None, :] - nbr_pts).astype(np.float32)
    if st.after_pgo:
        vec = quat_rotate_passive(nbr_quat, vec).astype(np.float32)
    vec[~valid] = 0.0
    fv = np.concatenate([nbr_feat, vec], -1)
    w = (np.float32(1.0) / (d2 + np.float32(IDW_EPS))).astype(np.float32)
    w[~valid] = 0.0
    w[nn_counts == 0] = np.float32(IDW_EPS)
    w = (w / w.sum(1, keepdims=True, dtype=np.float32)).astype(np.float32)
    w[~valid] = 0.0
    if training_mode:
        sidx = idx.copy()
        sidx[~valid] = 0
        if query_locally:
            np.add.at(st.local_certainties, sidx.ravel(), w.ravel())
            if query_ts is not None:
                tsr = np.repeat(np.asarray(query_ts, np.int64)[:, None], nn_k, 1)
                tsr[~valid] = 0
                np.maximum.at(st.local_ts_update, sidx.ravel(), tsr.ravel())
        else:
            np.add.at(st.certainties, sidx.ravel(), w.ravel())
    certainty[~valid] = 0.0
    qc = (certainty * w).sum(1, dtype=np.float32)
    if weighted_first:
        fv = (fv * w[..., None]).sum(1, dtype=np.float32)
    return Query(fv, w, nn_counts, qc, idx, d2, vec, nbr_pts, nbr_gpts, nbr_quat, nbr_feat)


# ---------------------------------------------------------------- decoder + gradient
@dataclasses.dataclass
class MLP:
    """model/decoder.py:16-57 with hidden_level=1: Linear(F+3,H)+ReLU, Linear(H,1), * sdf_scale."""
    W1: np.ndarray  # [H, D]
    b1: np.ndarray  # [H]
    W2: np.ndarray  # [1, H]
    b2: np.ndarray  # [1]
    sdf_scale: float

    def forward(self, x: np.ndarray):
        """model/decoder.py:66-88. Returns (sdf [...], pre-activation [..., H])."""
        pre = (x.astype(np.float32) @ self.W1.T.astype(np.float32) + self.b1).astype(np.float32)
        h = np.maximum(pre, 0)
        out = (h @ self.W2.T + self.b2)[..., 0].astype(np.float32)
        return (out * np.float32(self.sdf_scale)).astype(np.float32), pre

    def grad_x(self, pre: np.ndarray) -> np.ndarray:
        """d sdf / d x for each row: s * W1^T (w2 * 1[pre > 0]) (ReLU'(0) = 0)."""
        gh = (pre > 0) * self.W2[0].astype(np.float64)
        return (gh @ self.W1.astype(np.float64)) * float(self.sdf_scale)


def _weight_grads(qry: Query, q: np.ndarray):
    """du_k/dq = -2 u_k^2 (q - p_k) for valid k; returns (u, S, du) in float64."""
    valid = qry.idx >= 0
    d = qry.dist2.astype(np.float64)
    u = np.where(valid, 1.0 / (d + IDW_EPS), 0.0)
    S = u.sum(1)
    diff = q.astype(np.float64)[:, None, :] - qry.nbr_gpoints.astype(np.float64)
    du = (-2.0 * u * u)[..., None] * diff
    du[~valid] = 0.0
    return u, S, du


def _vec_jacobian_t(qry: Query, st_after_pgo: bool, gv: np.ndarray) -> np.ndarray:
    """(d vec_k / d q)^T gv : identity, or R(q_k) gv after pgo (vec = R^T (q - p))."""
    if not st_after_pgo:
        return gv
    R = quat_to_rotmat(qry.nbr_quat)
    return np.einsum("...ij,...j->...i", R, gv)


def sdf_and_grad(st: MapState, mlp: MLP, q: np.ndarray, nn_k: int, neighbor_dx: np.ndarray, maxd2: float,
                 weighted_first: bool = True, query_locally: bool = True, zero_empty: bool = False):
    """SDF, analytic dSDF/dq (what utils/tools.py:174 get_gradient returns through autograd at
    utils/tracker.py:252), per-neighbour weighted std (utils/tracker.py:245-249) and the
    query outputs.  ``zero_empty`` gives rows with nn_count == 0 sdf 0 (mesher, utils/mesher.py:96-103)."""
    qry = query_feature(st, q, nn_k, neighbor_dx, maxd2, weighted_first, False, query_locally)
    valid = qry.idx >= 0
    u, S, du = _weight_grads(qry, q)
    Ssafe = np.where(S > 0, S, 1.0)
    w64 = qry.weights.astype(np.float64)
    F = qry.nbr_feat.shape[-1]
    if weighted_first:
        sdf, pre = mlp.forward(qry.feat)
        gx = mlp.grad_x(pre)                                               # [N, F+3]
        fv = np.concatenate([qry.nbr_feat, qry.vec], -1).astype(np.float64)  # [N,k,F+3]
        a = (fv * gx[:, None, :]).sum(-1)                                  # [N,k]
        abar = (a * w64).sum(1)
        g1 = (((a - abar[:, None]) * valid)[..., None] * du).sum(1) / Ssafe[:, None]
        gv = np.broadcast_to(gx[:, None, F:], qry.vec.shape)
        g2 = (w64[..., None] * _vec_jacobian_t(qry, st.after_pgo, gv)).sum(1)
        grad = g1 + g2
        std = np.zeros(q.shape[0], np.float32)
    else:
        sdf_k, pre = mlp.forward(qry.feat)                                 # [N,k]
        mean = (sdf_k * qry.weights).sum(1, dtype=np.float32)
        var = (qry.weights * (sdf_k - mean[:, None]) ** 2).sum(1, dtype=np.float32)
        std = np.sqrt(var).astype(np.float32)
        gx = mlp.grad_x(pre)                                               # [N,k,F+3]
        s64 = sdf_k.astype(np.float64)
        sbar = (s64 * w64).sum(1)
        g1 = (((s64 - sbar[:, None]) * valid)[..., None] * du).sum(1) / Ssafe[:, None]
        g2 = (w64[..., None] * _vec_jacobian_t(qry, st.after_pgo, gx[..., F:])).sum(1)
        grad = g1 + g2
        sdf = mean
    empty = qry.nn_counts == 0
    grad[empty] = 0.0
    if zero_empty:
        sdf = np.where(empty, np.float32(0), sdf)
    return sdf.astype(np.float32), grad.astype(np.float32), std, qry


# ---------------------------------------------------------------- mapper (utils/mapper.py:425-593)
def bce_with_logits_grad(pred: np.ndarray, label: np.ndarray, sigma: float):
    """utils/loss.py:40-47 (unweighted, mean): loss and dL/dpred."""
    p = pred.astype(np.float64) / sigma
    y = 1.0 / (1.0 + np.exp(-label.astype(np.float64) / sigma))
    loss = np.mean(np.maximum(p, 0) - p * y + np.log1p(np.exp(-np.abs(p))))
    dp = (1.0 / (1.0 + np.exp(-p)) - y) / (pred.shape[0] * sigma)
    return loss, dp


def numerical_grad_points(x: np.ndarray, eps: float) -> np.ndarray:
    """utils/mapper.py:683-711: two-sided stencil, blocks ordered x+,x-,y+,y-,z+,z-."""
    out = []
    for a in range(3):
        e = np.zeros(3, np.float32)
        e[a] = np.float32(eps)
        out.append(x + e)
        out.append(x - e)
    return np.concatenate(out, 0).astype(np.float32)


def _mlp_backward(mlp: MLP, x: np.ndarray, pre: np.ndarray, dsdf: np.ndarray):
    """Accumulate MLP parameter grads and return dL/dx for rows x with upstream dsdf."""
    s = float(mlp.sdf_scale)
    d_out = dsdf.astype(np.float64) * s                                   # dL/d(lout output)
    h = np.maximum(pre.astype(np.float64), 0)
    dh = d_out[:, None] * mlp.W2[0].astype(np.float64)[None] * (pre > 0)
    gW2 = (d_out[:, None] * h).sum(0)[None]
    gb2 = np.array([d_out.sum()])
    gW1 = dh.T @ x.astype(np.float64)
    gb1 = dh.sum(0)
    dx = dh @ mlp.W1.astype(np.float64)
    return dx, dict(W1=gW1, b1=gb1, W2=gW2, b2=gb2)


def mapper_forward_backward(st: MapState, mlp: MLP, coord: np.ndarray, label: np.ndarray, ts: np.ndarray,
                            nn_k: int, neighbor_dx: np.ndarray, maxd2: float, weighted_first: bool,
                            sigma: float, weight_e: float, decimation: int, eps: float):
    """One mapping iteration up to the backward pass (utils/mapper.py:448-572): training-mode
    queries (main batch with ts, then the numerical-gradient stencil without ts), BCE +
    weight_e * eikonal, gradients w.r.t. local features [L+1,F] and MLP params."""
    N = coord.shape[0]
    Lp1, F = st.local_features.shape
    qm = query_feature(st, coord, nn_k, neighbor_dx, maxd2, weighted_first, True, True, ts)
    xd = coord[::decimation]
    Nd = xd.shape[0]
    qs_pts = numerical_grad_points(xd, eps)
    qn = query_feature(st, qs_pts, nn_k, neighbor_dx, maxd2, weighted_first, True, True, None)

    def predict(qry):
        if weighted_first:
            sdf, pre = mlp.forward(qry.feat)
            return sdf, pre
        sdf_k, pre = mlp.forward(qry.feat)
        return (sdf_k * qry.weights).sum(1, dtype=np.float32), pre

    sdf_m, pre_m = predict(qm)
    sdf_n, pre_n = predict(qn)
    sp = sdf_n.astype(np.float64).reshape(6, Nd)
    g = np.stack([(sp[0] - sp[1]), (sp[2] - sp[3]), (sp[4] - sp[5])], 1) / (2 * eps)
    gn = np.linalg.norm(g, axis=1)
    loss_bce, d_m = bce_with_logits_grad(sdf_m, label, sigma)
    loss = loss_bce + weight_e * np.mean((gn - 1.0) ** 2)
    dg = weight_e * 2.0 * (gn - 1.0)[:, None] * g / np.where(gn > 0, gn, 1.0)[:, None] / Nd
    d_n = np.zeros((6, Nd))
    for a in range(3):
        d_n[2 * a] = dg[:, a] / (2 * eps)
        d_n[2 * a + 1] = -dg[:, a] / (2 * eps)
    d_n = d_n.reshape(-1)
    feat_grad = np.zeros((Lp1, F))
    grads = dict(W1=0.0, b1=0.0, W2=0.0, b2=0.0)
    for qry, pre, dsdf in ((qm, pre_m, d_m), (qn, pre_n, d_n)):
        valid = qry.idx >= 0
        if weighted_first:
            dx, gp = _mlp_backward(mlp, qry.feat, pre, dsdf)
            contrib = qry.weights.astype(np.float64)[..., None] * dx[:, None, :F]   # [n,k,F]
        else:
            n, k = qry.weights.shape
            drow = (dsdf[:, None] * qry.weights.astype(np.float64)).reshape(-1)
            dx, gp = _mlp_backward(mlp, qry.feat.reshape(n * k, -1), pre.reshape(n * k, -1), drow)
            contrib = dx.reshape(n, k, -1)[..., :F]
        np.add.at(feat_grad, qry.idx[valid], contrib[valid])
        for key in grads:
            grads[key] = grads[key] + gp[key]
    return dict(loss=loss, sdf=sdf_m, numgrad=g.astype(np.float32), feat_grad=feat_grad.astype(np.float32),
                mlp_grads={k: v.astype(np.float32) for k, v in grads.items()})


def adam_step(param: np.ndarray, grad: np.ndarray, m: np.ndarray, v: np.ndarray, step: int,
              lr: float, beta1: float = 0.9, beta2: float = 0.99, eps: float = 1e-15) -> None:
    """torch.optim.Adam single-tensor update as configured by utils/tools.py:111-112
    (betas (0.9, 0.99), eps 1e-15, no weight decay), float32 in place."""
    f = np.float32
    grad = grad.astype(np.float32)
    m += f(1 - beta1) * (grad - m)                      # exp_avg.lerp_(grad, 1-beta1)
    v *= f(beta2)
    v += f(1 - beta2) * grad * grad                     # addcmul_(grad, grad, 1-beta2)
    bc1 = 1 - beta1 ** step
    bc2s = (1 - beta2 ** step) ** 0.5
    denom = np.sqrt(v) / f(bc2s) + f(eps)
    param += f(-lr / bc1) * m / denom


# ---------------------------------------------------------------- tracker (utils/tracker.py)
def expmap(axis_angle: np.ndarray) -> np.ndarray:
    """utils/tracker.py:580-589 (Rodrigues)."""
    angle = np.linalg.norm(axis_angle)
    axis = axis_angle / angle
    S = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + S * np.sin(angle) + (S @ S) * (1.0 - np.cos(angle))


def implicit_reg(points, sdf_grad, sdf_residual, weight, lm_lambda=0.0):
    """utils/tracker.py:468-496: J = [p x g, g], N = J^T W J (+ lambda diag), t = N^-1 (-(JW)^T r)."""
    p = points.astype(np.float64)
    g = sdf_grad.astype(np.float64)
    J = np.concatenate([np.cross(p, g), g], 1)
    w = weight.astype(np.float64).reshape(-1, 1)
    Nm = J.T @ (w * J)
    Nm = Nm + lm_lambda * np.diag(np.diag(Nm))
    gv = -(J * w).T @ sdf_residual.astype(np.float64)
    t = np.linalg.inv(Nm) @ gv
    T = np.eye(4)
    T[:3, :3] = expmap(t[:3])
    T[:3, 3] = t[3:]
    return T, Nm, gv


def registration_step(st: MapState, mlp: MLP, points: np.ndarray, sdf_labels: np.ndarray, nn_k: int,
                      neighbor_dx: np.ndarray, maxd2: float, weighted_first: bool, min_grad_norm: float,
                      max_grad_norm: float, GM_dist: float, GM_grad: float, lm_lambda: float,
                      max_sdf_std: float):
    """utils/tracker.py:277-452 without colours/normals: query, validity mask, Geman-McClure
    weights normalised by 2*mean, implicit_reg."""
    sdf, grad, std, qry = sdf_and_grad(st, mlp, points, nn_k, neighbor_dx, maxd2, weighted_first, True)
    mask = qry.nn_counts >= nn_k
    gnorm = np.linalg.norm(grad.astype(np.float64), axis=1)
    valid = mask & (gnorm < max_grad_norm) & (gnorm > min_grad_norm) & (std < max_sdf_std)
    cnt = int(valid.sum())
    if cnt < 10:
        return np.eye(4), cnt, 0.0, valid, None, None
    r = sdf[valid].astype(np.float64) - sdf_labels[valid]
    ga = gnorm[valid] - 1.0
    w = (GM_grad / (GM_grad ** 2 + ga ** 2)) ** 2 * (GM_dist / (GM_dist ** 2 + r ** 2)) ** 2
    w = w / (2.0 * w.mean())
    T, Nm, gv = implicit_reg(points[valid], grad[valid], r, w, lm_lambda)
    return T, cnt, float(np.mean(np.abs(r)) * 100.0), valid, Nm, gv


# ---------------------------------------------------------------- mesher (utils/mesher.py:41-136)
def mesher_query_points(st: MapState, mlp: MLP, coord: np.ndarray, nn_k: int, neighbor_dx: np.ndarray,
                        maxd2: float, weighted_first: bool, mask_min_nn_count: int):
    qry = query_feature(st, coord, nn_k, neighbor_dx, maxd2, weighted_first, False, False)
    if weighted_first:
        sdf, _ = mlp.forward(qry.feat)
    else:
        sdf_k, _ = mlp.forward(qry.feat)
        sdf = (sdf_k * qry.weights).sum(1, dtype=np.float32)
    sdf = np.where(qry.nn_counts >= 1, sdf, np.float32(0)).astype(np.float32)
    return sdf, qry.nn_counts >= mask_min_nn_count


def query_certainty(st: MapState, q: np.ndarray, resolution: float) -> np.ndarray:
    """model/neural_points.py:511-525 with the own-voxel neighbourhood (utils/mapper.py:283)."""
    dx = neighbor_offsets(1, 0.0)
    _, idx = radius_neighborhood_search(st, q, dx, max_valid_dist2(1, resolution), False)
    c = st.certainties[idx]
    c[idx < 0] = 0.0
    return c.max(-1)


# ---------------------------------------------------------------- map maintenance
INT64_MIN = np.iinfo(np.int64).min


def to_long(x) -> np.ndarray:
    """torch CPU float32 -> int64 (``.long()``): truncation toward zero; NaN, +-inf and values
    outside int64 give INT64_MIN (x86 cvttss2si "integer indefinite")."""
    x = np.asarray(x, np.float32)
    ok = np.isfinite(x) & (np.abs(x) < np.float32(2.0 ** 63))
    out = np.full(x.shape, INT64_MIN, np.int64)
    out[ok] = x[ok].astype(np.int64)
    return out


def voxel_down_sample(points: np.ndarray, voxel_size: float, value: Optional[np.ndarray] = None) -> np.ndarray:
    """utils/tools.py:409-442 (value None: closest to the voxel centre) and :444-477 (smallest
    value): one index per voxel in ascending flattened-key order.  Keeps the reference's
    v_size = grid.max() key (which aliases c0 = v with c1 + 1), the 1000-level quantisation
    and the packed "index + level * 10^digits" amin with int64 wrap-around."""
    p = np.asarray(points, np.float32)
    vs = np.float32(voxel_size)
    n = p.shape[0]
    grid = np.floor(p / vs)
    offset = np.floor(p.min(0) / vs).astype(np.int64)
    if value is None:
        d = p - (grid + np.float32(0.5)) * vs
        src = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])
    else:
        src = np.asarray(value, np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        level = src / src.max() * np.float32(999)
    c = grid.astype(np.int64) - offset
    v = c.max()
    key = c[:, 0] + c[:, 1] * v + c[:, 2] * v * v
    uniq, inv = np.unique(key, return_inverse=True)
    scale = 10 ** len(str(n - 1))
    with np.errstate(over="ignore"):
        packed = np.arange(n, dtype=np.int64) + to_long(level) * np.int64(scale)
    best = np.full(uniq.shape[0], np.iinfo(np.int64).max, np.int64)
    np.minimum.at(best, inv.reshape(-1), packed)
    return np.mod(best, np.int64(scale))


def _ts_used(st: MapState, use_mid_ts: bool) -> np.ndarray:
    """((ts_create + ts_update) / 2).long(): true division to float32, truncation."""
    if use_mid_ts:
        return to_long((st.ts_create + st.ts_update).astype(np.float32) / np.float32(2))
    return st.ts_create


def empty_map(resolution: float, buffer_size: int, travel_dist: np.ndarray, diff_travel_dist_local: float,
              feature_dim: int = 8) -> MapState:
    z = np.zeros
    return MapState(resolution=resolution, buffer_size=int(buffer_size),
                    table=np.full(int(buffer_size), -1, np.int64), points=z((0, 3), np.float32),
                    orientations=z((0, 4), np.float32), geo_features=z((1, feature_dim), np.float32),
                    ts_create=z(0, np.int64), ts_update=z(0, np.int64), certainties=z(0, np.float32),
                    travel_dist=np.asarray(travel_dist, np.float32), cur_ts=0,
                    diff_travel_dist_local=float(diff_travel_dist_local), local_mask=z(1, bool),
                    global2local=z(1, np.int64), local_points=None, local_orientations=None, local_features=None,
                    local_certainties=None, local_ts_update=None)


def map_update(st: MapState, points: np.ndarray, cur_ts: int) -> np.ndarray:
    """model/neural_points.py:205-268 without the reset_local_map tail: down-sample, probe,
    insert new / collided / stale samples with consecutive ids, last writer per slot.  New
    features are zeros here (the reference draws them at random).  Returns sample_idx."""
    res = st.resolution
    sidx = voxel_down_sample(points, res)
    sp = np.asarray(points, np.float32)[sidx]
    slots = hash_slots(voxel_coords(sp, res), st.buffer_size)
    hidx = st.table[slots]
    M = st.points.shape[0]
    if M == 0:
        fresh = np.ones(sidx.shape[0], bool)
    else:
        d = st.points[hidx] - sp
        d2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        dtd = st.travel_dist[cur_ts] - st.travel_dist[st.ts_update[hidx]]
        fresh = (hidx == -1) | (d2 > np.float32(3 * res ** 2)) | (dtd > np.float32(st.diff_travel_dist_local))
    added = sp[fresh]
    k = added.shape[0]
    cur = hidx.copy()
    cur[fresh] = np.arange(k, dtype=np.int64) + M
    st.table[slots] = cur  # repeated slots: the last assignment stays (CPU index_put order)
    st.points = np.concatenate([st.points, added])
    quat = np.zeros((k, 4), np.float32)
    quat[:, 0] = 1.0
    st.orientations = np.concatenate([st.orientations, quat])
    st.ts_create = np.concatenate([st.ts_create, np.full(k, cur_ts, np.int64)])
    st.ts_update = np.concatenate([st.ts_update, np.full(k, cur_ts, np.int64)])
    st.certainties = np.concatenate([st.certainties, np.zeros(k, np.float32)])
    st.geo_features = np.concatenate([st.geo_features[:-1], np.zeros((k + 1, st.geo_features.shape[1]), np.float32)])
    return sidx


def prune_keep(st: MapState, thre: float) -> np.ndarray:
    """model/neural_points.py:329-337: the rows prune_map keeps."""
    dtd = np.abs(st.travel_dist[st.cur_ts] - st.travel_dist[st.ts_update])
    prune = (dtd > np.float32(st.diff_travel_dist_local)) & (st.certainties < np.float32(thre))
    return ~prune


def select_rows(st: MapState, rows: np.ndarray) -> None:
    """Index selection of every per-point array, features keeping the padding row."""
    st.points = st.points[rows]
    st.orientations = st.orientations[rows]
    st.ts_create = st.ts_create[rows]
    st.ts_update = st.ts_update[rows]
    st.certainties = st.certainties[rows]
    st.geo_features = st.geo_features[np.concatenate([rows, [-1]])]


def recreate_hash(st: MapState, cur_ts: int, kept_points: bool, with_ts: bool, use_mid_ts: bool = False) -> None:
    """model/neural_points.py:372-426 (the reset_local_map tail is the caller's)."""
    res = st.resolution
    st.table = np.full(st.buffer_size, -1, np.int64)
    if with_ts:
        value = np.abs(_ts_used(st, use_mid_ts) - cur_ts).astype(np.float32)
    else:
        value = -st.certainties
    sidx = voxel_down_sample(st.points, res, value)
    if kept_points:
        slots = hash_slots(voxel_coords(st.points[sidx], res), st.buffer_size)
        st.table[slots] = sidx
    else:
        select_rows(st, sidx)
        st.table = build_table(st.points, res, st.buffer_size)


def rotmat_to_quat(R: np.ndarray) -> np.ndarray:
    """utils/tools.py:326-334."""
    R = R.astype(np.float32)
    qw = np.sqrt(np.float32(1.0) + R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2]) / np.float32(2.0)
    qx = (R[:, 2, 1] - R[:, 1, 2]) / (np.float32(4.0) * qw)
    qy = (R[:, 0, 2] - R[:, 2, 0]) / (np.float32(4.0) * qw)
    qz = (R[:, 1, 0] - R[:, 0, 1]) / (np.float32(4.0) * qw)
    return np.stack([qw, qx, qy, qz], 1)


def quat_multiply(q1: np.ndarray, q2: np.ndarray) -> np.ndarray:
    """utils/tools.py:356-369."""
    w1, x1, y1, z1 = q1.T
    w2, x2, y2, z2 = q2.T
    return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], 1)


def adjust_map(st: MapState, pose_diff: np.ndarray, use_mid_ts: bool = False) -> None:
    """model/neural_points.py:355-370 with transform_batch_torch (utils/tools.py:401-407)."""
    used = _ts_used(st, use_mid_ts)
    T = pose_diff.astype(np.float32)[used]
    p = st.points
    st.points = ((T[:, :3, 0] * p[:, 0:1] + T[:, :3, 1] * p[:, 1:2]) + T[:, :3, 2] * p[:, 2:3]) + T[:, :3, 3]
    dq = rotmat_to_quat(pose_diff[:, :3, :3])
    st.orientations = quat_multiply(dq[used], st.orientations).astype(np.float32)


# ---------------------------------------------------------------- training samples
def fma32(a, b, c):
    """f32 fused multiply-add (the f32 product is exact in f64; the sum is rounded once more
    to f32 -- double rounding can differ from a true fma in rare halfway cases)."""
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(np.float32)


def sample_rays(points: np.ndarray, randn_surface: np.ndarray, rand_front: np.ndarray, rand_behind: np.ndarray,
                surface_n: int, front_n: int, behind_n: int, surface_range: float, front_min_ratio: float,
                end_dist: float, dist_weight_on: bool, dist_weight_scale: float, max_range: float,
                behind_dropoff_on: bool):
    """utils/data_sampler.py:20-192 (DataSampler.sample) given its random draws, in f32 with the
    reference's op order.  Python-double scalar subexpressions are rounded once to f32 (as
    torch does when they meet a float tensor); ``scalar / tensor`` is Tensor.__rtruediv__ =
    reciprocal(tensor) * scalar.  Returns (coord [N*A,3], sdf_label [N*A], weight [N*A]) in the
    final ray-wise order (:165-171)."""
    f = np.float32
    p = points.astype(f)
    n = p.shape[0]
    d = np.sqrt(fma32(p[:, 2], p[:, 2], fma32(p[:, 1], p[:, 1], p[:, 0] * p[:, 0])))   # :43, torch's CPU norm
    inv = f(1.0) / d
    two_range = f(2.0 * surface_range)
    disp_parts, ratio_parts, surf_parts = [np.zeros(n, f)], [np.ones(n, f)], [np.ones(n, bool)]   # :45-46
    rs = randn_surface.astype(f).reshape(surface_n, n)
    for k in range(surface_n):                                                        # :50-53
        disp = rs[k] * f(surface_range)
        disp_parts.append(disp)
        ratio_parts.append(disp / d + f(1.0))
        surf_parts.append(np.ones(n, bool))
    rf = rand_front.astype(f).reshape(front_n, n)
    for k in range(front_n):                                                          # :72-78
        fmax = f(1.0) - inv * two_range
        fdiff = fmax - f(front_min_ratio)
        ratio = rf[k] * fdiff + f(front_min_ratio)
        ratio_parts.append(ratio)
        disp_parts.append((ratio - f(1.0)) * d)
        surf_parts.append(np.zeros(n, bool))
    rb = rand_behind.astype(f).reshape(behind_n, n)
    for k in range(behind_n):                                                         # :85-91
        bmax = inv * f(end_dist) + f(1.0)
        bmin = f(1.0) + inv * two_range
        ratio = rb[k] * (bmax - bmin) + bmin
        ratio_parts.append(ratio)
        disp_parts.append((ratio - f(1.0)) * d)
        surf_parts.append(np.zeros(n, bool))
    A = 1 + surface_n + front_n + behind_n
    disp = np.stack(disp_parts, 1)          # [n, A]: ray-wise order
    ratio = np.stack(ratio_parts, 1)
    surf = np.stack(surf_parts, 1)
    coord = p[:, None, :] * ratio[..., None]                                          # :106
    w = np.ones((n, A), f)
    if dist_weight_on:                                                                # :120-121
        wd = f(1 + dist_weight_scale * 0.5) - (d / f(max_range)) * f(dist_weight_scale)
        w = np.where(surf, wd[:, None], w)
    if behind_dropoff_on:                                                             # :125-134
        dmin, dmax = 0.2 * end_dist, end_dist
        dw = (f(dmax) - disp) / f(dmax - dmin)
        dw = np.clip(dw, f(0.0), f(1.0)) * f(0.8) + f(0.2)
        w = w * dw
    w = np.where(surf, w, w * f(-1.0))                                                # :137
    return coord.reshape(n * A, 3).astype(f), (disp * f(-1.0)).reshape(-1).astype(f), w.reshape(-1).astype(f)


def transform_points(points: np.ndarray, pose: np.ndarray) -> np.ndarray:
    """utils/tools.py:386-399 transform_torch: [p, 1] @ T^T with T cast to the points' f32; the
    CPU sgemm accumulates x, y, z, 1 in order with fused multiply-adds."""
    f = np.float32
    T = pose.astype(f)
    p = points.astype(f)
    out = np.empty_like(p)
    for a in range(3):
        acc = fma32(p[:, 2], T[a, 2], fma32(p[:, 1], T[a, 1], p[:, 0] * T[a, 0]))
        out[:, a] = acc + T[a, 3]
    return out


def rotmat_to_rotvec(R: np.ndarray) -> np.ndarray:
    """roma.rotmat_to_rotvec (roma 1.x, not installed here; its published algorithm): unit
    quaternion from the largest of (trace, diagonal) branch, w >= 0, then 2 atan2(|v|, w) v/|v|."""
    R = R.astype(np.float64)
    tr = np.trace(R)
    cand = [tr, R[0, 0], R[1, 1], R[2, 2]]
    k = int(np.argmax(cand))
    if k == 0:
        q = [1 + tr, R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]
    elif k == 1:
        q = [R[2, 1] - R[1, 2], 1 + R[0, 0] - R[1, 1] - R[2, 2], R[0, 1] + R[1, 0], R[0, 2] + R[2, 0]]
    elif k == 2:
        q = [R[0, 2] - R[2, 0], R[0, 1] + R[1, 0], 1 + R[1, 1] - R[0, 0] - R[2, 2], R[1, 2] + R[2, 1]]
    else:
        q = [R[1, 0] - R[0, 1], R[0, 2] + R[2, 0], R[1, 2] + R[2, 1], 1 + R[2, 2] - R[0, 0] - R[1, 1]]
    q = np.asarray(q) / np.linalg.norm(q)
    if q[0] < 0:
        q = -q
    vn = np.linalg.norm(q[1:])
    return q[1:] * (2 * np.arctan2(vn, q[0]) / vn if vn > 1e-12 else 2.0)


def rotvec_to_rotmat(w: np.ndarray) -> np.ndarray:
    th = np.linalg.norm(w)
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-8:
        return np.eye(3) + K + 0.5 * K @ K
    return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K


def deskewing(points: np.ndarray, ts: np.ndarray, pose: np.ndarray, ts_mid_pose: float = 0.5) -> np.ndarray:
    """utils/tools.py:540-567 in f64: s = normalised ts - ts_mid; R(s) = roma.rotmat_slerp(I, R, s)
    = exp(s log R); p <- R(s) p + s t.  PARITY UNPINNED: roma is absent here, so this follows
    roma's published algorithm, not outputs of the reference."""
    t = ts.reshape(-1).astype(np.float64)
    s = (t - t.min()) / (t.max() - t.min()) - ts_mid_pose
    w = rotmat_to_rotvec(pose[:3, :3])
    out = points.astype(np.float64).copy()
    for i in range(out.shape[0]):
        out[i, :3] = rotvec_to_rotmat(s[i] * w) @ out[i, :3] + s[i] * pose[:3, 3]
    return out


# ---------------------------------------------------------------- marching cubes
MC_CORNERS = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]
MC_EDGES = [(0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 7), (7, 4), (0, 4), (1, 5), (2, 6), (3, 7)]
MC_FACES = [(0, 3, 2, 1), (4, 5, 6, 7), (0, 1, 5, 4), (3, 7, 6, 2), (0, 4, 7, 3), (1, 2, 6, 5)]


def mc_case_triangles(case: int):
    """Triangles (cube-edge triples) of one corner sign pattern (bit c: corner c below the level).
    PARITY UNPINNED against the reference: it calls skimage.measure.marching_cubes (Lewiner),
    which is not installed here.  Construction: per face (corners CCW seen from outside) the
    boundary cuts off each run of inside corners (an ambiguous face separates them); the face
    segments (from a run's exit crossing back to its entry crossing) chain into loops, each
    fan-triangulated -- right-hand normals point from inside to outside."""
    inside = [(case >> c) & 1 for c in range(8)]
    edge_of = {frozenset(e): k for k, e in enumerate(MC_EDGES)}
    nxt = {}
    for f in MC_FACES:
        cross = []
        for k in range(4):
            a, b = f[k], f[(k + 1) % 4]
            if inside[a] != inside[b]:
                cross.append((edge_of[frozenset((a, b))], inside[a]))   # inside[a]: leaving an inside run
        for k, (e, leaving) in enumerate(cross):
            if not leaving:
                nxt[cross[(k + 1) % len(cross)][0]] = e
    tris, seen = [], set()
    for start in sorted(nxt):
        if start in seen:
            continue
        loop, cur = [start], nxt[start]
        seen.add(start)
        while cur != start:
            loop.append(cur)
            seen.add(cur)
            cur = nxt[cur]
        tris += [(loop[0], loop[i + 1], loop[i]) for i in range(1, len(loop) - 1)]
    return tris


def marching_cubes(values: np.ndarray, mask: Optional[np.ndarray] = None, level: float = 0.0):
    """Marching cubes with shared vertices (one per used grid edge, id order = (grid point, axis)
    order), cubes processed iff mask at their first corner; verts in index space (f32 crossing
    arithmetic as the kernel), faces in cube order.  Degenerate triangles are kept (the caller
    filters)."""
    v = values.astype(np.float32)
    nx, ny, nz = v.shape
    f = np.float32
    lvl = f(level)
    tables = [mc_case_triangles(c) for c in range(256)]
    edge_lo = []
    for a, b in MC_EDGES:
        pa, pb = np.array(MC_CORNERS[a]), np.array(MC_CORNERS[b])
        lo = np.minimum(pa, pb)
        edge_lo.append((tuple(lo), int(np.argmax(np.abs(pb - pa)))))
    used = {}
    cube_tris = []
    below = v < lvl
    for x in range(nx - 1):
        for y in range(ny - 1):
            for z in range(nz - 1):
                if mask is not None and not mask[x, y, z]:
                    continue
                case = 0
                for c, (dx, dy, dz) in enumerate(MC_CORNERS):
                    case |= int(below[x + dx, y + dy, z + dz]) << c
                for tri in tables[case]:
                    keys = []
                    for e in tri:
                        (dx, dy, dz), ax = edge_lo[e]
                        k = (((x + dx) * ny + (y + dy)) * nz + (z + dz)) * 3 + ax
                        used[k] = True
                        keys.append(k)
                    cube_tris.append(keys)
    order = sorted(used)
    vid = {k: i for i, k in enumerate(order)}
    verts = np.zeros((len(order), 3), f)
    for i, k in enumerate(order):
        g, ax = divmod(k, 3)
        gz, g2 = g % nz, g // nz
        gy, gx = g2 % ny, g2 // ny
        va = v[gx, gy, gz]
        d = [0, 0, 0]
        d[ax] = 1
        vb = v[gx + d[0], gy + d[1], gz + d[2]]
        t = (lvl - va) / (vb - va)
        p = [f(gx), f(gy), f(gz)]
        p[ax] = f(p[ax] + t)
        verts[i] = p
    faces = np.array([[vid[k] for k in tri] for tri in cube_tris], np.int64).reshape(-1, 3)
    return verts, faces


# ---------------------------------------------------------------- fixture helpers
def map_from_fixture(z, prefix: str = "map_") -> MapState:
    g = lambda k: z[prefix + k]  # noqa: E731
    st = MapState(
        resolution=float(g("resolution")), buffer_size=int(g("buffer_size")),
        table=table_from_slots(int(g("buffer_size")), g("table_slots"), g("table_vals")),
        points=g("neural_points").astype(np.float32), orientations=g("point_orientations").astype(np.float32),
        geo_features=g("geo_features").astype(np.float32), ts_create=g("point_ts_create").astype(np.int64),
        ts_update=g("point_ts_update").astype(np.int64), certainties=g("point_certainties").astype(np.float32),
        travel_dist=g("travel_dist").astype(np.float32), cur_ts=int(g("cur_ts")),
        diff_travel_dist_local=float(g("diff_travel_dist_local")),
        local_mask=g("local_mask"), global2local=g("global2local"),
        local_points=None, local_orientations=None, local_features=None,
        local_certainties=None, local_ts_update=None)
    m = st.local_mask
    st.local_points = st.points[m[:-1]]
    st.local_orientations = st.orientations[m[:-1]]
    st.local_certainties = st.certainties[m[:-1]]
    st.local_ts_update = st.ts_update[m[:-1]]
    st.local_features = st.geo_features[m].copy()
    return st


def mlp_from_fixture(z, prefix: str = "dec_") -> MLP:
    return MLP(z[prefix + "W1"].astype(np.float32), z[prefix + "b1"].astype(np.float32),
               z[prefix + "W2"].astype(np.float32), z[prefix + "b2"].astype(np.float32),
               float(z[prefix + "sdf_scale"]))
