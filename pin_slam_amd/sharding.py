"""Owner-partitioned (spatially sharded) data-parallel mapping: SURVEY.md 8e's alternative to the
dense all-reduce of the [L+1, 8] feature gradient (128 MB per iteration at 4M points).

Every rank holds the same local map (the SLAM front end is replicated).  The local-map points
are split into W cells: a x b equal-count columns x rows in the horizontal plane (cuts from
integer histograms of the coordinates, so every rank computes the same cuts; the factor pair
with the shortest cut length).  Rank r owns cell r and draws its batches from the pool samples
inside it.  Its rows then only reach owned points, the halo (the points of other cells within
the query reach -- search radius + numerical-gradient step -- of cell r) and the shared rows
(local row 1, which the reference's global2local fill quirk makes every non-local candidate
read).  Per iteration (Mapper.mapping with shard="space"):

  1. exchange_gradients: shared rows' gradients SUM all-reduced (one 32-B row); each rank sends
     the gradient rows of its halo to their owners, which add them to their own rows
     (point-to-point with the ranks whose cells are within reach);
  2. Adam on the owned rows and the shared rows (pin_adam_rows);
  3. exchange_features: owners send the updated rows that other ranks hold as halo.

At the end of mapping(): halo certainty deltas (sum) and ts (max) go to the owners (shared rows
by all-reduce), then the owned rows of every rank are all-gathered, so every replica holds the
whole updated local map.

With the same batches this is the dense data-parallel step: an owned row's gradient is the sum
of every rank's contribution (only ranks whose cell is within reach can contribute), and Adam
is elementwise.  Wire bytes per iteration: 2 x halo rows x 32 B (about 1 MB at 4M points on 8
ranks) instead of 2 x 7/8 x 128 MB.
"""
import math

import torch
import torch.distributed as dist


def _ranks(group):
    return dist.get_world_size(group), dist.get_rank(group)


def all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None):
    """In-place all-reduce; device tensors go through host copies on gloo (CPU tests, 1-GPU
    rehearsals), directly over RCCL otherwise."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)


class OwnerAdam:
    """The dense data-parallel optimiser step of SURVEY.md 8e: reduce-scatter of the per-rank
    feature gradients -> Adam on the rank's own 1/W of the rows -> all-gather of the stepped rows.
    It replaces the reference's single-process `optimizer.step()` (utils/mapper.py:570-572, Adam
    from utils/tools.py:89-116) for W ranks that each backpropagated their own batch (loss scaled
    by 1/W, so the sum over ranks is the gradient of the mean loss of the union of the batches).
    The wire bytes equal a ring all-reduce's (reduce-scatter + all-gather), the Adam work and the
    moments are 1/W of the dense step's.

    Layout of the n = 8 (L+1) feature floats: `buckets` contiguous buckets of W pieces of `piece`
    floats (a multiple of `align`); rank r owns piece r of every bucket, so each bucket is one
    reduce_scatter_tensor / all_gather_into_tensor on contiguous memory and the buckets pipeline:
    bucket k's Adam and all-gather are issued while buckets k+1.. are still being reduced.  The
    rest -- the last n - n_main floats, fewer than buckets * W * align -- travels with the
    decoder's gradients (contiguous behind the features in the caller's buffer) in one all-reduce
    and is stepped by every rank alike.

    adam(p, g, m, v, step_state) steps one contiguous piece in place (the HIP pin_adam_step on the
    GPU, a restatement in the CPU tests: this class only moves data).  Collectives are issued with
    async_op on every backend, so gloo runs the same sequence RCCL does."""

    def __init__(self, n, group=None, buckets=4, align=64):
        self.group = group
        self.world, self.rank = _ranks(group)
        W = self.world
        self.n = int(n)
        nb = max(1, int(buckets))
        piece = (self.n // (nb * W)) // align * align
        if piece == 0:   # a map too small to split: everything travels as the all-reduced rest
            nb = 0
        self.buckets, self.piece = nb, piece
        self.n_main = nb * W * piece
        self.rest = self.n - self.n_main

    def own_slices(self):
        """(start, end) of this rank's piece of every bucket in the flat feature array."""
        W, c = self.world, self.piece
        return [(k * W * c + self.rank * c, k * W * c + (self.rank + 1) * c) for k in range(self.buckets)]

    def moments_size(self):
        """Floats of this rank's feature moments (m or v): its pieces, then the rest."""
        return self.buckets * self.piece + self.rest

    def step(self, params, grads, m, v, adam, tail_step=None):
        """One optimiser step.  params: the flat features [n]; grads: the flat gradient buffer
        [n + extra] (features, then any tail gradients such as the decoder's, contiguous), this
        rank's unreduced contribution -- zero again when the call returns; m, v: [moments_size()]
        moments of this rank's rows; tail_step(): steps the extra tail (e.g. the decoder) once
        grads[n:] holds its reduced gradient.  Leaves params identical on every rank."""
        g, W, c = self.group, self.world, self.piece
        span = W * c
        own = getattr(self, "_own", None)   # the reduced pieces, kept for the next steps
        if self.buckets and (own is None or own.device != grads.device or own.dtype != grads.dtype):
            own = self._own = grads.new_empty((self.buckets, c))
        rs = [dist.reduce_scatter_tensor(own[k], grads[k * span:(k + 1) * span], group=g, async_op=True)
              for k in range(self.buckets)]
        tail = grads[self.n_main:]
        ar = dist.all_reduce(tail, group=g, async_op=True) if tail.numel() else None
        ag = []
        for k, (a, b) in enumerate(self.own_slices()):
            rs[k].wait()                                  # bucket k reduced: its piece is in own[k]
            grads[k * span:(k + 1) * span].zero_()        # this rank's contribution consumed
            adam(params[a:b], own[k], m[k * c:(k + 1) * c], v[k * c:(k + 1) * c])
            ag.append(dist.all_gather_into_tensor(params[k * span:(k + 1) * span], params[a:b], group=g,
                                                  async_op=True))
        if ar is not None:
            ar.wait()
            if self.rest:
                o = self.buckets * c
                adam(params[self.n_main:], grads[self.n_main:self.n], m[o:], v[o:])
            if tail_step is not None:
                tail_step()
        for w in ag:
            w.wait()


def _factor_pairs(W):
    return [(a, W // a) for a in range(1, W + 1) if W % a == 0]


def _equal_count_cuts(counts_cum, total, parts, lo, span, bins):
    """parts-1 cut coordinates at histogram bin edges so that each part holds ~total/parts points
    (integer cumulative counts: every rank computes the same cuts)."""
    cuts = []
    for k in range(1, parts):
        e = int(torch.searchsorted(counts_cum, torch.tensor(k * total / parts, dtype=counts_cum.dtype)))
        cuts.append(lo + span * (e + 1) / bins)
    return cuts


class SlabPartition:
    """Ownership of the local-map rows [L, 3] (the padding feature row L is nobody's) by a grid of
    cells: the map is cut into `a` equal-count columns along x, each column into `b` equal-count
    cells along y (a x b = W, a k-d split); rank r owns cell (r // b, r % b).  layout "auto"
    picks the factor pair with the shortest total cut length ((a-1) span_y + (b-1) span_x,
    proportional to the halo volume), so 8 ranks on a square map become 4 x 2 cells instead of 8
    thin strips, and a corridor stays 1-D; "1d" cuts only along the longer horizontal axis; an
    (a, b) pair forces that grid.

    shared_rows: local rows whose gradient may come from any slab.  The reference's global2local
    table maps every non-local point to local row 1 (neural_points.py:290-300, the fill quirk):
    a non-local candidate that passes the travel filter reads and trains row 1 wherever the
    query is.  Those rows are taken out of the halo lists and handled by tiny all-reduces
    instead (gradient and certainty delta SUM, ts MAX, Adam applied by every rank)."""

    def __init__(self, positions: torch.Tensor, reach: float, group=None, bins: int = 4096, layout: str = "auto",
                 shared_rows=(1,)):
        self.group = group
        self.world, self.rank = _ranks(group)
        W = self.world
        pos = positions.detach()
        L = pos.shape[0]
        self.L = L
        dev = pos.device
        if L == 0:
            raise ValueError("SlabPartition: empty local map")
        if isinstance(layout, (tuple, list)):
            if len(layout) != 2 or int(layout[0]) * int(layout[1]) != W or min(int(v) for v in layout) < 1:
                raise ValueError(f"layout {tuple(layout)}: a x b cells must equal the world size {W}")
        elif layout not in ("auto", "1d"):
            raise ValueError("layout must be 'auto', '1d' or an (a, b) pair with a * b = world size")
        lo = pos.min(0).values.double().cpu()
        hi = pos.max(0).values.double().cpu()
        span = [max(float(hi[d] - lo[d]), 1e-9) for d in (0, 1)]
        if isinstance(layout, (tuple, list)):
            self.shape = (int(layout[0]), int(layout[1]))
        elif layout == "1d":
            self.shape = (W, 1) if span[0] >= span[1] else (1, W)
        else:
            # shortest total cut length; ties to more columns (the 1-D case along x first)
            self.shape = min(_factor_pairs(W), key=lambda ab: ((ab[0] - 1) * span[1] + (ab[1] - 1) * span[0], -ab[0]))
        a, b = self.shape
        x = pos[:, 0].double()
        y = pos[:, 1].double()
        bx = torch.clamp(((x - float(lo[0])) / span[0] * bins).long(), 0, bins - 1)
        xcum = torch.bincount(bx, minlength=bins).cumsum(0).cpu()
        self.xcuts = torch.tensor(_equal_count_cuts(xcum, L, a, float(lo[0]), span[0], bins), dtype=torch.float64)
        col = torch.bucketize(x, self.xcuts.to(dev), right=True)          # column c = [xcut_{c-1}, xcut_c)
        by = torch.clamp(((y - float(lo[1])) / span[1] * bins).long(), 0, bins - 1)
        ycnt = torch.bincount(col * bins + by, minlength=a * bins).reshape(a, bins).cpu()
        ycum = ycnt.cumsum(1)
        ycuts = [_equal_count_cuts(ycum[c], int(ycum[c, -1]), b, float(lo[1]), span[1], bins) for c in range(a)]
        self.ycuts = torch.tensor(ycuts, dtype=torch.float64).reshape(a, b - 1)
        owner = self._owner_of(x, y)
        self.owner = owner
        # cell boxes [x_lo, x_hi) x [y_lo, y_hi)
        xe = [-math.inf] + self.xcuts.tolist() + [math.inf]
        self.boxes = []
        for r in range(W):
            c, k = divmod(r, b)
            ye = [-math.inf] + self.ycuts[c].tolist() + [math.inf]
            self.boxes.append((xe[c], xe[c + 1], ye[k], ye[k + 1]))
        self.reach = float(reach)
        shared = torch.as_tensor([s for s in shared_rows if 0 <= s < L], dtype=torch.long, device=dev)
        self.shared = shared
        not_shared = torch.ones(L, dtype=torch.bool, device=dev)
        not_shared[shared] = False
        mine = owner == self.rank
        self.owned = torch.nonzero(mine).flatten()
        # Adam runs on the owned rows plus the shared rows every rank holds the summed gradient of
        self.adam_rows = torch.unique(torch.cat((self.owned, shared)))
        self.counts = torch.bincount(owner, minlength=W).cpu().tolist()
        # halo lists, ordered by row: recv_rows[s] = rows owned by s inside my reach box (I hold
        # them as halo), send_rows[s] = my rows inside s's reach box (s holds them as halo).  Both
        # sides evaluate the same predicate on the same data, so the lists pair up element by element.
        self.recv_rows, self.send_rows = {}, {}
        for s in range(W):
            if s == self.rank:
                continue
            rr = torch.nonzero((owner == s) & self._in_reach(x, y, self.rank) & not_shared).flatten()
            sr = torch.nonzero(mine & self._in_reach(x, y, s) & not_shared).flatten()
            if rr.numel() or sr.numel():
                self.recv_rows[s] = rr
                self.send_rows[s] = sr
        self.halo = torch.cat(list(self.recv_rows.values())) if self.recv_rows else \
            torch.empty(0, dtype=torch.long, device=dev)
        # the group's first collective is then never a partial point-to-point batch (torch requires
        # every rank in the first batch_isend_irecv of a group)
        dist.barrier(group=group)

    @property
    def axis(self):
        """The cut axis of a 1-D partition (None for a 2-D grid)."""
        a, b = self.shape
        return 0 if b == 1 else (1 if a == 1 else None)

    def _owner_of(self, x, y):
        a, b = self.shape
        col = torch.bucketize(x, self.xcuts.to(x.device), right=True)
        if b == 1:
            return col
        yc = self.ycuts.to(x.device)[col]                          # [n, b-1] the column's cuts
        return col * b + (y[:, None] >= yc).sum(1)

    def _in_reach(self, x, y, r):
        x0, x1, y0, y1 = self.boxes[r]
        R = self.reach
        return (x >= x0 - R) & (x < x1 + R) & (y >= y0 - R) & (y < y1 + R)

    # ------------------------------------------------------------------ samples
    def sample_mask(self, coords: torch.Tensor) -> torch.Tensor:
        """Samples whose slab (by their coordinate) is this rank's."""
        return self._owner_of(coords[:, 0].double(), coords[:, 1].double()) == self.rank

    # ------------------------------------------------------------------ point-to-point
    def _p2p(self, sends, recv_like):
        """sends[s] -> rank s, receives into recv_like[s] from rank s (every peer both ways).
        RCCL moves device tensors directly over xGMI; gloo (CPU tests, 1-GPU rehearsals) gets
        host copies."""
        ops = []
        g = self.group
        host = dist.get_backend(g) == "gloo"
        staged = {}
        for s in sorted(sends):
            dst = dist.get_global_rank(g, s) if g is not None else s
            out = sends[s].contiguous()
            inp = recv_like[s]
            if host and out.is_cuda:
                out = out.cpu()
                staged[s] = torch.empty(inp.shape, dtype=inp.dtype)
                inp = staged[s]
            # empty directions are skipped on both sides alike (the sizes pair up element by
            # element), so no zero-byte transfer reaches the backend
            if out.numel():
                ops.append(dist.P2POp(dist.isend, out, dst, g))
            if inp.numel():
                ops.append(dist.P2POp(dist.irecv, inp, dst, g))
        # one group: with RCCL, a send and a receive to the same peer issued separately can
        # deadlock (each waits behind the other on the peer's stream)
        for q in dist.batch_isend_irecv(ops) if ops else []:
            q.wait()
        for s, t in staged.items():
            recv_like[s].copy_(t)

    def exchange_gradients(self, grad: torch.Tensor):
        """Shared rows take the sum over ranks; owners add the halo holders' gradient rows
        (grad [L+1, F], in place)."""
        if self.shared.numel():
            g = grad.index_select(0, self.shared)
            all_reduce(g, group=self.group)
            grad.index_copy_(0, self.shared, g)
        if not self.recv_rows:
            return
        sends = {s: grad.index_select(0, r) for s, r in self.recv_rows.items()}
        recv = {s: grad.new_empty((self.send_rows[s].numel(),) + tuple(grad.shape[1:])) for s in self.send_rows}
        self._p2p(sends, recv)
        for s, r in self.send_rows.items():
            if r.numel():
                grad.index_add_(0, r, recv[s])

    def exchange_features(self, feats: torch.Tensor):
        """Halo copies take the owners' current rows (feats [L+1, F], in place)."""
        if not self.recv_rows:
            return
        sends = {s: feats.index_select(0, r) for s, r in self.send_rows.items()}
        recv = {s: feats.new_empty((self.recv_rows[s].numel(),) + tuple(feats.shape[1:])) for s in self.recv_rows}
        self._p2p(sends, recv)
        for s, r in self.recv_rows.items():
            if r.numel():
                feats.index_copy_(0, r, recv[s])

    def zero_halo(self, grad: torch.Tensor):
        if self.halo.numel():
            grad.index_fill_(0, self.halo, 0)

    # ------------------------------------------------------------------ end of mapping()
    def reconcile_side_effects(self, cert_before: torch.Tensor, cert: torch.Tensor, ts: torch.Tensor):
        """Owners add the halo holders' certainty deltas (scatter_add) and take the max of their
        ts (scatter_reduce amax), neural_points.py:640-644; cert / ts [L] in place on owned rows.
        Shared rows: every rank's delta summed, the max ts."""
        if self.shared.numel():
            d = cert.index_select(0, self.shared) - cert_before.index_select(0, self.shared)
            all_reduce(d, group=self.group)
            cert.index_copy_(0, self.shared, cert_before.index_select(0, self.shared) + d)
            t = ts.index_select(0, self.shared)
            all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            ts.index_copy_(0, self.shared, t)
        if not self.recv_rows:
            return
        delta = cert - cert_before
        sends = {s: delta.index_select(0, r) for s, r in self.recv_rows.items()}
        recv = {s: delta.new_empty((self.send_rows[s].numel(),)) for s in self.send_rows}
        self._p2p(sends, recv)
        sends_t = {s: ts.index_select(0, r) for s, r in self.recv_rows.items()}
        recv_t = {s: ts.new_empty((self.send_rows[s].numel(),)) for s in self.send_rows}
        self._p2p(sends_t, recv_t)
        for s, r in self.send_rows.items():
            if r.numel():
                cert.index_add_(0, r, recv[s])
                ts.index_copy_(0, r, torch.maximum(ts.index_select(0, r), recv_t[s]))

    def gather_owned(self, *arrays):
        """Every rank's owned rows of each array ([L, ...] or [L+1, ...]) to every rank, in place."""
        W = self.world
        m = max(self.counts)
        rows_of = [torch.nonzero(self.owner == s).flatten() for s in range(W)]
        for t in arrays:
            flat = t.reshape(t.shape[0], -1)
            mine = flat.new_zeros((m, flat.shape[1]))
            mine[: self.owned.numel()] = flat.index_select(0, self.owned)
            host = dist.get_backend(self.group) == "gloo" and mine.is_cuda
            src = mine.cpu() if host else mine
            out = [torch.empty_like(src) for _ in range(W)]
            dist.all_gather(out, src, group=self.group)
            if host:
                out = [o.to(mine.device) for o in out]
            for s in range(W):
                if s != self.rank and rows_of[s].numel():
                    flat.index_copy_(0, rows_of[s], out[s][: rows_of[s].numel()])


def slab_batch_plan(part, pool_coords, new_idx, bs, bs_new_sample, new_mode):
    """The batch plan of one shard="space" mapping() call on this rank (Mapper._slab_partition):
    (the slab's pool rows, the slab's new samples, scales), or None on EVERY rank when any slab
    holds no pool samples (the counts are all-reduced first, so all ranks take the same branch and
    the call falls back to the dense gradient all-reduce together).

    scales(bs_hist_r, bs_new_r) -> (history-row scale, new-row scale): the rank draws its batch from
    its slab only, so its rows are weighted to keep the union of the ranks' batches an unbiased
    estimate of the reference's single batch (utils/mapper.py:323-350: bs_hist rows uniform over
    the N pool samples, bs_new rows uniform over the n new ones):
        scale_h = (bs_hist / bs_hist_r) (N_r / N),   scale_n = (bs_new / bs_new_r) (n_r / n)."""
    mask = part.sample_mask(pool_coords)
    slab_rows = torch.nonzero(mask).flatten()
    slab_new = new_idx[mask[new_idx]] if new_idx is not None else None
    n_r = 0 if slab_new is None else int(slab_new.numel())
    cnt = torch.tensor([float(slab_rows.numel()), float(n_r), 1.0 if slab_rows.numel() == 0 else 0.0],
                       dtype=torch.float64, device=pool_coords.device)
    all_reduce(cnt, group=part.group)
    if float(cnt[2]) > 0:
        return None
    N, n = float(cnt[0]), float(cnt[1])
    N_r = float(slab_rows.numel())
    bs_new = min(int(n), int(bs_new_sample)) if (new_mode and n > 0) else 0
    bs_hist = int(bs) - bs_new

    def scales(bs_hist_r, bs_new_r):
        sh = (bs_hist / bs_hist_r) * (N_r / N) if bs_hist_r > 0 else 0.0
        sn = (bs_new / bs_new_r) * (n_r / n) if bs_new_r > 0 else 0.0
        return sh, sn
    return slab_rows, slab_new, scales


def query_reach(nm, config) -> float:
    """Farthest point a mapping row can touch along a horizontal axis: the neighbour search radius
    (sqrt(max_valid_dist2)) + the numerical-gradient step, with a margin for float rounding."""
    eps = float(config.voxel_size_m * config.num_grad_step_ratio)
    return math.sqrt(float(nm.max_valid_dist2)) * 1.001 + eps + 1e-3
