"""Owner-partitioned (spatially sharded) data-parallel mapping: SURVEY.md 8e's alternative to the
dense all-reduce of the [L+1, 8] feature gradient (128 MB per iteration at 4M points).

Every rank holds the same local map (the SLAM front end is replicated).  The local-map points
are split into W slabs along the longer horizontal axis (cuts from a histogram of the
coordinates, so every rank computes the same cuts), rank r owns slab r and draws its batches
from the pool samples inside slab r.  Its rows then only reach owned points and the halo: the
points of other slabs within the query reach (search radius + numerical-gradient step) of slab
r.  Per iteration (Mapper.mapping with shard="space"):

  1. exchange_gradients: each rank sends the gradient rows of its halo to their owners, which
     add them to their own rows (point-to-point with the ranks whose slabs are within reach);
  2. Adam on the owned rows only (pin_adam_rows);
  3. exchange_features: owners send the updated rows that other ranks hold as halo.

At the end of mapping(): halo certainty deltas (sum) and ts (max) go to the owners, then the
owned rows of every rank are all-gathered, so every replica holds the whole updated local map.

With the same batches this is the dense data-parallel step: an owned row's gradient is the sum
of every rank's contribution (only ranks whose slab is within reach can contribute), and Adam is
elementwise.  Wire bytes per iteration: 2 x halo rows x 32 B (about 1 MB at 4M points on 8
ranks) instead of 2 x 7/8 x 128 MB.
"""
import math

import torch
import torch.distributed as dist


def _ranks(group):
    return dist.get_world_size(group), dist.get_rank(group)


class SlabPartition:
    """Slab ownership of the local-map rows [L, 3] (the padding feature row L is nobody's)."""

    def __init__(self, positions: torch.Tensor, reach: float, group=None, bins: int = 4096):
        self.group = group
        self.world, self.rank = _ranks(group)
        W = self.world
        pos = positions.detach()
        L = pos.shape[0]
        self.L = L
        dev = pos.device
        if L == 0:
            raise ValueError("SlabPartition: empty local map")
        lo = pos.min(0).values.double().cpu()
        hi = pos.max(0).values.double().cpu()
        self.axis = 0 if (hi[0] - lo[0]) >= (hi[1] - lo[1]) else 1
        a = pos[:, self.axis].double()
        a_lo, a_hi = float(lo[self.axis]), float(hi[self.axis])
        span = max(a_hi - a_lo, 1e-9)
        # equal-count cuts at histogram bin edges (integer counts: identical on every rank)
        b = torch.clamp(((a - a_lo) / span * bins).long(), 0, bins - 1)
        cnt = torch.bincount(b, minlength=bins).cumsum(0).cpu()
        cuts = []
        for k in range(1, W):
            e = int(torch.searchsorted(cnt, torch.tensor(k * L / W, dtype=cnt.dtype)))
            cuts.append(a_lo + span * (e + 1) / bins)
        self.cuts = torch.tensor(cuts, dtype=torch.float64)
        self.bounds = [(-math.inf if r == 0 else cuts[r - 1], math.inf if r == W - 1 else cuts[r]) for r in range(W)]
        self.reach = float(reach)
        cuts_d = self.cuts.to(dev)
        owner = torch.bucketize(a, cuts_d, right=True)          # slab r = [cut_{r-1}, cut_r)
        self.owner = owner
        self.owned = torch.nonzero(owner == self.rank).flatten()
        self.counts = torch.bincount(owner, minlength=W).cpu().tolist()
        # halo lists, ordered by row: recv_rows[s] = rows owned by s inside my band (I hold them
        # as halo), send_rows[s] = my rows inside s's band (s holds them as halo).  Both sides
        # evaluate the same predicate on the same data, so the lists pair up element by element.
        self.recv_rows, self.send_rows = {}, {}
        mine_lo, mine_hi = self.bounds[self.rank]
        for s in range(W):
            if s == self.rank:
                continue
            s_lo, s_hi = self.bounds[s]
            rr = torch.nonzero((owner == s) & (a >= mine_lo - self.reach) & (a < mine_hi + self.reach)).flatten()
            sr = torch.nonzero((owner == self.rank) & (a >= s_lo - self.reach) & (a < s_hi + self.reach)).flatten()
            if rr.numel() or sr.numel():
                self.recv_rows[s] = rr
                self.send_rows[s] = sr
        self.halo = torch.cat(list(self.recv_rows.values())) if self.recv_rows else \
            torch.empty(0, dtype=torch.long, device=dev)
        # the group's first collective is then never a partial point-to-point batch (torch requires
        # every rank in the first batch_isend_irecv of a group)
        dist.barrier(group=group)

    # ------------------------------------------------------------------ samples
    def sample_mask(self, coords: torch.Tensor) -> torch.Tensor:
        """Samples whose slab (by their coordinate) is this rank's."""
        a = coords[:, self.axis].double()
        return torch.bucketize(a, self.cuts.to(coords.device), right=True) == self.rank

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
        """Owners add the halo holders' gradient rows (grad [L+1, F], in place)."""
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
        ts (scatter_reduce amax), neural_points.py:640-644; cert / ts [L] in place on owned rows."""
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


def query_reach(nm, config) -> float:
    """Farthest point a mapping row can touch along a horizontal axis: the neighbour search radius
    (sqrt(max_valid_dist2)) + the numerical-gradient step, with a margin for float rounding."""
    eps = float(config.voxel_size_m * config.num_grad_step_ratio)
    return math.sqrt(float(nm.max_valid_dist2)) * 1.001 + eps + 1e-3
