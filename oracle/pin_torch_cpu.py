"""PyTorch-CPU restatement of the SDF + gradient query and of one mapping iteration.

TEST INFRASTRUCTURE ONLY (like oracle/pin_oracle.py): bench.py's cpu_baseline legs time it on
the GPU box's host cores, as BASELINE.md's CPU-baseline plan specifies (all the process's cores,
one warm-up, median of 5); tests/test_oracle_golden.py pins it to the reference's fixtures.
Nothing in pin_slam_amd imports it.

The reference's hot path IS a sequence of ATen ops, so the same algorithm written as torch CPU
ops is what that path costs on a CPU.  Written from the algorithm, with
the reference's numerics where they decide results:
  model/neural_points.py:459-509  voxel floor (f32 division), int64 cell products, fmod hash with
                                  the negative-index wrap, candidate gather, distance gate
  model/neural_points.py:528-674  nn_count before truncation, torch's (unstable) sort, k nearest, IDW weights
                                  1/(d2 + 1e-15) row-normalised, training-mode certainty / ts
                                  side effects, weighted_first feature sum
  model/decoder.py:66-88          Linear(11, 64) + ReLU + Linear(64, 1), times sdf_scale
  utils/tools.py:174-184          dsdf/dq by autograd
  utils/mapper.py:443-575         batch + numerical-gradient stencil (:683-711), BCE on sdf/sigma
                                  vs sigmoid(label/sigma) (utils/loss.py:40-47) + weight_e *
                                  eikonal, backward, Adam (utils/tools.py:89-116)
"""
import torch

PRIMES = (73856093, 19349669, 83492791)   # model/neural_points.py:69


class TorchMap:
    """The tensors one query mode reads: the hash table (int64, -1 empty) over `points`, and the
    feature rows the candidates index -- global mode: the map itself; local mode
    (query_locally, the tracker / mapper): `time_ok` [M] bool, the travel-distance filter of each
    point (model/neural_points.py:480-488), `global2local` [M+1] (the reference's table, with its
    fill quirk) and the local points / features the neighbours are then read from."""

    def __init__(self, resolution, buffer_size, table, points, features, certainties, neighbor_dx, max_valid_dist2,
                 nn_k, weighted_first, time_ok=None, global2local=None, local_points=None):
        self.time_ok = time_ok
        self.g2l = global2local
        self.local_points = local_points if local_points is not None else points
        self.res = float(resolution)
        self.B = int(buffer_size)
        self.table = table.to(torch.int64)
        self.points = points.to(torch.float32)
        self.features = features.to(torch.float32)
        self.certainties = certainties.to(torch.float32)
        self.dx = torch.as_tensor(neighbor_dx, dtype=torch.int64)
        self.max_d2 = float(max_valid_dist2)
        self.nn_k = int(nn_k)
        self.wf = bool(weighted_first)
        self.primes = torch.tensor(PRIMES, dtype=torch.int64)


class TorchMLP:
    def __init__(self, W1, b1, W2, b2, sdf_scale, requires_grad=False):
        self.params = [torch.as_tensor(t, dtype=torch.float32).clone().requires_grad_(requires_grad)
                       for t in (W1, b1, W2, b2)]
        self.s = float(sdf_scale)

    def __call__(self, x):
        W1, b1, W2, b2 = self.params
        h = torch.relu(x @ W1.T + b1)
        return (h @ W2.T + b2) * self.s


def knn(m: TorchMap, q: torch.Tensor):
    """Candidates of every neighbour cell, the k nearest in cell order on ties; d2 keeps q's
    autograd history.  Returns (idx [N,k] (-1 invalid), d2 [N,k], nn_count [N])."""
    g = torch.floor(q.detach() / m.res).to(torch.int64)
    cells = g[:, None, :] + m.dx[None]
    slot = torch.fmod((cells * m.primes).sum(-1), m.B)            # negative: indexes from the end
    idx = m.table[slot]
    if m.time_ok is not None:
        idx = torch.where((idx >= 0) & m.time_ok[idx], idx, torch.full_like(idx, -1))
    d2 = ((m.points[idx] - q[:, None, :]) ** 2).sum(-1)
    bad = (idx < 0) | (d2.detach() > m.max_d2)
    idx = torch.where(bad, torch.full_like(idx, -1), idx)
    if m.g2l is not None:
        idx = m.g2l[idx]                       # g2l[-1] = -1 keeps rejected candidates rejected
        bad = idx < 0
    nn_count = (~bad).sum(-1)
    key = torch.where(bad, torch.full_like(d2.detach(), 9e3), d2.detach())
    _, order = torch.sort(key, dim=1)   # the reference's unstable sort: its order of equal distances
    order = order[:, :m.nn_k]
    return torch.gather(idx, 1, order), torch.gather(d2, 1, order), nn_count


def query(m: TorchMap, q: torch.Tensor, features=None):
    """IDW neighbour interpolation: (decoder input [N,11] or [N,k,11], weights [N,k], idx,
    nn_count)."""
    feats = m.features if features is None else features
    idx, d2, nn_count = knn(m, q)
    valid = idx >= 0
    safe = torch.where(valid, idx, torch.zeros_like(idx))
    f = feats[safe] * valid[..., None]
    vec = (q[:, None, :] - m.local_points[safe]) * valid[..., None]
    x = torch.cat((f, vec), -1)
    u = torch.where(valid, 1.0 / (d2 + 1e-15), torch.zeros_like(d2))
    u = torch.where((nn_count == 0)[:, None], torch.full_like(u, 1e-15), u)
    w = u / u.sum(1, keepdim=True)
    w = w * valid
    if m.wf:
        x = (x * w[..., None]).sum(1)
    return x, w, idx, nn_count


def predict(m: TorchMap, mlp: TorchMLP, q, features=None):
    x, w, idx, nn = query(m, q, features)
    s = mlp(x)[..., 0]
    if not m.wf:
        s = (s * w).sum(1)
    return s, w, idx, nn


def sdf_and_grad(m: TorchMap, mlp: TorchMLP, q: torch.Tensor):
    """SDF and dsdf/dq (autograd, as get_gradient) of a query batch."""
    q = q.detach().to(torch.float32).requires_grad_(True)
    s, _, _, nn = predict(m, mlp, q)
    (g,) = torch.autograd.grad(s.sum(), q)
    return s.detach(), g, nn


def mapping_iteration(m: TorchMap, mlp: TorchMLP, features: torch.nn.Parameter, opt, coord, label, sigma, weight_e,
                      decimation, eps, certainties=None):
    """One iteration of Mapper.mapping with a frozen or trainable decoder: training-mode query of
    the batch and of the numerical-gradient stencil (certainty side effect), BCE + eikonal,
    backward, optimiser step.  Returns the loss."""
    def side_effect(w, idx):
        if certainties is not None:
            ok = idx >= 0
            certainties.index_add_(0, idx[ok], w.detach()[ok])

    s, w, idx, _ = predict(m, mlp, coord, features)
    side_effect(w, idx)
    xd = coord[::decimation]
    n = xd.shape[0]
    e = torch.eye(3) * eps
    stencil = torch.cat([xd + e[0], xd - e[0], xd + e[1], xd - e[1], xd + e[2], xd - e[2]], 0)
    sn, wn, idxn, _ = predict(m, mlp, stencil, features)
    side_effect(wn, idxn)
    sn = sn.reshape(6, n)
    g = torch.stack(((sn[0] - sn[1]), (sn[2] - sn[3]), (sn[4] - sn[5])), 1) / (2 * eps)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(s / sigma, torch.sigmoid(label / sigma))
    loss = loss + weight_e * ((g.norm(dim=-1) - 1.0) ** 2).mean()
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
    return float(loss.detach())


def sdf_grad_std(m: TorchMap, mlp: TorchMLP, q: torch.Tensor):
    """utils/tracker.py:176-275 (query_source_points, one batch): SDF, autograd dsdf/dq, nn_count and,
    with per-neighbour decoding, the IDW standard deviation of the neighbours' SDFs (:245-249)."""
    q = q.detach().to(torch.float32).requires_grad_(True)
    x, w, _, nn = query(m, q)
    s = mlp(x)[..., 0]
    if m.wf:
        mean, std = s, torch.zeros_like(s)
    else:
        mean = (s * w).sum(1)
        std = torch.sqrt((w * (s - mean[:, None]) ** 2).sum(1))
    (g,) = torch.autograd.grad(mean.sum(), q)
    return mean.detach(), g, nn, std.detach()


def registration_step(m: TorchMap, mlp: TorchMLP, points, labels, min_grad_norm, max_grad_norm, gm_dist, gm_grad,
                      lm_lambda, max_sdf_std, min_nn):
    """utils/tracker.py:277-452 + implicit_reg :468-520 without colours / normals: the query, the
    validity mask (nn_count >= min_nn, gradient norm window, sdf std), Geman-McClure weights
    normalised by 2 mean(w), J = [p x g, g], N = J^T W J (+ lm_lambda diag N), g = -(J W)^T r and
    the f64 6x6 solve.  Returns (the 6-vector increment, the valid-point count)."""
    sdf, grad, nn, std = sdf_grad_std(m, mlp, points)
    gn = grad.norm(dim=-1)
    valid = (nn >= min_nn) & (gn < max_grad_norm) & (gn > min_grad_norm) & (std < max_sdf_std)
    p, g, r, gv = points[valid], grad[valid], sdf[valid] - labels[valid], gn[valid]
    w = ((gm_grad / (gm_grad ** 2 + (gv - 1.0) ** 2)) ** 2 * (gm_dist / (gm_dist ** 2 + r ** 2)) ** 2)[:, None]
    w = w / (2.0 * w.mean())
    J = torch.cat((torch.cross(p, g, dim=-1), g), -1)
    N = J.T @ (w * J)
    N = N + lm_lambda * torch.diag(torch.diag(N))
    rhs = -(J * w).T @ r
    t = torch.linalg.inv(N.to(torch.float64)) @ rhs.to(torch.float64)
    return t, int(valid.sum())


def sdf_only(m: TorchMap, mlp: TorchMLP, q: torch.Tensor, min_nn):
    """utils/mesher.py:41-136 (query_points, one batch): SDF of the rows with nn_count >= 1 (0
    elsewhere) and mc_mask = nn_count >= mesh_min_nn, no gradient."""
    with torch.no_grad():
        s, _, _, nn = predict(m, mlp, q.to(torch.float32))
        s = torch.where(nn >= 1, s, torch.zeros_like(s))
    return s, nn >= min_nn
