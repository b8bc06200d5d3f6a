"""Synthetic workloads of SURVEY.md 8(d) (the KITTI example data is not available offline).

Map: one neural point per ``res`` voxel column on z = 0.5 sin(x/7) cos(y/5) + 0.15 over
an n x n grid, xy = (i + 0.5) * res; features ~ N(0, 0.05^2) (the reference default
feature_std = 0 would make the benchmark degenerate); decoder = nn.Linear default init
under torch.manual_seed(seed).  Queries: random map points + N(0, sigma^2) per axis.
"""
import torch

from .config import Config
from .decoder import Decoder
from .neural_points import NeuralPoints


def surface_points(n_side, res=0.3):
    i = torch.arange(n_side, dtype=torch.float64)
    x, y = torch.meshgrid((i + 0.5) * res, (i + 0.5) * res, indexing="ij")
    x, y = x.reshape(-1), y.reshape(-1)
    z = 0.5 * torch.sin(x / 7.0) * torch.cos(y / 5.0) + 0.15
    return torch.stack([x, y, z], 1).to(torch.float32)


def surface_map(n_side, res=0.3, seed=42, device="cuda", buffer_size=int(5e7), nn_k=8, weighted_first=True,
                feature_std=0.05, num_nei_cells=2, search_alpha=0.2, **cfg_kw):
    """Returns (NeuralPoints with the whole map local, Decoder, host points [M,3])."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    pts = surface_points(n_side, res)
    cfg = Config(device=device, voxel_size_m=res, buffer_size=buffer_size, query_nn_k=nn_k,
                 weighted_first=weighted_first, local_map_radius=1e9, num_nei_cells=num_nei_cells,
                 search_alpha=search_alpha, **cfg_kw)
    nm = NeuralPoints(cfg)
    M = pts.shape[0]
    nm.neural_points = pts.to(device)
    quat = torch.zeros(M, 4, device=device)
    quat[:, 0] = 1.0
    nm.point_orientations = quat
    nm.point_ts_create = torch.zeros(M, dtype=torch.int64, device=device)
    nm.point_ts_update = torch.zeros(M, dtype=torch.int64, device=device)
    feats = torch.randn(M + 1, 8, generator=g) * feature_std
    feats[-1] = 0
    nm.geo_features = feats.to(device)
    nm.point_certainties = (torch.rand(M, generator=g) * 10).to(device)
    nm.travel_dist = torch.zeros(1, device=device)
    nm.rebuild_hash()
    nm.reset_local_map(torch.zeros(3, device=device), torch.eye(3, device=device), 0)
    torch.manual_seed(seed)
    dec = Decoder(cfg, 64, 1, 1)
    return nm, dec, pts


def surface_scan(cx, cy, radius, n, seed=0, sigma=0.02, device="cuda"):
    """A lidar-like frame: n points area-uniform in a disk of ``radius`` around (cx, cy) on the
    surface, z noise N(0, sigma^2).  Returns [n,3] f32 on ``device``."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    r = radius * torch.sqrt(torch.rand(n, generator=g, dtype=torch.float64))
    a = 2 * torch.pi * torch.rand(n, generator=g, dtype=torch.float64)
    x, y = cx + r * torch.cos(a), cy + r * torch.sin(a)
    z = 0.5 * torch.sin(x / 7.0) * torch.cos(y / 5.0) + 0.15 + sigma * torch.randn(n, generator=g, dtype=torch.float64)
    return torch.stack([x, y, z], 1).to(torch.float32).to(device)


def surface_queries(pts, n, seed=7, sigma=0.25, device="cuda"):
    g = torch.Generator(device="cpu").manual_seed(seed)
    idx = torch.randint(0, pts.shape[0], (n,), generator=g)
    q = pts[idx] + torch.randn(n, 3, generator=g) * sigma
    return q.to(device)


def surface_pool(pts, n, seed=11, sigma=0.25, device="cuda"):
    """Mapper training pool: map points offset along z by
    N(0, sigma^2), label = -offset, frame ts 0.  Returns (coord [n,3], label [n], ts [n])."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    idx = torch.randint(0, pts.shape[0], (n,), generator=g)
    off = torch.randn(n, generator=g) * sigma
    coord = pts[idx].clone()
    coord[:, 2] += off
    return coord.to(device), (-off).to(device), torch.zeros(n, dtype=torch.int64, device=device)


def train_surface(nm, dec, pts, iters=300, bs=16384, seed=3, pool=1 << 20):
    """Fit the map + decoder to the synthetic surface with the fused Mapper (sdf label = -z offset),
    so that SDF gradients are meaningful (tracker workloads).  Returns the last loss."""
    from .mapper import Mapper
    cfg = nm.config
    old_bs = cfg.bs
    cfg.bs = bs
    for p in dec.parameters():
        p.requires_grad_(True)
    coord, label, ts = surface_pool(pts, pool, seed=seed, device=nm.neural_points.device)
    mapper = Mapper(cfg, None, nm, dec)
    mapper.set_pool(coord, label, ts)
    torch.manual_seed(seed)
    mapper.mapping(iters)
    cfg.bs = old_bs
    nm.reset_local_map(torch.zeros(3, device=nm.neural_points.device),
                       torch.eye(3, device=nm.neural_points.device), 0)
    return float(mapper.last_loss)
