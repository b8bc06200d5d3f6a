"""Drop-in for utils/mesher.py:Mesher.query_points (utils/mesher.py:41-136).

Each ``bs`` batch is one fused launch (pin_query_sdf / pin_query_sdf_grid with zero_empty):
query_feature in inference mode (no side effects, query_locally as given) + Decoder.sdf on
rows with nn_count >= 1 (0 elsewhere, :100-105) + mc_mask = nn_count >= mask_min_nn_count
(:126-132).  Host-resident coordinates are copied batch by batch through pinned memory on a
side stream so the copy of batch i+1 overlaps the launch of batch i.  Output types follow
the reference: float64 numpy arrays (mask as 0./1.) or, with out_torch, CPU float32 tensors.
"""
import math

import numpy as np
import torch

from .query import query_sdf as fused_query_sdf


class Mesher:
    def __init__(self, config, neural_points, geo_decoder, sem_decoder=None, color_decoder=None):
        self.config = config
        self.silence = config.silence
        self.neural_points = neural_points
        self.geo_decoder = geo_decoder
        self.sem_decoder = sem_decoder
        self.color_decoder = color_decoder
        self.device = config.device
        self.cur_device = self.device
        self.dtype = config.dtype
        self.ts = 0
        self.global_transform = np.eye(4)

    def query_points(self, coord, bs, query_sdf=True, query_sem=False, query_color=False, query_mask=True,
                     query_locally=False, mask_min_nn_count: int = 4, out_torch: bool = False):
        """Returns (sdf_pred, sem_pred, color_pred, mc_mask) like utils/mesher.py:41-136."""
        if query_sem or query_color:
            raise NotImplementedError("semantic / colour heads are outside the fused SDF path")
        n = coord.shape[0]
        iter_n = math.ceil(n / bs)
        sdf_out = (torch.zeros(n) if out_torch else np.zeros(n)) if query_sdf else None
        mask_out = (torch.zeros(n) if out_torch else np.zeros(n)) if query_mask else None
        dev = torch.device(self.device)
        on_host = not coord.is_cuda
        copy_stream = torch.cuda.Stream(device=dev) if on_host else None
        nxt = None

        def stage(i):
            head, tail = i * bs, min((i + 1) * bs, n)
            src = coord[head:tail].to(torch.float32)
            if not on_host:
                return src.contiguous()
            with torch.cuda.stream(copy_stream):
                d = src.pin_memory().to(dev, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            return d, ev

        with torch.no_grad():
            if iter_n > 0:
                nxt = stage(0)
            for i in range(iter_n):
                head, tail = i * bs, min((i + 1) * bs, n)
                cur = nxt
                if on_host:
                    batch, ev = cur
                    torch.cuda.current_stream(dev).wait_event(ev)
                    batch.record_stream(torch.cuda.current_stream(dev))
                else:
                    batch = cur
                if i + 1 < iter_n:
                    nxt = stage(i + 1)
                sdf, _, nn, _, _ = fused_query_sdf(self.neural_points, self.geo_decoder, batch, query_locally=query_locally,
                                             want_grad=False, zero_empty=True, want_std=False, want_certainty=False)
                if query_sdf:
                    if out_torch:
                        sdf_out[head:tail] = sdf.detach().cpu()
                    else:
                        sdf_out[head:tail] = sdf.detach().cpu().numpy()
                if query_mask:
                    m = nn >= mask_min_nn_count
                    if out_torch:
                        mask_out[head:tail] = m.detach().cpu()
                    else:
                        mask_out[head:tail] = m.detach().cpu().numpy()
        return sdf_out, None, None, mask_out


def marching_cubes(values: torch.Tensor, mask: torch.Tensor = None, level: float = 0.0, allow_degenerate=False):
    """Marching cubes on the device (pin_mc_count / pin_mc_emit) over a [nx, ny, nz] grid of
    values (x slowest); ``mask`` [nx, ny, nz] bool selects the processed cubes by their first
    corner.  Returns (verts [V,3] f32 in index space, faces [F,3] int64) device tensors; with
    allow_degenerate False, triangles with two coincident vertices are dropped (the reference
    passes allow_degenerate=False to skimage, utils/mesher.py:327-328)."""
    from . import _lib
    _lib.require_device(values)
    v = values.detach().to(torch.float32).contiguous()
    nx, ny, nz = (int(s) for s in v.shape)
    dev = v.device
    m = None
    if mask is not None:
        m = mask.detach().to(device=dev, dtype=torch.uint8).contiguous()
        if tuple(m.shape) != (nx, ny, nz):
            raise ValueError("mask must have the grid's shape")
    wsb = int(_lib.load().pin_mc_workspace_bytes(nx, ny, nz))
    if wsb < 0:
        raise ValueError(f"marching cubes grid {nx}x{ny}x{nz} outside 2..2^29 points")
    ws = torch.empty((wsb,), dtype=torch.uint8, device=dev)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    _lib.call("pin_mc_count", _lib.ptr(v), _lib.ptr(m), nx, ny, nz, float(level), _lib.ptr(ws), _lib.ptr(counts),
              _lib.stream())
    nv, nf = (int(c) for c in counts.cpu())
    verts = torch.empty((nv, 3), dtype=torch.float32, device=dev)
    faces = torch.empty((nf, 3), dtype=torch.int32, device=dev)
    if nf > 0:
        _lib.call("pin_mc_emit", _lib.ptr(v), nx, ny, nz, float(level), _lib.ptr(ws), _lib.ptr(verts),
                  _lib.ptr(faces), _lib.stream())
    faces = faces.long()
    if not allow_degenerate and nf > 0:
        p = verts[faces]                                       # [F, 3 vertices, 3]
        same = ((p[:, 0] == p[:, 1]).all(-1) | (p[:, 1] == p[:, 2]).all(-1) | (p[:, 0] == p[:, 2]).all(-1))
        faces = faces[~same]
    return verts, faces


def mc_mesh(self, mc_sdf, mc_mask, voxel_size, mc_origin):
    """utils/mesher.py:310-337 with the marching cubes on the device: mc_sdf / mc_mask as the
    reference's assign_to_bbx leaves them (numpy or tensors), returns numpy (verts [V,3] f64 =
    mc_origin + index verts * voxel_size, faces [F,3])."""
    v = torch.as_tensor(mc_sdf, dtype=torch.float32, device=self.device)
    m = None if mc_mask is None else torch.as_tensor(mc_mask, device=self.device).to(torch.bool)
    try:
        verts, faces = marching_cubes(v, m, 0.0, allow_degenerate=False)
    except ValueError:
        # the reference wraps skimage in a bare try/except and returns an empty mesh
        # (utils/mesher.py:324-333); a grid outside 2..2^29 points lands here (the reference's
        # get_query_from_bbx already refuses more than 5e8 voxels, mesher.py:163)
        return np.asarray(mc_origin) + np.zeros((0, 3)) * voxel_size, np.zeros((0, 3))
    verts = np.asarray(mc_origin) + verts.cpu().numpy() * voxel_size
    return verts, faces.cpu().numpy()


Mesher.mc_mesh = mc_mesh
