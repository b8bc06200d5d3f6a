"""Drop-in ``DataSampler`` (utils/data_sampler.py:11-192): training samples along the scan rays.

``sample`` draws the reference's random numbers with the reference's calls, in the reference's
order (``torch.randn`` [N*surface_n,1], then ``torch.rand`` [N*free_front_n,1] and
[N*free_behind_n,1], on ``config.device``) and hands them to one fused HIP launch
(``pin_sample_rays``) that writes the samples, their projective SDF labels and weights directly
in the reference's final ray-wise order -- and, when a pose is given, the same samples in the
world frame (``transform_torch``), which ``Mapper.process_frame`` needs twice.
"""
import ctypes

import numpy as np
import torch

from . import _lib


def sample_cfg(config, pose_f32=None) -> "_lib.PinSampleCfg":
    c = config
    rng = float(c.surface_sample_range_m)
    end = float(c.free_sample_end_dist_m)
    scale = float(c.dist_weight_scale)
    return _lib.PinSampleCfg(
        surface_n=int(c.surface_sample_n), front_n=int(c.free_front_n), behind_n=int(c.free_behind_n),
        surface_range=rng, two_range=float(np.float32(2.0 * rng)), front_min_ratio=float(c.free_sample_begin_ratio),
        end_dist=end, dist_weight_on=int(bool(c.dist_weight_on)), dist_weight_base=float(np.float32(1 + scale * 0.5)),
        dist_weight_scale=scale, max_range=float(c.max_range), behind_dropoff_on=int(bool(c.behind_dropoff_on)),
        dropoff_max=end, dropoff_diff=float(np.float32(end - 0.2 * end)),
        pose=None if pose_f32 is None else pose_f32.data_ptr())


class DataSampler:
    """utils/data_sampler.py:DataSampler."""

    def __init__(self, config):
        self.config = config
        self.dev = config.device

    def draws(self, n):
        """The reference's random draws for n rays (data_sampler.py:50, :76, :89), in its call order."""
        c, dev = self.config, self.dev
        rs = torch.randn(n * int(c.surface_sample_n), 1, device=dev)
        rf = torch.rand(n * int(c.free_front_n), 1, device=dev)
        rb = torch.rand(n * int(c.free_behind_n), 1, device=dev)
        return rs, rf, rb

    def sample(self, points_torch, normal_torch, sem_label_torch, color_torch, pose=None, draws=None):
        """Returns (coord, sdf_label, normal_label, sem_label, color, weight) like the reference
        (utils/data_sampler.py:20-192); with ``pose`` ([4,4], any float dtype) a 7th element, the
        samples transformed to the world frame (utils/tools.py:386-399 on the f32-cast pose).
        ``draws``: optional (randn_surface, rand_front, rand_behind) to replay given draws."""
        c = self.config
        _lib.require_device(points_torch)
        pts = points_torch[:, :3].detach().to(torch.float32).contiguous()
        n = pts.shape[0]
        dev = pts.device
        A = 1 + int(c.surface_sample_n) + int(c.free_front_n) + int(c.free_behind_n)
        rs, rf, rb = self.draws(n) if draws is None else draws
        rs, rf, rb = (t.to(device=dev, dtype=torch.float32).contiguous() for t in (rs, rf, rb))
        coord = torch.empty((n * A, 3), dtype=torch.float32, device=dev)
        sdf_label = torch.empty((n * A,), dtype=torch.float32, device=dev)
        weight = torch.empty((n * A,), dtype=torch.float32, device=dev)
        glob = None
        pose_f32 = None
        if pose is not None:
            pose_f32 = pose.detach().to(device=dev, dtype=torch.float32).contiguous()
            glob = torch.empty((n * A, 3), dtype=torch.float32, device=dev)
        cfg = sample_cfg(c, pose_f32)
        _lib.call("pin_sample_rays", _lib.ptr(pts), n, _lib.ptr(rs), _lib.ptr(rf), _lib.ptr(rb), ctypes.byref(cfg),
                  _lib.ptr(coord), _lib.ptr(sdf_label), _lib.ptr(weight), _lib.ptr(glob), _lib.stream())
        S = int(c.surface_sample_n)
        normal_label = None
        if normal_torch is not None:                                   # :148-150, :173-174
            normal_label = normal_torch.repeat_interleave(A, dim=0)
        sem_label = None
        if sem_label_torch is not None:                                # :153-155, :175-176
            s = sem_label_torch.reshape(-1, 1).int()
            sem_label = torch.cat((s.repeat(1, 1 + S), torch.zeros((n, A - 1 - S), dtype=torch.int32, device=dev)),
                                  1).reshape(-1)
        color = None
        if color_torch is not None:                                    # :157-159, :177-178
            ch = color_torch.shape[1]
            color = torch.cat((color_torch.unsqueeze(1).repeat(1, 1 + S, 1),
                               torch.zeros((n, A - 1 - S, ch), dtype=color_torch.dtype, device=dev)), 1).reshape(-1, ch)
        out = (coord, sdf_label, normal_label, sem_label, color, weight)
        return out + (glob,) if pose is not None else out
