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
