#!/usr/bin/env python3
"""Timing attribution for the fused mapper iteration (GPU only): forward with / without the
training side effects, backward, Adam, and the inference kernel on the same rows."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd import _lib  # noqa: E402
from pin_slam_amd.query import mlp_view  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_pool  # noqa: E402


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    side = int(os.environ.get("SIDE", "2000"))
    bs = int(os.environ.get("BS", str(1 << 20)))
    for wf in (True, False):
        nm, dec, pts = surface_map(side, device="cuda", weighted_first=wf, bs=bs)
        for p in dec.parameters():
            p.requires_grad_(False)
        coord, label, ts = surface_pool(pts, bs, device="cuda")
        mapper = P.Mapper(nm.config, None, nm, dec)
        mapper.set_pool(coord, label, ts)
        fg = torch.zeros_like(nm.local_geo_features.data)
        c = nm.config
        n = bs
        nd = (n + 9) // 10
        rows = n + 6 * nd
        b = mapper._buf.get(rows, 8, wf, coord.device)
        cfg = _lib.PinTrainCfg(n_main=n, n_stencil=nd, decimation=10, nn_k=8, weighted_first=int(wf),
                               eps=float(np.float32(0.06)), sigma=float(np.float32(0.055)), weight_e=0.5,
                               grad_scale=1.0, flags=0)
        hv, pv = nm._views("local", True)
        mv = mlp_view(dec)
        res = {}
        for backend in ("grid", "hash"):
            gv = nm.grid_view("local", False) if backend == "grid" else None
            for tag, cert, tsp in (("full", nm.local_point_certainties, ts), ("no_ts", nm.local_point_certainties, None),
                                   ("no_side", None, None)):
                st = _lib.PinTrainState(ids=b.ids.data_ptr(), weights=b.weights.data_ptr(), x=b.x.data_ptr(),
                                        sdf=b.sdf.data_ptr(), certainties=cert.data_ptr() if cert is not None else None,
                                        ts_update=nm.local_point_ts_update.data_ptr() if tsp is not None else None)

                def fwd():
                    _lib.call("pin_train_forward", hv.ref() if gv is None else None, gv.ref() if gv else None,
                              pv.ref(), mv.ref(), _lib.ptr(coord), _lib.ptr(tsp), ctypes.byref(cfg), ctypes.byref(st),
                              _lib.stream())
                res[f"fwd_{backend}_{tag}"] = timeit(fwd)
            st = _lib.PinTrainState(ids=b.ids.data_ptr(), weights=b.weights.data_ptr(), x=b.x.data_ptr(),
                                    sdf=b.sdf.data_ptr(), certainties=None, ts_update=None)

        def bwd():
            _lib.call("pin_train_backward", pv.ref(), mv.ref(), _lib.ptr(label), ctypes.byref(cfg), ctypes.byref(st),
                      _lib.ptr(fg), None, _lib.ptr(b.workspace), _lib.ptr(b.loss), _lib.stream())
        res["bwd"] = timeit(bwd)

        def bwd_nofeat():
            _lib.call("pin_train_backward", pv.ref(), mv.ref(), _lib.ptr(label), ctypes.byref(cfg), ctypes.byref(st),
                      None, None, _lib.ptr(b.workspace), _lib.ptr(b.loss), _lib.stream())
        res["bwd_no_scatter"] = timeit(bwd_nofeat)
        m, v = torch.zeros_like(fg), torch.zeros_like(fg)
        from pin_slam_amd.mapper import adam_scalars
        a = adam_scalars(0.01, 1, 1e-15)
        res["adam"] = timeit(lambda: _lib.call("pin_adam_step", _lib.ptr(nm.local_geo_features.data), _lib.ptr(fg),
                                               _lib.ptr(m), _lib.ptr(v), fg.numel(), ctypes.byref(a), _lib.stream()))
        allrows = torch.cat([coord] + [coord[::10] + 0.06 * torch.tensor(e, device="cuda") for e in
                                       ([1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1])])
        res["infer_grid_fat_nograd"] = timeit(lambda: P.query_sdf(nm, dec, allrows, want_grad=False,
                                                                  want_certainty=False))
        res["mapping_iter"] = timeit(lambda: mapper.mapping(1), reps=5)
        print(f"wf={wf} rows={rows} map={pts.shape[0]}:", {k: round(v_, 1) for k, v_ in res.items()}, flush=True)
        del nm, dec, pts, mapper


if __name__ == "__main__":
    main()
