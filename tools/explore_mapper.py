#!/usr/bin/env python3
"""Timing attribution for one mapper iteration as mapping() runs it (GPU only): the forward, the
backward with and without the training side effects (certainty / ts, applied there) and without
the feature scatter, on the rows of a real iteration (tile-sorted, PIN_TRAIN_DX when the decoder
is frozen)."""
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
    for wf in [bool(int(x)) for x in os.environ.get("WFS", "1,0").split(",")]:
        nm, dec, pts = surface_map(side, device="cuda", weighted_first=wf, bs=bs, query_backend="grid")
        for p in dec.parameters():
            p.requires_grad_(False)
        coord, label, ts = surface_pool(pts, 1 << 22, device="cuda")
        mapper = P.Mapper(nm.config, None, nm, dec)
        mapper.set_pool(coord, label, ts)
        mapper.mapping(1)
        b = mapper._buf
        n = bs
        nd = (n + 9) // 10
        rows = n + 6 * nd
        dx = os.environ.get("DX", "1") != "0"   # PIN_TRAIN_DX (frozen decoder), both decoding modes
        cfg = _lib.PinTrainCfg(n_main=n, n_stencil=nd, decimation=10, nn_k=8, weighted_first=int(wf),
                               eps=float(np.float32(0.06)), sigma=float(np.float32(0.055)), weight_e=0.5,
                               grad_scale=1.0, flags=_lib.PIN_TRAIN_ROWS | (_lib.PIN_TRAIN_DX if dx else 0))
        hv, pv = nm._views("local", True)
        gv = nm.grid_view("local", False)
        mv = mlp_view(dec, packed=dx)
        fg = torch.zeros_like(nm.local_geo_features.data)
        res = {}

        def state(side, cert=True, ts=True):
            return _lib.PinTrainState(ids=b.ids.data_ptr(), weights=b.weights.data_ptr(), x=b.x.data_ptr(),
                                      sdf=b.sdf.data_ptr(),
                                      certainties=nm.local_point_certainties.data_ptr() if side and cert else None,
                                      ts_update=nm.local_point_ts_update.data_ptr() if side and ts else None,
                                      order=None, sorted_rows=b.rows4.data_ptr(),
                                      row_ts=b.ts.data_ptr() if side and ts else None)
        st = state(False)

        def fwd():
            _lib.call("pin_train_forward", None, gv.ref(), pv.ref(), mv.ref(), _lib.ptr(b.rows), _lib.ptr(b.ts),
                      ctypes.byref(cfg), ctypes.byref(st), _lib.stream())
        res["fwd"] = timeit(fwd)
        for tag, sb in (("bwd", state(True)), ("bwd_cert_only", state(True, ts=False)),
                        ("bwd_ts_only", state(True, cert=False)), ("bwd_no_side", state(False))):

            def bwd():
                _lib.call("pin_train_backward", pv.ref(), mv.ref(), _lib.ptr(b.label), ctypes.byref(cfg),
                          ctypes.byref(sb), _lib.ptr(fg), None, _lib.ptr(b.workspace), _lib.ptr(b.loss),
                          _lib.stream())
            res[tag] = timeit(bwd)

        def bwd_nofeat():
            _lib.call("pin_train_backward", pv.ref(), mv.ref(), _lib.ptr(b.label), ctypes.byref(cfg),
                      ctypes.byref(st), None, None, _lib.ptr(b.workspace), _lib.ptr(b.loss), _lib.stream())
        res["bwd_no_scatter"] = timeit(bwd_nofeat)
        print(f"wf={int(wf)} rows={rows} " + "  ".join(f"{k} {v:.1f}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
