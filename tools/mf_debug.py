"""Debug: numpy emulation of mlp_sdf_mfma16 from the pin_mlp_pack image vs both GPU decoders."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pin_slam_amd import _lib  # noqa: E402
from pin_slam_amd.query import mlp_view  # noqa: E402
from pin_slam_amd.synthetic import surface_map, surface_queries  # noqa: E402

nm, dec, pts = surface_map(60, buffer_size=1 << 20, weighted_first=True, query_backend="grid")
q = surface_queries(pts, 256)
gv = nm.grid_view("global", True)
_, pv = nm._views("global", False)
n = q.shape[0]
res = []
for packed in (False, True):
    mv = mlp_view(dec, packed=packed)
    sdf = torch.empty(n, device="cuda")
    grad = torch.empty((n, 3), device="cuda")
    nn = torch.empty(n, dtype=torch.int32, device="cuda")
    _lib.call("pin_query_sdf_grid", gv.ref(), pv.ref(), mv.ref(), _lib.ptr(q), n, 8, 1, 0, _lib.ptr(sdf),
              _lib.ptr(grad), _lib.ptr(nn), None, None, None, _lib.stream())
    res.append((sdf.cpu().numpy(), grad.cpu().numpy()))
mv = mlp_view(dec, packed=True)
pk = torch.empty(_lib.MLP_PACK_BYTES, dtype=torch.uint8, device="cuda")
_lib.call("pin_mlp_pack", mv.ref(), _lib.ptr(pk), _lib.stream())
b = pk.cpu().numpy()
feat = nm.query_feature(q, training_mode=False, query_locally=False)[0].detach().cpu().numpy()  # [n,11]
W1 = dec.layers[0].weight.detach().cpu().numpy().astype(np.float64)
b1 = dec.layers[0].bias.detach().cpu().numpy().astype(np.float64)
w2 = dec.lout.weight.detach().cpu().numpy()[0].astype(np.float64)
b2 = float(dec.lout.bias)
s = float(dec.sdf_scale)
pre = feat.astype(np.float64) @ W1.T + b1
ref = s * (np.maximum(pre, 0) @ w2 + b2)
print("f64 ref vs VALU", np.abs(ref - res[0][0]).max(), " vs MF", np.abs(ref - res[1][0]).max())
# emulate from the image
A1 = b[0:4096].view(np.float16).reshape(4, 64, 8).astype(np.float64)
A1L = b[4096:6144].view(np.float16).reshape(4, 64, 4).astype(np.float64)
A2 = b[6144:10240].view(np.float16).reshape(2, 2, 64, 8).astype(np.float64)
us = b[10240:10304].view(np.float32).astype(np.float64)
Afull = np.zeros((64, 32))
AL = np.zeros((64, 16))
for mt in range(4):
    for lane in range(64):
        c = 16 * mt + (lane & 15)
        g = lane >> 4
        Afull[c, 8 * g:8 * g + 8] = A1[mt, lane]
        AL[c, 4 * g:4 * g + 4] = A1L[mt, lane]
A2f = np.zeros((2, 16, 64))
for ch in range(2):
    for t in range(2):
        for lane in range(64):
            i, g = lane & 15, lane >> 4
            for sl in range(8):
                c = 32 * ch + (4 * g + sl if sl < 4 else 16 + 4 * g + sl - 4)
                A2f[t, i, c] += A2[ch, t, lane, sl]
x = feat.astype(np.float32)
out = np.zeros(n)
for qi in range(n):
    xv = x[qi]
    mx = np.abs(xv).max()
    eb = (np.float32(mx).view(np.int32) >> 23) & 0xff
    e = min(max(140 - eb, -14), 15)
    sc = np.float32(2.0 ** e)
    v = xv * sc
    xh = (v.view(np.int32) & np.int32(-8192)).view(np.float32)
    xl = (v - xh).astype(np.float16).astype(np.float64)
    Bh = np.concatenate([xh, xh, [sc, sc], np.zeros(8)]).astype(np.float16).astype(np.float64)
    Bl = np.concatenate([xl, np.zeros(5)])
    D1 = Afull @ Bh + AL @ Bl
    mask = (D1 > 0).astype(np.float64)
    g = (A2f[0] + A2f[1]) @ mask * us
    out[qi] = s * (g[11] + b2 + (xv.astype(np.float64) * g[:11]).sum())
print("emul vs f64", np.abs(out - ref).max(), "emul vs MF kernel", np.abs(out - res[1][0]).max())
print("first", ref[:4], res[0][0][:4], res[1][0][:4], out[:4])
