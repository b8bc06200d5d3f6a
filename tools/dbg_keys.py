"""Repeat-determinism probe of the grid query (WF=1: weighted-first, default per-neighbour): runs the configs[1]
batch twice, reports the queries whose outputs differ and the oracle's values for them."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pin_slam_amd as P  # noqa: E402
from oracle import pin_oracle as O  # noqa: E402
from tests import helpers as H  # noqa: E402

wf = os.environ.get("WF", "0") == "1"
nm, dec, pts = H.surface_map(1000, device="cuda", buffer_size=int(5e7), weighted_first=wf)
q = H.surface_queries(pts, 262144, seed=7, device="cuda")
outs = []
for order in ("input", "input", "input"):
    s, g, nn, _, std = P.query_sdf(nm, dec, q, query_locally=False, want_grad=True, want_certainty=False,
                                   want_std=True, out_order=order)
    outs.append((s.clone(), g.clone(), nn.clone(), std.clone()))
torch.cuda.synchronize()
for k in (1, 2):
    for name, a, b in zip(("sdf", "grad", "nn", "std"), outs[0], outs[k]):
        d = (a != b).reshape(a.shape[0], -1).any(-1)
        print(f"run0 vs run{k} {name}: {int(d.sum())} differ")
bad = torch.nonzero((outs[0][0] != outs[1][0]) | (outs[0][0] != outs[2][0])).flatten()[:16].cpu().numpy()
if bad.size:
    st, mlp = H.oracle_state(nm), H.oracle_mlp(dec)
    qq = q.cpu().numpy()[bad]
    osdf, _, ostd, oq = O.sdf_and_grad(st, mlp, qq, 8, O.neighbor_offsets(2, 0.2), nm.max_valid_dist2, wf, False)
    for t, i in enumerate(bad):
        print(i, "nn", int(outs[0][2][i]), int(oq.nn_counts[t]), "sdf", [float(o[0][i]) for o in outs],
              "oracle", float(osdf[t]), "std", [float(o[3][i]) for o in outs])
