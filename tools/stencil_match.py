"""Share of the stencil rows' top-k entries that also appear in their group's first row (x + eps):
the merge potential of a per-group pre-sum of the stencil scatter (configs[3] batch)."""
import sys, torch, numpy as np
sys.path.insert(0, "/root/repo")
import pin_slam_amd as P
from pin_slam_amd.synthetic import surface_map, surface_pool
nm, dec, pts = surface_map(2000, device="cuda", buffer_size=int(5e7))
cfg = nm.config; cfg.bs = 1 << 20
coord, label, ts = surface_pool(pts, 1 << 20, seed=11, device="cuda")
m = P.Mapper(cfg, None, nm, dec)
fg = torch.zeros_like(nm.local_geo_features.data)
m.train_step(coord, label, ts, fg)
b = m._buf; n = 1 << 20; nd = (n + 9) // 10; rows = n + 6 * nd
order = b.rows4[:rows, 3].contiguous().view(torch.int32).long()
inv = torch.empty_like(order); inv[order] = torch.arange(rows, device="cuda")
ids = b.ids[:rows].long()[inv]          # per original row
st = ids[n:].view(6, nd, 8)
base = st[0]
tot = match = 0
for r in range(1, 6):
    eq = (st[r][:, :, None] == base[:, None, :]).any(-1) & (st[r] >= 0)
    match += int(eq.sum()); tot += int((st[r] >= 0).sum())
print("stencil entries matched to row 0:", match / tot, "of", tot)
same = (torch.sort(st, dim=-1)[0] == torch.sort(base, dim=-1)[0][None]).all(-1).float().mean(1)
print("rows with identical sets:", same.tolist())
