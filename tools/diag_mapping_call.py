"""Diagnose a whole-mapping() fixture on the GPU: first-step gradients against the reference's
(it0_*), then the features after the call (distribution of the differences)."""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from tests.conftest import GOLDEN  # noqa: E402
from tests.test_gpu_mapper import _mapping_call_setup  # noqa: E402
import pin_slam_amd as P  # noqa: E402
from pin_slam_amd import _lib  # noqa: E402


def main(case, backend="grid"):
    z = dict(np.load(f"{GOLDEN}/{case}.npz"))
    dev = "cuda"
    nm, dec, mapper, replay = _mapping_call_setup(z, dev, backend)
    # first step: the same draws, the gradients before Adam
    fdata = nm.local_geo_features.data
    fg = torch.zeros_like(fdata)
    mg = None if bool(z["frozen"]) else torch.zeros((_lib.MLP_GRAD_SIZE,), device=dev)
    index = mapper._batch_index()
    mapper.train_step(mapper.global_coord_pool, mapper.sdf_label_pool, mapper.time_pool, fg, mg, 1, index=index,
                      weight=mapper.weight_pool)
    g = fg.cpu().numpy()
    w = z["it0_feat_grad"]
    d = np.abs(g - w)
    scale = np.abs(w).max()
    print(f"{case}: first-step feature gradient |diff| max {d.max():.3e} (scale {scale:.3e}), "
          f"rel norm {np.linalg.norm(g - w) / np.linalg.norm(w):.3e}, spread norm {float(z['spread_norm_it0_feat_grad']):.3e}"
          f" vs ||diff|| {np.linalg.norm(g - w):.3e}")
    small = np.abs(w) < 1e-6 * scale
    print("  elements with |g_ref| < 1e-6 max:", int(small.sum()), "sign differs:", int((np.sign(g) != np.sign(w)).sum()),
          "of which tiny:", int(((np.sign(g) != np.sign(w)) & small).sum()))
    if mg is not None:
        off = 0
        for k, n in zip(["W1", "b1", "W2", "b2"], (704, 64, 64, 1)):
            a = mg[off:off + n].cpu().numpy()
            r = z[f"it0_grad_{k}"].ravel()
            print(f"  {k}: rel norm {np.linalg.norm(a - r) / np.linalg.norm(r):.3e}, spread {float(z['spread_norm_it0_grad_' + k]) / np.linalg.norm(r):.3e}")
            off += n


if __name__ == "__main__":
    main(*sys.argv[1:])
