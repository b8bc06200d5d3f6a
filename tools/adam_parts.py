#!/usr/bin/env python3
"""Attribution of the SLAM mapping iteration's optimiser launch (pin_adam_step_train): the full
launch (feature step + 8 gradient replicas summed and re-zeroed + the decoder's step and re-pack)
against the same launch without the decoder segments, without the replicas, and the decoder block
alone, at a SLAM frame's sizes (52,288-point local map, 11-64-1 decoder).  GPU only."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pin_slam_amd import _lib  # noqa: E402


def main():
    dev = "cuda"
    L = int(os.environ.get("ADAM_ROWS", "52288"))
    n = L * 8
    f = lambda k: torch.zeros(k, device=dev)
    prm, grad, m, v = torch.randn(n, device=dev), f(n), f(n), f(n)
    rep = f(8 * n)
    dec = torch.randn(64 * 11 + 64 + 64 + 1, device=dev) * 0.1
    dg, dm, dv = f(dec.numel()), f(dec.numel()), f(dec.numel())
    sizes = [64 * 11, 64, 64, 1]
    offs = [0, 704, 768, 832]
    ptrs = (ctypes.c_void_p * 4)(*[dec.data_ptr() + 4 * o for o in offs])
    szs = (ctypes.c_int64 * 4)(*sizes)
    mlp = _lib.PinMlp(W1=ptrs[0], b1=ptrs[1], W2=ptrs[2], b2=ptrs[3], sdf_scale=1.0)
    packed = torch.empty(_lib.MLP_PACK_BYTES, dtype=torch.uint8, device=dev)
    a = _lib.PinAdamStep(neg_step_size=-1e-3, one_minus_beta1=0.1, beta2=0.99, one_minus_beta2=0.01,
                         bias_correction2_sqrt=1.0, eps=1e-15, zero_grad=1, grad_stride=8)
    fn = _lib.fn("pin_adam_step_train")
    s = torch.cuda.current_stream().cuda_stream

    def launch(nf, use_rep, nseg):
        rc = fn(prm.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(), nf,
                rep.data_ptr() if use_rep else None, 8 if use_rep else 1, None, 0,
                ptrs if nseg else None, szs if nseg else None, nseg, dg.data_ptr(), dm.data_ptr(), dv.data_ptr(),
                ctypes.byref(mlp) if nseg else None, packed.data_ptr() if nseg else None, ctypes.byref(a), s)
        assert rc == 0, rc

    cases = [("full (features + 8 replicas + decoder step + pack)", n, True, 4),
             ("features + 8 replicas", n, True, 0),
             ("features + decoder step + pack", n, False, 4),
             ("features only", n, False, 0),
             ("decoder step + pack (8 feature floats)", 8, False, 4)]
    for rnd in range(2):
        for name, nf, use_rep, nseg in cases:
            for _ in range(20):
                launch(nf, use_rep, nseg)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(200):
                launch(nf, use_rep, nseg)
            e1.record()
            torch.cuda.synchronize()
            print(f"round {rnd} {name:52s} {e0.elapsed_time(e1) / 200 * 1e3:7.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()
