"""The drop-in Decoder.sdf on the HIP row kernels (pin_mlp_forward / pin_mlp_backward) against
the reference's own formulation: model/decoder.py:66-88 as nn.Linear layers under torch autograd
(PIN_DECODER_ATEN path of the same module, float32), for the value, the first-order gradients
(input and parameters) and the double backward of get_gradient (utils/tools.py:174-184 with
create_graph=True, the analytic-eikonal training loss of utils/mapper.py:482-547).

Tolerances (float32 sums in another order): values 1e-5 abs (the north_star SDF bar), gradients
1e-4 of each tensor's largest element + 1e-7."""
import pytest
import torch

import pin_slam_amd.decoder as D


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return "cuda"


def _decoder(dev, seed=3):
    import pin_slam_amd as P
    cfg = P.Config(device=dev)
    torch.manual_seed(seed)
    dec = P.Decoder(cfg, cfg.geo_mlp_hidden_dim, cfg.geo_mlp_level, 1).to(dev)
    with torch.no_grad():   # spread the pre-activations so both ReLU branches are common
        dec.layers[0].weight.mul_(3.0)
        dec.lout.weight.mul_(2.0)
    return dec


def _close(a, b, name):
    tol = 1e-4 * float(b.abs().max()) + 1e-7
    err = float((a - b).abs().max())
    assert err <= tol, (name, err, tol)


def _run(dec, x, monkeypatch, aten, second):
    monkeypatch.setattr(D, "_ATEN_SDF", aten)
    x = x.clone().requires_grad_(True)
    ps = list(dec.parameters())
    sdf = dec.sdf(x)
    if not second:
        c = torch.linspace(0.2, 1.0, sdf.numel(), device=x.device).view_as(sdf)   # no cancelling sum
        grads = torch.autograd.grad((sdf * c).sum(), [x] + ps)
        return sdf.detach(), grads
    g, = torch.autograd.grad(sdf, x, torch.ones_like(sdf), create_graph=True)
    label = torch.sin(torch.arange(sdf.numel(), device=x.device, dtype=torch.float32)).view_as(sdf) * 0.05
    loss = torch.nn.functional.binary_cross_entropy_with_logits(sdf / 0.1, torch.sigmoid(label / 0.1)) + \
        0.5 * ((g.norm(2, dim=-1) - 1.0) ** 2).mean() + (g[..., 8:] * 0.3).sum() * 1e-3
    grads = torch.autograd.grad(loss, [x] + ps, allow_unused=True)
    return sdf.detach(), [torch.zeros_like(t) if gr is None else gr for gr, t in zip(grads, [x] + ps)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(50_003, 11), (6_001, 8, 11), (1, 11), (7, 1, 11)])
@pytest.mark.parametrize("second", [False, True])
def test_decoder_rows_match_module(dev, monkeypatch, shape, second):
    dec = _decoder(dev)
    g = torch.Generator(device="cpu").manual_seed(5)
    x = (torch.randn(shape, generator=g) * 0.7).to(dev)
    ref_sdf, ref = _run(dec, x, monkeypatch, True, second)
    got_sdf, got = _run(dec, x, monkeypatch, False, second)
    assert got_sdf.shape == ref_sdf.shape
    assert float((got_sdf - ref_sdf).abs().max()) <= 1e-5
    for name, a, b in zip(["x", "W1", "b1", "W2", "b2"], got, ref):
        _close(a, b, name)


@pytest.mark.gpu
def test_decoder_rows_run_native(dev, monkeypatch):
    """The geo decoder's sdf goes through the row kernels (no nn.Linear GEMM on the way), and a
    decoder shape the kernels do not cover (two outputs) stays on the module's layers."""
    import pin_slam_amd as P
    monkeypatch.setattr(D, "_ATEN_SDF", False)
    dec = _decoder(dev)
    calls = []
    real = D._lib.call
    monkeypatch.setattr(D._lib, "call", lambda name, *a: (calls.append(name), real(name, *a))[1])
    x = torch.randn(100, 11, device=dev, requires_grad=True)
    dec.sdf(x).sum().backward()
    assert calls[:2] == ["pin_mlp_forward", "pin_mlp_backward"], calls
    cfg = P.Config(device=dev)
    sem = P.Decoder(cfg, cfg.geo_mlp_hidden_dim, 1, 2).to(dev)
    assert not sem._rows_ok(x)
