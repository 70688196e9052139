"""Conv networks on the MI355X vs the reference golden vectors and the CPU oracle.

Tolerances: fp32 compute mode — output within 1e-4 relative (L2), every parameter gradient within
2e-3; bf16 compute mode — 2e-2 / 8e-2 (bf16 operands, fp32 accumulation)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from conftest import load_golden, sub_grads, sub_state  # noqa: E402
from kair_amd.models.network_rrdbnet import RRDBNet  # noqa: E402
from oracle import convnets as ocv  # noqa: E402

dev = torch.device("cuda")
TOL = {"fp32": (1e-4, 2e-3), "bf16": (2e-2, 8e-2)}


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def check_fwd_bwd(net, x, out_ref, gout, grads_ref, dt):
    out = net(x.to(dev))
    assert rel(out, out_ref) < TOL[dt][0]
    out.backward(gout.to(dev))
    worst = {k: rel(p.grad, grads_ref[k]) for k, p in net.named_parameters()}
    k = max(worst, key=worst.get)
    assert worst[k] < TOL[dt][1], (k, worst[k])


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_rrdbnet_vs_golden(dt):
    z = load_golden("conv_nets")
    net = RRDBNet(3, 3, 32, 1, 16, 4, compute_dtype=dt)
    net.load_state_dict(sub_state(z, "rrdbnet."), strict=True)
    net = net.to(dev).train()
    check_fwd_bwd(net, torch.from_numpy(z["rrdbnet.x"]), torch.from_numpy(z["rrdbnet.out"]),
                  torch.from_numpy(z["rrdbnet.gout"]), sub_grads(z, "rrdbnet."), dt)


@pytest.mark.parametrize("sf", [2, 4])
def test_rrdbnet_full_width_vs_oracle(sf):
    """nf 64 / gc 32 (the C5 widths), 3 RRDBs, 32-px LQ, fp32 parity mode vs the CPU oracle."""
    torch.manual_seed(3)
    net = RRDBNet(3, 3, 64, 3, 32, sf, compute_dtype="fp32")
    ref = ocv.RRDBNet(3, 3, 64, 3, 32, sf)
    ref.load_state_dict(net.state_dict(), strict=True)
    g = torch.Generator().manual_seed(4)
    x = torch.rand(2, 3, 32, 32, generator=g)
    out_ref = ref(x)
    gout = torch.randn(out_ref.shape, generator=g)
    out_ref.backward(gout)
    grads = {k: p.grad for k, p in ref.named_parameters()}
    check_fwd_bwd(net.to(dev).train(), x, out_ref, gout, grads, "fp32")


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_dncnn_bn_train_vs_golden(dt):
    """DnCNN with BatchNorm in train mode: output, gradients and the running-stat update."""
    from kair_amd.models.network_dncnn import DnCNN
    z = load_golden("conv_nets")
    net = DnCNN(1, 1, 64, 5, "BR", compute_dtype=dt)
    net.load_state_dict(sub_state(z, "dncnn."), strict=True)
    net = net.to(dev).train()
    check_fwd_bwd(net, torch.from_numpy(z["dncnn.x"]), torch.from_numpy(z["dncnn.out"]),
                  torch.from_numpy(z["dncnn.gout"]), sub_grads(z, "dncnn."), dt)
    sd = net.state_dict()
    for k in z.files:
        if k.startswith("dncnn.after."):
            name = k[len("dncnn.after."):]
            assert rel(sd[name], torch.from_numpy(z[k])) < 1e-5, name
    for k, v in sd.items():
        if k.endswith("num_batches_tracked"):
            assert int(v) == int(z["dncnn.param." + k]) + 1


def test_dncnn_eval_and_fdncnn_vs_reference():
    """eval-mode BN (running statistics; oracle DnCNN) and FDnCNN (no residual, noise-map channel;
    the same layer stack evaluated with torch fp32 ops on the CPU), fp32 parity mode."""
    from kair_amd.models.network_dncnn import DnCNN, FDnCNN
    torch.manual_seed(5)
    net = DnCNN(1, 1, 64, 6, "BR", compute_dtype="fp32")
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
    ref = ocv.DnCNN(1, 1, 64, 6, "BR")
    ref.load_state_dict(net.state_dict(), strict=True)
    x = torch.rand(3, 1, 24, 20)
    assert rel(net.to(dev).eval()(x.to(dev)), ref.eval()(x)) < 1e-4
    f = FDnCNN(2, 1, 32, 5, "R", compute_dtype="fp32")
    cpu = FDnCNN(2, 1, 32, 5, "R")
    cpu.load_state_dict(f.state_dict())
    x2 = torch.rand(2, 2, 16, 24)
    assert rel(f.to(dev).eval()(x2.to(dev)), cpu.model(x2)) < 1e-4
