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


def grad_errors(named_grads, grads_ref):
    """Error of each gradient relative to max(its own norm, 1e-4 x the largest gradient norm): a conv
    bias feeding a train-mode BatchNorm has an analytically zero gradient."""
    scale = max(v.double().norm().item() for v in grads_ref.values())
    out = {}
    for k, a in named_grads:
        a, b = a.detach().double().cpu(), grads_ref[k].detach().double().cpu()
        if b.norm().item() < 1e-4 * scale:     # analytically zero: both must be rounding noise
            out[k] = a.norm().item() / (1e-4 * scale) * 1e-3
        else:
            out[k] = ((a - b).norm() / b.norm()).item()
    return out


def check_fwd_bwd(net, x, out_ref, gout, grads_ref, dt, bf16_yardstick=None):
    """bf16_yardstick: the same network run in torch bf16 on the CPU; when given, each bf16 gradient
    may be off by up to 1.5x torch's own bf16 error on it (+ the base tolerance)."""
    out = net(x.to(dev))
    assert rel(out, out_ref) < TOL[dt][0]
    out.backward(gout.to(dev))
    worst = grad_errors([(k, p.grad) for k, p in net.named_parameters()], grads_ref)
    allow = {k: TOL[dt][1] for k in worst}
    if bf16_yardstick is not None and dt == "bf16":
        ref_net = bf16_yardstick.to(torch.bfloat16)
        ref_net(x.bfloat16()).backward(gout.bfloat16())
        yard = grad_errors([(k, p.grad) for k, p in ref_net.named_parameters()], grads_ref)
        allow = {k: TOL[dt][1] + 1.5 * yard[k] for k in worst}
    bad = {k: (worst[k], allow[k]) for k in worst if worst[k] > allow[k]}
    assert not bad, bad


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_rrdbnet_vs_golden(dt):
    z = load_golden("conv_nets")
    net = RRDBNet(3, 3, 32, 1, 16, 4, compute_dtype=dt)
    net.load_state_dict(sub_state(z, "rrdbnet."), strict=True)
    yard = ocv.RRDBNet(3, 3, 32, 1, 16, 4)
    yard.load_state_dict(sub_state(z, "rrdbnet."), strict=True)
    net = net.to(dev).train()
    check_fwd_bwd(net, torch.from_numpy(z["rrdbnet.x"]), torch.from_numpy(z["rrdbnet.out"]),
                  torch.from_numpy(z["rrdbnet.gout"]), sub_grads(z, "rrdbnet."), dt, bf16_yardstick=yard)


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_rrdb_basicblock_vs_golden(dt):
    """option net_type 'rrdb' (network_rrdb.RRDB: ReLU, upconv), reduced depth."""
    from kair_amd.models.network_rrdb import RRDB
    z = load_golden("conv_nets")
    net = RRDB(3, 3, 32, 1, 16, 4, "R", "upconv", compute_dtype=dt)
    net.load_state_dict(sub_state(z, "rrdb."), strict=True)
    yard = ocv.RRDB(3, 3, 32, 1, 16, 4, "R", "upconv")
    yard.load_state_dict(sub_state(z, "rrdb."), strict=True)
    net = net.to(dev).train()
    check_fwd_bwd(net, torch.from_numpy(z["rrdb.x"]), torch.from_numpy(z["rrdb.out"]),
                  torch.from_numpy(z["rrdb.gout"]), sub_grads(z, "rrdb."), dt, bf16_yardstick=yard)


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
    yard = ocv.DnCNN(1, 1, 64, 5, "BR").train()
    yard.load_state_dict(sub_state(z, "dncnn."), strict=True)
    net = net.to(dev).train()
    check_fwd_bwd(net, torch.from_numpy(z["dncnn.x"]), torch.from_numpy(z["dncnn.out"]),
                  torch.from_numpy(z["dncnn.gout"]), sub_grads(z, "dncnn."), dt, bf16_yardstick=yard)
    sd = net.state_dict()
    for k in z.files:
        if k.startswith("dncnn.after."):
            name = k[len("dncnn.after."):]
            assert rel(sd[name], torch.from_numpy(z[k])) < (1e-5 if dt == "fp32" else 2e-2), name
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


@pytest.mark.parametrize("kind", ["rrdbnet", "dncnn"])
def test_fused_trainer_conv_nets_vs_oracle_trainer(kind):
    """4 fused training steps (HIP graph after 2 warm steps; fp32 parity mode) vs the CPU oracle
    trainer (ModelPlain.optimize_parameters semantics: L1, Adam, EMA 0.999): parameters, EMA and
    (DnCNN) BatchNorm running statistics."""
    from kair_amd.engine.trainer import FusedTrainer
    from kair_amd.models.network_dncnn import DnCNN
    from oracle.train import OracleTrainer
    torch.manual_seed(11)
    if kind == "rrdbnet":
        mk, mko, shp, sc = (lambda: RRDBNet(3, 3, 32, 1, 16, 4, compute_dtype="fp32")), \
            (lambda: ocv.RRDBNet(3, 3, 32, 1, 16, 4)), (2, 3, 12, 12), 4
    else:
        mk, mko, shp, sc = (lambda: DnCNN(1, 1, 32, 5, "BR", compute_dtype="fp32")), \
            (lambda: ocv.DnCNN(1, 1, 32, 5, "BR")), (4, 1, 16, 16), 1
    net, ema = mk(), mk()
    ema.load_state_dict(net.state_dict())
    ref, ref_e = mko(), mko()
    ref.load_state_dict(net.state_dict())
    ref_e.load_state_dict(net.state_dict())
    ref.train()
    otr = OracleTrainer(ref, ref_e, lr=1e-3, E_decay=0.999)
    net, ema = net.to(dev).train(), ema.to(dev).eval()
    tr = FusedTrainer(net, ema, lr=1e-3, E_decay=0.999, use_graph=True)
    g = torch.Generator().manual_seed(12)
    for s in range(4):
        L = torch.rand(*shp, generator=g)
        Hh = torch.rand(shp[0], shp[1], shp[2] * sc, shp[3] * sc, generator=g)
        _, lo = otr.optimize_parameters(L, Hh)
        lg = tr.step(L.to(dev), Hh.to(dev)).item()
        assert abs(lg - lo) < 1e-4 * abs(lo), (s, lg, lo)
    # a conv bias feeding a train-mode BatchNorm has an analytically zero gradient; Adam turns its
    # rounding noise into +-lr steps in any implementation (the reference's included), so skip those
    pre_bn = set()
    if kind == "dncnn":
        seq = list(net.model)
        for i in range(len(seq) - 1):
            if isinstance(seq[i + 1], torch.nn.BatchNorm2d):   # (its running_mean carries that bias too)
                pre_bn |= {f"model.{i}.bias", f"model.{i + 1}.running_mean"}
    for k, v in net.state_dict().items():
        if k not in pre_bn:
            assert rel(v.float(), ref.state_dict()[k].float()) < 1e-4, k
    for k, v in ema.state_dict().items():
        if "running" not in k and "num_batches" not in k and k not in pre_bn:
            assert rel(v.float(), ref_e.state_dict()[k].float()) < 1e-4, k


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_dncnn_kat_on_hip(dt):
    """Reference-held known-answer test on the HIP path: model_zoo/dncnn_25.pth (stored weights-only
    in dncnn_kat.npz by make_golden.py) on utils/test.bmp + sigma-25 noise -> 29.8535 dB
    (main_test_dncnn.py).  fp32 within 1e-3 dB; bf16 (split conv weights) reported and within 2e-2."""
    from kair_amd.models.network_dncnn import DnCNN
    from kair_amd.utils import utils_image as U
    z = load_golden("dncnn_kat")
    net = DnCNN(1, 1, 64, 17, "R", compute_dtype=dt)
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")}
    net.load_state_dict(sd, strict=True)
    net = net.to(dev).eval()
    L = torch.from_numpy(z["img_L"]).view(1, 1, *z["img_L"].shape).to(dev)
    with torch.no_grad():
        E = net(L).float().cpu()
    psnr = U.calculate_psnr(U.tensor2uint(E), z["img_H"], border=0)
    print(f"DnCNN KAT {dt}: {psnr:.5f} dB (reference 29.8535)")
    assert abs(psnr - 29.8535) < (1e-3 if dt == "fp32" else 2e-2), psnr
    # and the denoised image itself against the reference's recorded output
    ref = torch.from_numpy(z["E"])
    assert (E.squeeze() - ref).abs().max().item() < (1e-4 if dt == "fp32" else 2e-2)
