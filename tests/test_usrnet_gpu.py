"""USRNet on the MI355X vs the reference golden vectors and the CPU oracle.

Tolerances: the FFT / DataNet kernels (fp32 complex) within 2e-5 relative (L2) of a float64 torch
reference; the whole network in fp32 parity mode — output within 1e-4 relative, every parameter
gradient within 5e-3 and their mean within 1e-3 (fp32 DFT rounding passes through the 1/alpha of the
closed form in every unrolled iteration; measured worst 2.9e-3); bf16 mode — output within 2e-2, every gradient within 0.2 and their mean within
5e-2 (bf16 GEMM operands, fp32 accumulation and DFTs: the unrolled iterations compound the operand
rounding on the small-norm ResBlock weight gradients, measured 0.08-0.115 on 4 of 58 tensors).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from conftest import load_golden, sub_grads, sub_state  # noqa: E402
from kair_amd import _hip as H  # noqa: E402
from kair_amd.models.network_usrnet import USRNet  # noqa: E402
from oracle import convnets as ocv  # noqa: E402

dev = torch.device("cuda")
TOL = {"fp32": (1e-4, 5e-3, 1e-3), "bf16": (2e-2, 0.2, 5e-2)}   # out, worst grad, mean grad


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def untranspose(t, planes, Hh, Ww):
    """kernel layout float2 [planes][W][H] -> complex128 [planes, H, W] on the CPU"""
    return torch.view_as_complex(t.view(planes, Ww, Hh, 2).double().cpu().contiguous()).transpose(-1, -2)


def fb_gpu(k, Hh, Ww, sf):
    B = k.shape[0]
    FB = torch.empty(B * Hh * Ww * 2, device=dev)
    invW = torch.empty(B * (Hh // sf) * (Ww // sf), device=dev)
    kd = k.float().to(dev).contiguous()
    H.usr_fft_rows(kd, H.USR_SRC_PSF, 1, 0, k.shape[-2], k.shape[-1], 1, FB, B, Hh, Ww)
    H.usr_fft_cols(H.USR_COL_FB, FB, FB, None, None, None, invW, None, 0, None, B, 1, Hh, Ww, sf)
    return FB, invW


def fbfy_gpu(FB, invW, y, sf):
    B, C, h, w = y.shape
    Hh, Ww = h * sf, w * sf
    FBFy = torch.empty(B * C * Hh * Ww * 2, device=dev)
    H.usr_fft_rows(y.float().to(dev).contiguous(), H.USR_SRC_ZUP, C, 0, 0, 0, sf, FBFy, B * C, Hh, Ww)
    H.usr_fft_cols(H.USR_COL_FBFY, FBFy, FBFy, FB, None, None, invW, None, 0, None, B * C, C, Hh, Ww, sf)
    return FBFy


def datanet_gpu(x, FB, invW, FBFy, alpha, sf, FR=None):
    B, C, Hh, Ww = x.shape
    T = torch.empty(B * C * Hh * Ww * 2, device=dev)
    z = torch.empty(B, C, Hh, Ww, device=dev)
    H.usr_fft_rows(x.float().to(dev).contiguous(), H.USR_SRC_NCHW, C, 0, 0, 0, 1, T, B * C, Hh, Ww)
    H.usr_fft_cols(H.USR_COL_DATA_FWD, T, T, FB, FBFy, FR, invW, alpha.float().to(dev).contiguous(), 1, None, B * C, C,
                   Hh, Ww, sf)
    H.usr_ifft_rows(T, z, False, C, 0, 1.0 / (Hh * Ww), B * C, Hh, Ww)
    return z


def rand_kernel(B, n, g):
    k = torch.rand(B, 1, n, n, generator=g, dtype=torch.float64)
    return k / k.sum((-2, -1), keepdim=True)


@pytest.mark.parametrize("Hh,Ww,sf", [(64, 64, 4), (96, 96, 3), (512, 512, 4), (64, 48, 2), (96, 64, 1)])
def test_p2o_and_alias_mean_vs_torch(Hh, Ww, sf):
    """FB = p2o(k) (v1:48-69) and invW = mean(splits(|FB|^2, sf)) (v1:188) vs float64 torch.fft."""
    g = torch.Generator().manual_seed(Hh + Ww + sf)
    k = rand_kernel(2, 25, g)
    FB, invW = fb_gpu(k, Hh, Ww, sf)
    ref = ocv.p2o(k, (Hh, Ww))
    assert rel(torch.view_as_real(untranspose(FB, 2, Hh, Ww)), torch.view_as_real(ref[:, 0])) < 2e-6
    ref_w = ocv.splits(torch.abs(ref) ** 2, sf).mean(-1)                     # [2, 1, H/sf, W/sf]
    got_w = invW.view(2, Ww // sf, Hh // sf).transpose(-1, -2).cpu().double()
    assert rel(got_w, ref_w[:, 0]) < 2e-6


def test_datanet_vs_golden():
    """The reference DataNet (imported in this container) at a 64x64 HR grid, sf 4 (golden vectors)."""
    z = load_golden("usrnet")
    k = torch.from_numpy(z["k"])
    FB, invW = fb_gpu(k, 64, 64, 4)
    got = untranspose(FB, 1, 64, 64)
    assert rel(got.real, torch.from_numpy(z["datanet.FB_re"])[0, 0]) < 2e-6
    assert rel(got.imag, torch.from_numpy(z["datanet.FB_im"])[0, 0]) < 2e-6
    FBFy = fbfy_gpu(FB, invW, torch.from_numpy(z["datanet.y"]), 4)
    out = datanet_gpu(torch.from_numpy(z["datanet.x"]), FB, invW, FBFy, torch.from_numpy(z["datanet.alpha"]).view(1), 4)
    assert rel(out, torch.from_numpy(z["datanet.z"])) < 2e-5


@pytest.mark.parametrize("Hh,Ww,sf", [(64, 64, 4), (96, 96, 3), (128, 64, 2)])
def test_datanet_backward_vs_autograd(Hh, Ww, sf):
    """dL/dx and dL/dalpha of the closed-form step vs torch autograd through the float64 oracle."""
    g = torch.Generator().manual_seed(7 * Hh + sf)
    B, C = 2, 3
    k = rand_kernel(B, 13, g)
    y = torch.rand(B, C, Hh // sf, Ww // sf, generator=g, dtype=torch.float64)
    x = torch.rand(B, C, Hh, Ww, generator=g, dtype=torch.float64, requires_grad=True)
    alpha = (torch.rand(B, 1, 1, 1, generator=g, dtype=torch.float64) * 0.2 + 0.01).requires_grad_(True)
    gz = torch.randn(B, C, Hh, Ww, generator=g, dtype=torch.float64)
    FBr = ocv.p2o(k, (Hh, Ww))
    FBFyr = torch.conj(FBr) * torch.fft.fftn(ocv.zero_upsample(y, sf), dim=(-2, -1))
    zr = ocv.datanet(x, FBr, torch.conj(FBr), torch.abs(FBr) ** 2, FBFyr, alpha, sf)
    zr.backward(gz)
    FB, invW = fb_gpu(k, Hh, Ww, sf)
    FBFy = fbfy_gpu(FB, invW, y, sf)
    FR = torch.empty(B * C * Hh * Ww * 2, device=dev)
    al = alpha.detach().view(B).float().to(dev)
    zg = datanet_gpu(x.detach(), FB, invW, FBFy, al, sf, FR=FR)
    assert rel(zg, zr) < 2e-5
    # backward: rows of dL/dz (NHWC source, ld 8) -> closed-form adjoint -> inverse rows
    gx_nhwc = torch.zeros(B, Hh, Ww, 8, device=dev)
    gx_nhwc[..., :C] = gz.permute(0, 2, 3, 1).float().to(dev)
    T = torch.empty_like(FR)
    part = torch.empty(B * C * (Ww // sf), device=dev)
    gal = torch.empty(B, device=dev)
    H.usr_fft_rows(gx_nhwc, H.USR_SRC_NHWC, C, 8, 0, 0, 1, T, B * C, Hh, Ww)
    H.usr_fft_cols(H.USR_COL_DATA_BWD, T, T, FB, FBFy, FR, invW, al, 1, part, B * C, C, Hh, Ww, sf)
    H.usr_seg_sum(part, C * (Ww // sf), B, 1.0 / (Hh * Ww), gal, 1)
    gx = torch.empty(B, C, Hh, Ww, device=dev)
    H.usr_ifft_rows(T, gx, False, C, 0, 1.0 / (Hh * Ww), B * C, Hh, Ww)
    assert rel(gx, x.grad) < 5e-5
    assert rel(gal, alpha.grad.view(B)) < 1e-4


def _usrnet_fwd_bwd_check(net, x, k, sf, sigma, out_ref, gout, grads_ref, dt):
    out = net(x.to(dev), k.to(dev), sf, sigma.to(dev))
    assert rel(out, out_ref) < TOL[dt][0]
    out.backward(gout.to(dev))
    errs = {name: rel(p.grad, grads_ref[name]) for name, p in net.named_parameters()}
    bad = {k: e for k, e in errs.items() if e > TOL[dt][1]}
    assert not bad, bad
    assert sum(errs.values()) / len(errs) < TOL[dt][2], sorted(errs.items(), key=lambda kv: -kv[1])[:5]


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_usrnet_vs_golden(dt):
    """The reference USRNet (n_iter 2, nc 16/32/64/64, HR 64x64, sf 4): output and every gradient."""
    z = load_golden("usrnet")
    net = USRNet(n_iter=2, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2, compute_dtype=dt)
    net.load_state_dict(sub_state(z, ""), strict=True)
    net = net.to(dev).train()
    _usrnet_fwd_bwd_check(net, torch.from_numpy(z["x"]), torch.from_numpy(z["k"]), int(z["sf"]),
                          torch.from_numpy(z["sigma"]), torch.from_numpy(z["out"]), torch.from_numpy(z["gout"]),
                          sub_grads(z, ""), dt)


@pytest.mark.parametrize("lq,sf,n_iter,B", [(32, 4, 6, 2), (32, 3, 2, 2), (24, 2, 3, 2), (128, 4, 6, 1), (27, 4, 2, 1),
                                             (18, 3, 2, 2)])
def test_usrnet_option_config_vs_oracle(lq, sf, n_iter, B):
    """train_usrnet.json widths (h_nc 32, nc 16/32/64/64, nb 2), fp32 parity mode vs the CPU oracle;
    (128, 4, 6, 1) is config C3 at its configured size: 128-px LQ, x4, i.e. a 512^2 HR grid through six
    DataNet + ResUNet stages (network_usrnet_v1.py:237-262), forward and every parameter gradient.
    (27, 4) and (18, 3): HR 108^2 / 54^2, not multiples of 8 -- the ResUNet's ReplicationPad2d and crop
    (v1:148-151, 164) and their adjoints."""
    torch.manual_seed(21 + sf)
    net = USRNet(n_iter=n_iter, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2, compute_dtype="fp32")
    ref = ocv.USRNet(n_iter=n_iter, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2)
    ref.load_state_dict(net.state_dict(), strict=True)
    g = torch.Generator().manual_seed(22 + sf)
    x = torch.rand(B, 3, lq, lq, generator=g)
    k = rand_kernel(B, 25, g).float()
    sigma = torch.rand(B, 1, 1, 1, generator=g) * (25.0 / 255)
    out_ref = ref(x, k, sf, sigma)
    gout = torch.randn(out_ref.shape, generator=g)
    out_ref.backward(gout)
    grads = {n: p.grad for n, p in ref.named_parameters()}
    _usrnet_fwd_bwd_check(net.to(dev).train(), x, k, sf, sigma, out_ref, gout, grads, "fp32")


def test_usrnet_modelplain4_step():
    """define_Model('plain4') drives the USRNet engine through the fused, graph-captured trainer
    (ModelPlain4: (k, sf, sigma) are the step's extra inputs)."""
    from kair_amd.models.select_model import define_Model
    from kair_amd.utils.utils_option import dict_to_nonedict
    opt = {"model": "plain4", "is_train": True, "dist": False, "gpu_ids": [0], "scale": 4, "path": {"models": "/tmp/k"},
           "netG": {"net_type": "usrnet", "n_iter": 2, "h_nc": 32, "in_nc": 4, "out_nc": 3, "nc": [16, 32, 64, 64],
                    "nb": 2, "act_mode": "R", "downsample_mode": "strideconv", "upsample_mode": "convtranspose",
                    "init_type": "orthogonal", "init_bn_type": "uniform", "init_gain": 0.2},
           "train": {"G_lossfn_type": "l1", "G_lossfn_weight": 1.0, "G_optimizer_type": "adam", "G_optimizer_lr": 1e-4,
                     "G_optimizer_betas": [0.9, 0.999], "G_optimizer_wd": 0, "G_optimizer_clipgrad": None,
                     "G_optimizer_reuse": False, "G_scheduler_type": "MultiStepLR", "G_scheduler_milestones": [100],
                     "G_scheduler_gamma": 0.5, "E_decay": 0, "G_param_strict": True, "E_param_strict": True}}
    model = define_Model(dict_to_nonedict(opt))
    model.init_train()
    g = torch.Generator().manual_seed(3)
    B = 2
    data = {"L": torch.rand(B, 3, 16, 16, generator=g), "H": torch.rand(B, 3, 64, 64, generator=g),
            "k": rand_kernel(B, 25, g).float(), "sf": torch.full((B, 1), 4), "sigma": torch.full((B, 1, 1, 1), 0.02)}
    before = {k: v.detach().clone() for k, v in model.netG.state_dict().items()}
    losses = []
    for step in range(3):
        model.feed_data(data)
        model.optimize_parameters(step)
        losses.append(model.log_dict["G_loss"])
    after = model.netG.state_dict()
    assert model.trainer is not None and model.trainer.graph is not None   # fused path, captured at step 3
    assert all(torch.isfinite(torch.tensor(losses)))
    assert any((after[k] - before[k]).abs().max() > 0 for k in before)


def test_usrnet_fused_trainer_vs_oracle_trainer():
    """4 graph-captured FusedTrainer steps of USRNet (fp32 mode: L1, Adam, EMA) against the oracle
    trainer on the same (L, k, sf, sigma) batches (model_plain4.py:22-23 / model_plain.py:270-318)."""
    from kair_amd.engine.trainer import FusedTrainer
    from oracle.train import OracleTrainer
    torch.manual_seed(31)
    mk = lambda: USRNet(n_iter=2, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2, compute_dtype="fp32")
    net, ema = mk(), mk()
    ema.load_state_dict(net.state_dict())
    ref = ocv.USRNet(n_iter=2, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2)
    ref_e = ocv.USRNet(n_iter=2, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2)
    ref.load_state_dict(net.state_dict(), strict=True)
    ref_e.load_state_dict(net.state_dict(), strict=True)
    net, ema = net.to(dev).train(), ema.to(dev).eval()
    tr = FusedTrainer(net, ema, lr=1e-4, E_decay=0.999, use_graph=True)
    otr = OracleTrainer(ref, ref_e, lr=1e-4, E_decay=0.999)
    g = torch.Generator().manual_seed(32)
    B, sf = 2, 4
    for _ in range(4):
        L = torch.rand(B, 3, 16, 16, generator=g)
        Hh = torch.rand(B, 3, 64, 64, generator=g)
        k = rand_kernel(B, 25, g).float()
        sigma = torch.rand(B, 1, 1, 1, generator=g) * (25.0 / 255)
        loss = tr.step(L.to(dev), Hh.to(dev), k.to(dev), sf, sigma.to(dev)).item()
        _, lo = otr.optimize_parameters(L, Hh, forward=lambda x: ref(x, k, sf, sigma))
        assert abs(loss - lo) < 1e-4 * abs(lo), (loss, lo)
    assert tr.graph is not None
    sd, sdr = net.state_dict(), ref.state_dict()
    for key in sdr:
        a, b = sd[key].double().cpu(), sdr[key].double()
        r = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert r < (1e-3 if sdr[key].dim() == 1 else 1e-4), (key, r)
