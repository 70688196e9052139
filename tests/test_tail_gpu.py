"""The narrow-output 3x3 conv kernels (csrc/tail.hip) -- SwinIR's conv_last 64 -> 3 at the HR size
(network_swinir.py:745, :817) -- against float64 torch autograd of the same conv: forward over a hi/lo
pair image (split activations, split weights: ~2^-16 relative), input gradient into a row layout and
into the PixelUnshuffle(2) sub-pixel-major layout of the previous conv, weight + bias gradient
(deterministic: two launches agree bit for bit)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from kair_amd import _hip as H  # noqa: E402

dev = torch.device("cuda")
F = torch.nn.functional


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def pair_image(x):
    """NCHW fp32 -> NHWC bf16 [hi | lo] rows (128 channels), as the split tail stores its activations."""
    B, C, Hh, Ww = x.shape
    r = x.permute(0, 2, 3, 1).reshape(-1, C)
    hi = r.bfloat16()
    lo = (r - hi.float()).bfloat16()
    return torch.cat([hi, lo], 1).contiguous()


@pytest.mark.parametrize("NR,shape", [(3, (2, 32, 64)), (1, (1, 16, 64)), (3, (1, 48, 192))])
def test_narrow_fwd(NR, shape):
    B, Hh, Ww = shape
    g = torch.Generator().manual_seed(NR + Ww)
    x = torch.randn(B, 64, Hh, Ww, generator=g)
    w = torch.randn(NR, 64, 3, 3, generator=g) * 0.05
    b = torch.randn(NR, generator=g) * 0.1
    mean = torch.tensor([0.4488, 0.4371, 0.4040])[:NR]
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1) + mean.double().view(1, -1, 1, 1)
    xp = pair_image(x).to(dev)
    Wn = torch.empty(16, 2 * 9 * 64, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), Wn, H.wmap(15, NR, 64, (1, NR, 16), (1, 64, 64)))
    bp = torch.zeros(16, device=dev)
    bp[:NR] = b.to(dev)
    errs = []
    for lo_off in (64, 0):
        out = torch.full((B, NR, Hh, Ww), float("nan"), device=dev)
        H.conv3x3_narrow_fwd(xp, 128, lo_off, Wn, bp, NR, mean.to(dev), 1.0, None, out, B, Hh, Ww)
        torch.cuda.synchronize()
        errs.append(rel_err(out, ref))
    assert errs[0] < 3e-5 and errs[1] > 8 * errs[0], errs


@pytest.mark.parametrize("ps_r", [0, 2])
def test_narrow_dgrad(ps_r):
    B, Hh, Ww, NR = 2, 16, 64, 3
    g = torch.Generator().manual_seed(9 + ps_r)
    dE = torch.randn(B, NR, Hh, Ww, generator=g).bfloat16().float()
    w = torch.randn(NR, 64, 3, 3, generator=g) * 0.05
    x = torch.zeros(B, 64, Hh, Ww, dtype=torch.float64, requires_grad=True)
    F.conv2d(x, w.double(), padding=1).backward(dE.double())
    ref = x.grad   # [B, 64, H, W]
    rows = torch.zeros(B * Hh * Ww, 16)
    rows[:, :NR] = dE.permute(0, 2, 3, 1).reshape(-1, NR)
    dEd = rows.to(dev, torch.bfloat16)
    ws = torch.empty(H.conv3x3_narrow_dgrad_ws(), device=dev)
    if ps_r:
        r = ps_r
        out = torch.full((B * (Hh // r) * (Ww // r), r * r * 64), float("nan"), device=dev, dtype=torch.bfloat16)
        H.conv3x3_narrow_dgrad(dEd, 16, w.to(dev), NR, ws, out, r * r * 64, r, B, Hh, Ww)
        torch.cuda.synchronize()
        # pre-shuffle row (b, y, x), column (i r + j) 64 + c  ->  pixel (b, y r + i, x r + j), channel c
        got = out.float().cpu().view(B, Hh // r, Ww // r, r, r, 64).permute(0, 5, 1, 3, 2, 4).reshape(B, 64, Hh, Ww)
    else:
        out = torch.full((B * Hh * Ww, 64), float("nan"), device=dev)
        H.conv3x3_narrow_dgrad(dEd, 16, w.to(dev), NR, ws, out, 64, 0, B, Hh, Ww)
        torch.cuda.synchronize()
        got = out.cpu().view(B, Hh, Ww, 64).permute(0, 3, 1, 2)
    assert rel_err(got, ref) < (4e-3 if ps_r else 3e-3)   # bf16 weights (MFMA), bf16 output for ps_r


def test_narrow_wgrad():
    B, Hh, Ww, NR = 2, 48, 64, 3
    g = torch.Generator().manual_seed(21)
    x = torch.randn(B, 64, Hh, Ww, generator=g).bfloat16().float()
    dE = torch.randn(B, NR, Hh, Ww, generator=g).bfloat16().float()
    w = torch.zeros(NR, 64, 3, 3, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(NR, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.double(), w, b, padding=1).backward(dE.double())
    rows = torch.zeros(B * Hh * Ww, 16)
    rows[:, :NR] = dE.permute(0, 2, 3, 1).reshape(-1, NR)
    xp = pair_image(x).to(dev)   # the hi half is read (ld 128)
    ws = torch.empty(H.conv3x3_narrow_wgrad_ws(NR), device=dev)
    outs = []
    for _ in range(2):
        gw = torch.full((NR, 64, 3, 3), float("nan"), device=dev)
        gb = torch.full((NR,), float("nan"), device=dev)
        H.conv3x3_narrow_wgrad(rows.to(dev, torch.bfloat16), 16, xp, 128, NR, ws, gw, gb, B, Hh, Ww)
        torch.cuda.synchronize()
        outs.append((gw.cpu(), gb.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert rel_err(outs[0][0], w.grad) < 1e-5
    assert rel_err(outs[0][1], b.grad) < 1e-5


@pytest.mark.parametrize("mode", ["punshuf", "gate"])
def test_halo_channel_groups(mode):
    """The upsampling convs' input gradients (network_swinir.py:584 Upsample, its backward): a 256-channel
    image (the pre-shuffle gradient) through the 3x3 halo kernel in four 64-channel passes, into the
    PixelUnshuffle(2) sub-pixel-major layout of the previous conv ("punshuf") or, gated by LeakyReLU'
    of a stored activation, into plain rows ("gate") -- vs float64 conv_transpose (flipped taps)."""
    B, Hh, Ww, C, N = 2, 24, 48, 256, 64
    g = torch.Generator().manual_seed(31)
    x = torch.randn(B, C, Hh, Ww, generator=g).bfloat16().float()
    w = (torch.randn(C, N, 3, 3, generator=g) * 0.03).bfloat16().float()   # forward conv N -> C
    # dgrad of a forward conv N -> C: dX = conv_transpose(x, w)
    ref = F.conv_transpose2d(x.double(), w.double(), padding=1)   # [B, N, H, W]
    M = B * Hh * Ww
    xin = x.permute(0, 2, 3, 1).contiguous().view(M, C).to(dev, torch.bfloat16)
    Wd = torch.empty(N, 9 * C, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), Wd, H.wmap(2, C, N, (1, C, C), (1, N, N)))
    A = H.im2col(xin, Hh, Ww, C, flip=True)
    if mode == "punshuf":
        r = 2
        out = torch.full((M // (r * r), r * r * N), float("nan"), device=dev)
        H.gemm_nt(A, H.rows(Wd), H.epilogue(out, mode=H.OUT_PUNSHUF_SPM, ldo=r * r * N, ps=(r, Hh // r, Ww // r)), M, N,
                  9 * C, H.BF16)
        torch.cuda.synchronize()
        got = out.cpu().view(B, Hh // r, Ww // r, r, r, N).permute(0, 5, 1, 3, 2, 4).reshape(B, N, Hh, Ww)
    else:
        gate = torch.randn(M, 128, generator=g).bfloat16()
        out = torch.full((M, N), float("nan"), device=dev)
        H.gemm_nt(A, H.rows(Wd), H.epilogue(out, gate=gate.to(dev), ldg=128, gate_kind=2, slope=0.01), M, N, 9 * C, H.BF16)
        torch.cuda.synchronize()
        got = out.cpu().view(B, Hh, Ww, N).permute(0, 3, 1, 2)
        gs = torch.where(gate[:, :N].float() > 0, 1.0, 0.01).view(B, Hh, Ww, N).permute(0, 3, 1, 2)
        ref = ref * gs.double()
    assert rel_err(got, ref) < 1e-5


# ---- fp32x3 forms (fp32 operands as fp16 pairs, three products): the fp32 engine's 1e-5-class bar ----------
def rows_of(t, ld):
    """NCHW fp32 -> NHWC fp32 rows of ld channels (zero padded)."""
    B, C, Hh, Ww = t.shape
    r = torch.zeros(B * Hh * Ww, ld)
    r[:, :C] = t.permute(0, 2, 3, 1).reshape(-1, C)
    return r


@pytest.mark.parametrize("NR,shape", [(3, (2, 32, 64)), (1, (1, 16, 128)), (3, (1, 48, 192))])
def test_narrow_fwd_x3(NR, shape):
    B, Hh, Ww = shape
    g = torch.Generator().manual_seed(40 + NR + Ww)
    x = torch.randn(B, 64, Hh, Ww, generator=g)
    w = torch.randn(NR, 64, 3, 3, generator=g) * 0.05
    b = torch.randn(NR, generator=g) * 0.1
    mean = torch.tensor([0.4488, 0.4371, 0.4040])[:NR]
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1) + mean.double().view(1, -1, 1, 1)
    bp = torch.zeros(16, device=dev)
    bp[:NR] = b.to(dev)
    ws = torch.empty(H.conv3x3_narrow_x3_ws(), device=dev)
    out = torch.full((B, NR, Hh, Ww), float("nan"), device=dev)
    H.conv3x3_narrow_fwd_x3(rows_of(x, 64).to(dev), 64, 4, w.to(dev), bp, NR, ws, mean.to(dev), 1.0, None, out, B, Hh, Ww)
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 2e-6


@pytest.mark.parametrize("ps_r", [0, 2])
def test_narrow_dgrad_x3(ps_r):
    B, Hh, Ww, NR = 2, 16, 64, 3
    g = torch.Generator().manual_seed(49 + ps_r)
    dE = torch.randn(B, NR, Hh, Ww, generator=g) * 2.0 ** -12   # a mean-loss gradient's scale, exponent 12 + 4
    w = torch.randn(NR, 64, 3, 3, generator=g) * 0.05
    x = torch.zeros(B, 64, Hh, Ww, dtype=torch.float64, requires_grad=True)
    F.conv2d(x, w.double(), padding=1).backward(dE.double())
    ref = x.grad
    dEd = rows_of(dE, 16).to(dev)
    ws = torch.empty(H.conv3x3_narrow_x3_ws(), device=dev)
    if ps_r:
        r = ps_r
        out = torch.full((B * (Hh // r) * (Ww // r), r * r * 64), float("nan"), device=dev)
        H.conv3x3_narrow_dgrad_x3(dEd, 16, 16, w.to(dev), NR, ws, out, r * r * 64, r, B, Hh, Ww)
        torch.cuda.synchronize()
        got = out.cpu().view(B, Hh // r, Ww // r, r, r, 64).permute(0, 5, 1, 3, 2, 4).reshape(B, 64, Hh, Ww)
    else:
        out = torch.full((B * Hh * Ww, 64), float("nan"), device=dev)
        H.conv3x3_narrow_dgrad_x3(dEd, 16, 16, w.to(dev), NR, ws, out, 64, 0, B, Hh, Ww)
        torch.cuda.synchronize()
        got = out.cpu().view(B, Hh, Ww, 64).permute(0, 3, 1, 2)
    assert rel_err(got, ref) < 2e-6


def test_narrow_wgrad_x3():
    B, Hh, Ww, NR = 2, 48, 64, 3
    g = torch.Generator().manual_seed(61)
    x = torch.randn(B, 64, Hh, Ww, generator=g)
    dE = torch.randn(B, NR, Hh, Ww, generator=g) * 2.0 ** -12
    w = torch.zeros(NR, 64, 3, 3, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(NR, dtype=torch.float64, requires_grad=True)
    F.conv2d(x.double(), w, b, padding=1).backward(dE.double())
    ws = torch.empty(H.conv3x3_narrow_wgrad_ws(NR), device=dev)
    outs = []
    for _ in range(2):
        gw = torch.full((NR, 64, 3, 3), float("nan"), device=dev)
        gb = torch.full((NR,), float("nan"), device=dev)
        H.conv3x3_narrow_wgrad_x3(rows_of(dE, 16).to(dev), 16, 16, rows_of(x, 64).to(dev), 64, 4, NR, ws, gw, gb, B, Hh, Ww)
        torch.cuda.synchronize()
        outs.append((gw.cpu(), gb.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert rel_err(outs[0][0], w.grad) < 2e-6
    assert rel_err(outs[0][1], b.grad) < 2e-6
