"""hi/lo split activations (kair_operand.a_split / kair_epilogue.out_lo / kair_image_to_nhwc_hilo), the
operand precision of the split bf16 engine's forward convs: with split weights AND split activations a
bf16 conv must carry both operands to ~2^-16 (float64 reference), against ~2^-9 when either is plain
bf16.  Paths: the two-pass halo conv (fp32 image, with and without residual), the register-staged
implicit GEMM over an fp32 image (lo formed in the kernel) and over a bf16 hi/lo plane pair (PSHUF_SPM
producer writing out_lo, as the SwinIR tail does)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from kair_amd import _hip as H  # noqa: E402

dev = torch.device("cuda")


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def split_w(w, Cout, Cin, Cop=None):
    Cop = Cop or Cout
    kf = 2 * ((9 * Cin + 63) // 64) * 64
    W = torch.empty(Cop, kf, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), W, H.wmap(9, Cout, Cin, (1, Cout, Cop), (1, Cin, Cin)))
    return W


def test_image_to_nhwc_hilo():
    g = torch.Generator().manual_seed(3)
    B, C, Hh, Ww, ldc = 2, 3, 20, 24, 8
    x = torch.rand(B, C, Hh, Ww, generator=g)
    mean = torch.tensor([0.4488, 0.4371, 0.4040])
    out = torch.full((B * Hh * Ww, ldc), float("nan"), device=dev, dtype=torch.bfloat16)
    H.image_to_nhwc_hilo(x.to(dev), out, ldc, mean.to(dev), 1.0, B, C, Hh, Ww)
    torch.cuda.synchronize()
    o = out.float().cpu()
    ref = ((x - mean.view(1, -1, 1, 1)) * 1.0).permute(0, 2, 3, 1).reshape(-1, C).double()
    rec = o[:, :C].double() + o[:, 4:4 + C].double()
    assert torch.equal(o[:, :C], ref.float().bfloat16().float())
    assert (rec - ref).abs().max().item() < 2 ** -17 * ref.abs().max().item()
    assert o[:, C:4].abs().max().item() == 0 and o[:, 4 + C:].abs().max().item() == 0


def test_conv_first_tied_weights():
    """conv_first over the hi/lo input: weights packed tied over both channel halves (kair_wmap kG = 2):
    the conv sees the fp32 image and weights to ~2^-16."""
    g = torch.Generator().manual_seed(5)
    B, C, Hh, Ww, Cout, Cip = 2, 3, 16, 24, 180, 8
    x = torch.rand(B, C, Hh, Ww, generator=g)
    w = torch.randn(Cout, C, 3, 3, generator=g) * 0.1
    ref = torch.nn.functional.conv2d(x.double(), w.double(), padding=1)
    M = B * Hh * Ww
    xin = torch.empty(M, Cip, device=dev, dtype=torch.bfloat16)
    H.image_to_nhwc_hilo(x.to(dev), xin, Cip, None, 1.0, B, C, Hh, Ww)
    kf = 2 * ((9 * Cip + 63) // 64) * 64
    W = torch.empty(192, kf, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), W, H.wmap(9, Cout, C, (1, Cout, 192), (2, C, Cip // 2)))
    out = torch.empty(M, 192, device=dev)
    H.gemm_nt(H.im2col(xin, Hh, Ww, Cip), H.rows(W, w_split=True), H.epilogue(out), M, 192, 9 * Cip, H.BF16)
    torch.cuda.synchronize()
    got = out[:, :Cout].cpu().view(B, Hh, Ww, Cout).permute(0, 3, 1, 2)
    assert rel_err(got, ref) < 3e-5


@pytest.mark.parametrize("resid", [False, True])
@pytest.mark.parametrize("shape", [(2, 48, 48, 192, 180), (2, 48, 48, 192, 64), (1, 16, 16, 64, 64)])
def test_conv_asplit_fp32_image(shape, resid):
    """fp32 image: the halo kernel's second (lo) pass for N <= 192, with the residual epilogue; the
    first two shapes are the RSTB conv and conv_before_upsample of SwinIR classical x4."""
    B, Hh, Ww, Cin, Cout = shape
    g = torch.Generator().manual_seed(Hh + Cout + resid)
    x = torch.randn(B, Cin, Hh, Ww, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * 0.05
    bias = torch.randn(Cout, generator=g)
    M = B * Hh * Ww
    r = torch.randn(M, Cout, generator=g) if resid else None
    ref = torch.nn.functional.conv2d(x.double(), w.double(), padding=1) + bias.double().view(1, -1, 1, 1)
    if resid:
        ref = ref + r.double().view(B, Hh, Ww, Cout).permute(0, 3, 1, 2)
    xin = x.permute(0, 2, 3, 1).contiguous().view(M, Cin).to(dev)
    W = split_w(w, Cout, Cin)
    errs = []
    for split in (True, False):
        out = torch.empty(M, Cout, device=dev)
        A = H.im2col(xin, Hh, Ww, Cin)
        if split:
            A = H.asplit(A)
        H.gemm_nt(A, H.rows(W, w_split=True), H.epilogue(out, bias=bias.to(dev), resid=r.to(dev) if resid else None),
                  M, Cout, 9 * Cin, H.BF16)
        torch.cuda.synchronize()
        errs.append(rel_err(out.cpu().view(B, Hh, Ww, Cout).permute(0, 3, 1, 2), ref))
    assert errs[0] < 3e-5 and errs[1] > 8 * errs[0], errs


@pytest.mark.parametrize("hw", [(12, 16), (8, 8)])
def test_conv_asplit_hilo_pairs(hw):
    """The SwinIR x4 tail chain under split_act: a producer conv (fp32 image, two-pass split) writes its
    PixelShuffle output as a [hi | lo] pair (PSHUF_SPM, out_lo = the second half of each 128-wide row);
    a second upsampling conv reads the pair as one 128-channel image through weights tied over both
    halves (a_split 2: the halo kernel, N = 256 in two 128-wide tiles, skips lo . lo); conv_last-style
    N = 16 convs read the hi half with the lo half as lo plane (a_split 1).  (12, 16): halo kernels;
    (8, 8): 8x8 images, the register-staged fallback for the producer."""
    B, Cin, r = 2, 64, 2
    Hh, Ww = hw
    Cmid = 64 * r * r
    g = torch.Generator().manual_seed(17)
    x = torch.randn(B, Cin, Hh, Ww, generator=g)
    w1 = torch.randn(Cmid, Cin, 3, 3, generator=g) * 0.05
    b1 = torch.randn(Cmid, generator=g) * 0.1
    w2 = torch.randn(Cmid, 64, 3, 3, generator=g) * 0.05
    w3 = torch.randn(3, 64, 3, 3, generator=g) * 0.05
    F = torch.nn.functional
    mid = F.pixel_shuffle(F.conv2d(x.double(), w1.double(), b1.double(), padding=1), r)
    mid2 = F.pixel_shuffle(F.conv2d(mid, w2.double(), padding=1), r)
    ref3 = F.conv2d(mid, w3.double(), padding=1)
    M = B * Hh * Ww
    xin = x.permute(0, 2, 3, 1).contiguous().view(M, Cin).to(dev)
    W1 = torch.empty(Cmid, 2 * ((9 * Cin + 63) // 64) * 64, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w1.to(dev), W1, H.wmap(9, Cmid, Cin, (1, Cmid, Cmid), (1, Cin, Cin), n_perm=r * r))
    b1p = torch.empty(Cmid, device=dev)
    H.pack_weight(b1.to(dev), b1p, H.wmap(4, Cmid, 0, (1, Cmid, Cmid), (1, 1, 1), n_perm=r * r))
    pair = torch.empty(M * r * r, 128, device=dev, dtype=torch.bfloat16)
    H.gemm_nt(H.asplit(H.im2col(xin, Hh, Ww, Cin)), H.rows(W1, w_split=True),
              H.epilogue(pair, mode=H.OUT_PSHUF_SPM, ldo=128, bias=b1p, ps=(r, Hh, Ww), out_lo=pair[:, 64:]),
              M, Cmid, 9 * Cin, H.BF16)
    torch.cuda.synchronize()
    mid_got = (pair[:, :64].double() + pair[:, 64:].double()).cpu().view(B, Hh * r, Ww * r, 64).permute(0, 3, 1, 2)
    assert rel_err(mid_got, mid) < 3e-5
    h2, w2_ = Hh * r, Ww * r
    M2 = B * h2 * w2_
    # second upsampling conv over the pair image, tied split weights
    W2 = torch.empty(Cmid, 2 * 9 * 128, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w2.to(dev), W2, H.wmap(9, Cmid, 64, (1, Cmid, Cmid), (2, 64, 64), n_perm=r * r))
    out2 = torch.empty(M2 * r * r, 64, device=dev)
    H.gemm_nt(H.asplit(H.im2col(pair, h2, w2_, 128), pair=True), H.rows(W2, w_split=True),
              H.epilogue(out2, mode=H.OUT_PSHUF_SPM, ldo=64, ps=(r, h2, w2_)), M2, Cmid, 9 * 128, H.BF16)
    torch.cuda.synchronize()
    got2 = out2.cpu().view(B, h2 * r, w2_ * r, 64).permute(0, 3, 1, 2)
    assert rel_err(got2, mid2) < 5e-5
    # conv_last over the pair: hi half + lo plane, and the hi half alone (plain bf16 activation)
    W3 = split_w(w3, 3, 64, Cop=16)
    errs = []
    for split in (True, False):
        img = torch.empty(B, 3, h2, w2_, device=dev)
        A = H.im2col(pair, h2, w2_, 64, ld=128)
        if split:
            A = H.asplit(A, pair[:, 64:])
        H.gemm_nt(A, H.rows(W3, w_split=True), H.epilogue(img, mode=H.OUT_NCHW, ldo=0, img=(None, 1.0, 3, h2, w2_)),
                  M2, 16, 9 * 64, H.BF16)
        torch.cuda.synchronize()
        errs.append(rel_err(img, ref3))
    assert errs[0] < 5e-5 and errs[1] > 8 * errs[0], errs


def test_asplit_rejects_bad_operands():
    """a_split is an A flag for a bf16 product without rowscale / ones column; a bf16 A needs its lo plane."""
    M, K, N = 64, 64, 64
    a = torch.zeros(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
    out = torch.empty(M, N, device=dev)
    with pytest.raises(RuntimeError):
        H.gemm_nt(H.asplit(H.rows(a)), H.rows(b), H.epilogue(out), M, N, K, H.BF16)   # no lo plane
    with pytest.raises(RuntimeError):
        H.gemm_nt(H.rows(a), H.asplit(H.rows(b), a), H.epilogue(out), M, N, K, H.BF16)  # B flag
    with pytest.raises(RuntimeError):   # out_lo needs a bf16 output
        H.gemm_nt(H.rows(a), H.rows(b), H.epilogue(out, out_lo=a), M, N, K, H.BF16)
