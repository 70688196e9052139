"""Per-kernel parity on the MI355X: every libkair_hip entry point against a plain fp32 PyTorch
reference of the same op (CPU, float64 where cheap).  fp32 compute mode must match to ~1e-5
relative (exact fp32 MFMA); bf16 mode to bf16 rounding (~1e-2 relative)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from kair_amd import _hip as H  # noqa: E402
from oracle.swinir import relative_position_index, shift_region_mask  # noqa: E402

dev = torch.device("cuda")
TOL = {H.F32: (2e-5, 2e-5), H.BF16: (2e-2, 2e-2)}
DT = {H.F32: torch.float32, H.BF16: torch.bfloat16}


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def win_perm(B, Hh, Ww, ws, shift):
    """row m (window order) -> token index, as the kernels' WinMap does"""
    idx = torch.arange(B * Hh * Ww).view(B, Hh, Ww)
    idx = torch.roll(idx, (-shift, -shift), (1, 2))
    return idx.view(B, Hh // ws, ws, Ww // ws, ws).permute(0, 1, 3, 2, 4).reshape(-1)


@pytest.mark.parametrize("compute", [H.F32, H.BF16])
@pytest.mark.parametrize("M,N,K", [(1000, 576, 192), (4096, 180, 192), (333, 16, 72), (2048, 64, 1728)])
def test_gemm_nt_rows(compute, M, N, K):
    g = torch.Generator().manual_seed(M + N)
    a = torch.randn(M, K, generator=g)
    b = torch.randn(N, K, generator=g) * 0.1
    bias = torch.randn(N, generator=g)
    ref = a.double() @ b.double().T + bias.double()
    A = a.to(dev, DT[compute])
    Bw = b.to(dev, DT[compute])
    out = torch.empty(M, N, device=dev)
    H.gemm_nt(H.rows(A), H.rows(Bw), H.epilogue(out, bias=bias.to(dev)), M, N, K, compute)
    torch.cuda.synchronize()
    assert rel_err(out, ref) < TOL[compute][0]


@pytest.mark.parametrize("compute", [H.F32, H.BF16])
def test_gemm_window_map_gelu_resid(compute):
    B, Hh, Ww, ws, shift, C, N = 2, 16, 24, 8, 4, 64, 96
    M = B * Hh * Ww
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, C, generator=g)
    w = torch.randn(N, C, generator=g) * 0.1
    res = torch.randn(M, N, generator=g)
    perm = win_perm(B, Hh, Ww, ws, shift)
    win = (Hh, Ww, ws, shift)
    # A gathered through the window map, output scattered back to token rows, + residual
    out = torch.empty(M, N, device=dev)
    pre = torch.empty(M, N, device=dev)
    H.gemm_nt(H.rows(x.to(dev, DT[compute]), win=win), H.rows(w.to(dev, DT[compute])),
              H.epilogue(out, win=win, act=H.ACT_GELU, pre=pre, resid=res.to(dev)), M, N, C, compute)
    torch.cuda.synchronize()
    y_win = x[perm] @ w.T                      # rows in window order
    ref = torch.empty(M, N)
    ref[perm] = torch.nn.functional.gelu(y_win)
    ref += res
    pref = torch.empty(M, N)
    pref[perm] = y_win
    assert rel_err(out, ref) < TOL[compute][0]
    assert rel_err(pre, pref) < TOL[compute][0]


@pytest.mark.parametrize("compute", [H.F32, H.BF16])
@pytest.mark.parametrize("flip", [False, True])
def test_conv3x3_implicit_gemm(compute, flip):
    B, Hh, Ww, Cin, Cout = 2, 12, 20, 24, 40
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, Cin, Hh, Ww, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1
    if flip:  # dgrad: conv of dy with the transposed kernel == conv_transpose
        ref = torch.nn.functional.conv_transpose2d(x, w.transpose(0, 1).contiguous(), padding=1)  # Cin->Cout flipped
        wk = w.transpose(0, 1).contiguous()  # [Cin_as_out? ] build packed [Cout][9*Cin] for transpose conv
        # conv_transpose2d(x, W') with W' [Cin, Cout, 3, 3] == sum_tap x[p - off] W'[ci, co, tap]
        packed = wk.permute(1, 2, 3, 0).reshape(Cout, 9 * Cin)  # [co][tap*Cin + ci] = W'[ci][co][tap]
    else:
        ref = torch.nn.functional.conv2d(x, w, padding=1)
        packed = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)  # [co][tap*Cin + ci]
    xin = x.permute(0, 2, 3, 1).contiguous().view(B * Hh * Ww, Cin)
    out = torch.empty(B * Hh * Ww, Cout, device=dev)
    H.gemm_nt(H.im2col(xin.to(dev, DT[compute]), Hh, Ww, Cin, flip=flip), H.rows(packed.to(dev, DT[compute])),
              H.epilogue(out), B * Hh * Ww, Cout, 9 * Cin, compute)
    torch.cuda.synchronize()
    got = out.cpu().view(B, Hh, Ww, Cout).permute(0, 3, 1, 2)
    assert rel_err(got, ref) < TOL[compute][0]


@pytest.mark.parametrize("shape", [(2, 48, 48, 192, 192), (1, 12, 96, 64, 64), (1, 6, 192, 64, 180), (3, 24, 32, 128, 96),
                                   (2, 16, 64, 64, 64), (1, 6, 128, 64, 60)])
@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("a_f32", [False, True])
@pytest.mark.parametrize("resid", [False, True])
def test_conv3x3_halo_path(shape, flip, a_f32, resid):
    """bf16 3x3 convs whose geometry selects the LDS-halo kernel (W | 96 or 96 | W, Cin % 64 == 0,
    N <= 192; or the 128-pixel tile for N <= 64 where 128 | W or W | 128 -- SwinIR-lightweight's 64-pixel
    rows): fp32 or bf16 input rows, forward or flipped taps, bias + optional fp32 residual."""
    B, Hh, Ww, Cin, Cout = shape
    g = torch.Generator().manual_seed(Hh * Ww + Cin)
    x = torch.randn(B, Cin, Hh, Ww, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.05).bfloat16().float()
    bias = torch.randn(Cout, generator=g)
    r = torch.randn(B * Hh * Ww, Cout, generator=g)
    if flip:
        ref = torch.nn.functional.conv_transpose2d(x, w.transpose(0, 1).contiguous(), padding=1)
        packed = w.transpose(0, 1).contiguous().permute(1, 2, 3, 0).reshape(Cout, 9 * Cin)
    else:
        ref = torch.nn.functional.conv2d(x, w, padding=1)
        packed = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin)
    ref = ref + bias.view(1, -1, 1, 1)
    xin = x.permute(0, 2, 3, 1).contiguous().view(B * Hh * Ww, Cin)
    M = B * Hh * Ww
    out = torch.empty(M, Cout, device=dev)
    A = xin.to(dev, torch.float32 if a_f32 else torch.bfloat16)
    ops = (H.im2col(A, Hh, Ww, Cin, flip=flip), H.rows(packed.to(dev, torch.bfloat16)),
           H.epilogue(out, bias=bias.to(dev), resid=r.to(dev) if resid else None))
    torch.cuda.synchronize()
    H.ktime_begin(8)
    try:
        H.gemm_nt(*ops, M, Cout, 9 * Cin, H.BF16)
    finally:
        nk = H.ktime_end()
    torch.cuda.synchronize()
    assert nk == 1 and "conv3x3_halo_kernel" in H.ktime_read(0)[1], H.ktime_read(0)[1]
    got = out.cpu()
    if resid:
        got = got - r
    got = got.view(B, Hh, Ww, Cout).permute(0, 3, 1, 2)
    assert rel_err(got, ref) < 1e-2


@pytest.mark.parametrize("shape", [(2, 48, 48, 192, 180), (2, 12, 20, 64, 256), (1, 16, 16, 8, 180), (2, 24, 24, 64, 16)])
def test_conv3x3_split_weights(shape):
    """hi/lo split bf16 weights (pack kind 9, kair_operand.w_split) through the halo kernel (first
    shape) and the register-staged kernel (others, incl. K = 72 with a partial last chunk): with
    bf16-exact activations the product must carry the fp32 weights to ~2^-16, against ~2^-9 for
    plain bf16 weights."""
    B, Hh, Ww, Cin, Cout = shape
    g = torch.Generator().manual_seed(Hh + Cin + Cout)
    x = torch.randn(B, Cin, Hh, Ww, generator=g).bfloat16().float()
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * 0.05
    bias = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), padding=1) + bias.double().view(1, -1, 1, 1)
    M = B * Hh * Ww
    xin = x.permute(0, 2, 3, 1).contiguous().view(M, Cin).to(dev, torch.bfloat16)
    kf = 2 * ((9 * Cin + 63) // 64) * 64
    Wsplit = torch.empty(Cout, kf, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), Wsplit, H.wmap(9, Cout, Cin, (1, Cout, Cout), (1, Cin, Cin)))
    Wplain = torch.empty(Cout, 9 * Cin, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), Wplain, H.wmap(1, Cout, Cin, (1, Cout, Cout), (1, Cin, Cin)))
    errs = []
    for Wb, split in ((Wsplit, True), (Wplain, False)):
        out = torch.empty(M, Cout, device=dev)
        H.gemm_nt(H.im2col(xin, Hh, Ww, Cin), H.rows(Wb, w_split=split), H.epilogue(out, bias=bias.to(dev)), M, Cout,
                  9 * Cin, H.BF16)
        torch.cuda.synchronize()
        errs.append(rel_err(out.cpu().view(B, Hh, Ww, Cout).permute(0, 3, 1, 2), ref))
    assert errs[0] < 3e-5 and errs[1] > 8 * errs[0], errs


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,Np,ld", [(100003, 16, 16), (70000, 256, 256), (4097, 64, 72), (5000, 20, 20)])
def test_colsum_bias_gradient(dt, M, Np, ld):
    """Bias gradient = column sums of the output-gradient rows (vectorised and scalar paths),
    deterministic (two launches agree bit for bit)."""
    g = torch.Generator().manual_seed(M)
    x = torch.randn(M, ld, generator=g).to(dt)
    ref = x[:, :Np].double().sum(0)
    m = H.wmap(0, Np, 0)
    out = torch.empty(Np, device=dev)
    out2 = torch.empty(Np, device=dev)
    ws = torch.empty(512 * max(Np, 256), device=dev)
    G = H.rows(x.to(dev))
    H.colsum(G, M, Np, m, out, ws)
    H.colsum(G, M, Np, m, out2, ws)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    assert (out.double().cpu() - ref).abs().max().item() < 1e-3 * (1 + ref.abs().max().item())


@pytest.mark.parametrize("compute", [H.F32, H.BF16])
def test_conv_pixelshuffle_and_nchw(compute):
    B, Hh, Ww, Cin, r = 2, 8, 8, 16, 2
    Cout = 8 * r * r
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, Cin, Hh, Ww, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * 0.1
    bias = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.pixel_shuffle(torch.nn.functional.conv2d(x, w, bias, padding=1), r)
    xin = x.permute(0, 2, 3, 1).contiguous().view(-1, Cin).to(dev, DT[compute])
    packed = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin).to(dev, DT[compute])
    out = torch.empty(B * Hh * r * Ww * r, 8, device=dev)
    H.gemm_nt(H.im2col(xin, Hh, Ww, Cin), H.rows(packed),
              H.epilogue(out, mode=H.OUT_PSHUF, bias=bias.to(dev), ps=(r, Hh, Ww)), B * Hh * Ww, Cout, 9 * Cin, compute)
    torch.cuda.synchronize()
    assert rel_err(out.cpu().view(B, Hh * r, Ww * r, 8).permute(0, 3, 1, 2), ref) < TOL[compute][0]
    # NCHW image epilogue with mean/range
    mean = torch.tensor([0.1, 0.2, 0.3])
    w3 = torch.randn(3, Cin, 3, 3, generator=g) * 0.1
    img = torch.empty(B, 3, Hh, Ww, device=dev)
    p3 = torch.zeros(16, 9 * Cin)
    p3[:3] = w3.permute(0, 2, 3, 1).reshape(3, 9 * Cin)
    H.gemm_nt(H.im2col(xin, Hh, Ww, Cin), H.rows(p3.to(dev, DT[compute])),
              H.epilogue(img, mode=H.OUT_NCHW, ldo=0, img=(mean.to(dev), 1.0, 3, Hh, Ww)), B * Hh * Ww, 16, 9 * Cin,
              compute)
    torch.cuda.synchronize()
    ref3 = torch.nn.functional.conv2d(x, w3, padding=1) + mean.view(1, 3, 1, 1)
    assert rel_err(img, ref3) < TOL[compute][0]


@pytest.mark.parametrize("in_data", [False, True])
@pytest.mark.parametrize("compute", [H.F32, H.BF16])
@pytest.mark.parametrize("M,N,K", [(5000, 576, 192), (4096, 64, 64), (777, 192, 384), (2000, 384, 200),
                                   (3000, 32, 576), (1500, 24, 152), (2500, 64, 1728)])
def test_gemm_tn_wgrad(compute, M, N, K, in_data):
    """in_data=True: the ones column is stored by the producer (bf16: the LDS-DMA ring kernel)."""
    g = torch.Generator().manual_seed(11)
    dy = torch.randn(M, N, generator=g)
    x = torch.randn(M, K, generator=g)
    ones = K - 3
    xr = x.clone()
    xr[:, ones] = 1.0
    ref = dy.double().T @ xr.double()
    S = H.wgrad_splits(M, N, K)
    ws = torch.empty(S, N, K, device=dev)
    xin = xr if in_data else x
    H.gemm_tn(H.rows(dy.to(dev, DT[compute])), H.rows(xin.to(dev, DT[compute]), ones_col=ones, ones_in_data=in_data), ws,
              S, M, N, K, compute)
    torch.cuda.synchronize()
    got = ws.sum(0).cpu()
    assert rel_err(got, ref) < TOL[compute][0]
    # finalize into reference layout [N][K-?] with bias from the ones column
    m = H.wmap(0, N, ones, (1, N, N), (1, ones, K))
    grad = torch.empty(N, ones, device=dev)
    bg = torch.empty(N, device=dev)
    H.wgrad_finalize(ws, S, m, grad, bg, ones)
    torch.cuda.synchronize()
    assert rel_err(grad, ref[:, :ones]) < TOL[compute][0]
    assert rel_err(bg, dy.double().sum(0)) < TOL[compute][0]


@pytest.mark.parametrize("compute", [H.F32, H.BF16])
def test_conv_wgrad_im2col(compute):
    B, Hh, Ww, Cin, Cout = 2, 10, 12, 16, 24
    g = torch.Generator().manual_seed(13)
    x = torch.randn(B, Cin, Hh, Ww, generator=g, requires_grad=True)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, requires_grad=True)
    y = torch.nn.functional.conv2d(x, w, padding=1)
    gy = torch.randn_like(y)
    y.backward(gy)
    M = B * Hh * Ww
    dy = gy.permute(0, 2, 3, 1).reshape(M, Cout)
    xin = x.detach().permute(0, 2, 3, 1).reshape(M, Cin)
    K = 9 * Cin
    S = H.wgrad_splits(M, Cout, K)
    ws = torch.empty(S, Cout, K, device=dev)
    H.gemm_tn(H.rows(dy.to(dev, DT[compute])), H.im2col(xin.contiguous().to(dev, DT[compute]), Hh, Ww, Cin), ws, S, M, Cout,
              K, compute)
    grad = torch.empty(Cout, Cin, 3, 3, device=dev)
    H.wgrad_finalize(ws, S, H.wmap(1, Cout, Cin), grad)
    torch.cuda.synchronize()
    assert rel_err(grad, w.grad) < TOL[compute][0]


@pytest.mark.parametrize("B,Hh,Ww,Cout", [(2, 16, 16, 180), (3, 10, 12, 96), (1, 64, 64, 180)])
def test_conv_wgrad_tap_ring(B, Hh, Ww, Cout):
    """The RSTB conv weight gradient on the tap-per-tile ring (gemm.hip BM_TAP): bf16 G rows x a bf16
    192-channel image holding 1.0 in channel C (the bias, read through the center tap), against float64
    conv2d backward on the same bf16 values (network_swinir.py:465 conv 3x3, RSTB.forward :481-482)."""
    C, Cp = 180, 192
    g = torch.Generator().manual_seed(17)
    x = torch.randn(B, C, Hh, Ww, generator=g).to(torch.bfloat16).double().requires_grad_(True)
    w = torch.randn(Cout, C, 3, 3, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(Cout, dtype=torch.float64, requires_grad=True)
    y = torch.nn.functional.conv2d(x, w, b, padding=1)
    gy = torch.randn(y.shape, generator=g).to(torch.bfloat16).double()
    y.backward(gy)
    M, Np = B * Hh * Ww, -(-Cout // 8) * 8
    dy = torch.zeros(M, Np, dtype=torch.bfloat16)
    dy[:, :Cout] = gy.permute(0, 2, 3, 1).reshape(M, Cout).to(torch.bfloat16)
    xin = torch.zeros(M, Cp, dtype=torch.bfloat16)
    xin[:, :C] = x.detach().permute(0, 2, 3, 1).reshape(M, C).to(torch.bfloat16)
    xin[:, C] = 1.0
    K, oc = 9 * Cp, 4 * Cp + C
    S = H.wgrad_splits(M, Np, K)
    assert H.wgrad_tiles(Np, K) == -(-Np // 192) * 9
    ws = torch.full((S, Np, K), float("nan"), device=dev)
    H.gemm_tn(H.rows(dy.to(dev)), H.im2col(xin.to(dev), Hh, Ww, Cp, ones_col=oc, ones_in_data=True), ws, S, M, Np, K,
              H.BF16)
    grad = torch.empty(Cout, C, 3, 3, device=dev)
    bg = torch.empty(Cout, device=dev)
    H.wgrad_finalize(ws, S, H.wmap(1, Cout, C, (1, Cout, Np), (1, C, Cp)), grad, bg, oc)
    torch.cuda.synchronize()
    assert rel_err(grad, w.grad) < 1e-5
    assert rel_err(bg, b.grad) < 1e-5


@pytest.mark.parametrize("flip", [False, True])
def test_conv_halo_acopy(flip):
    """The halo conv's side output (kair_epilogue.a_copy): the bf16 image of its fp32 A operand, channel
    ones_col forced to 1.0 -- the tap ring's weight-gradient operand -- next to an unchanged conv."""
    B, Hh, Ww, C = 2, 48, 48, 192
    M = B * Hh * Ww
    assert H.conv_halo_geometry(Hh, Ww, C, M, C) and not H.conv_halo_geometry(16, 16, C, 256, C)
    g = torch.Generator().manual_seed(19)
    x = torch.randn(M, C, generator=g).to(dev)
    w = (torch.randn(C, 9 * C, generator=g) * 0.05).to(dev, torch.bfloat16)
    out0, out1 = torch.empty(M, C, device=dev), torch.empty(M, C, device=dev)
    cp = torch.full((M, C), float("nan"), device=dev, dtype=torch.bfloat16)
    H.gemm_nt(H.im2col(x, Hh, Ww, C, flip=flip), H.rows(w), H.epilogue(out0), M, C, 9 * C, H.BF16)
    H.gemm_nt(H.im2col(x, Hh, Ww, C, flip=flip), H.rows(w), H.epilogue(out1, acopy=(cp, 180)), M, C, 9 * C, H.BF16)
    torch.cuda.synchronize()
    ref = x.to(torch.bfloat16)
    ref[:, 180] = 1.0
    assert torch.equal(out0, out1)
    assert torch.equal(cp, ref)


@pytest.mark.parametrize("dtype", [H.F32, H.BF16])
@pytest.mark.parametrize("win", [(0, 0, 0, 0), (16, 16, 8, 4)])
def test_layernorm(dtype, win):
    M, C, ld = 2 * 256, 180, 192
    g = torch.Generator().manual_seed(17)
    x = torch.zeros(M, ld)
    x[:, :C] = torch.randn(M, C, generator=g) * 2 + 0.5
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.1
    xr = x[:, :C].clone().requires_grad_(True)
    gm, bt = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    y = torch.nn.functional.layer_norm(xr, (C,), gm, bt, 1e-5)
    gy = torch.randn(M, C, generator=g)
    y.backward(gy)
    perm = win_perm(2, 16, 16, 8, 4) if win[2] else torch.arange(M)
    xd = x.to(dev)
    yo = torch.empty(M, ld, device=dev, dtype=DT[dtype])
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    H.layernorm_fwd(xd, ld, yo, ld, gamma.to(dev), beta.to(dev), mean, rstd, M, C, 1e-5, win, one_col=C + 1)
    torch.cuda.synchronize()
    assert rel_err(yo[:, :C].float(), y.detach()[perm]) < TOL[dtype][0]
    assert (yo[:, C + 1] == 1).all().item()
    yo[:, C + 1] = 0
    assert yo[:, C:].abs().max().item() == 0
    dy = torch.zeros(M, ld)
    dy[:, :C] = gy[perm]
    dx = torch.ones(M, ld, device=dev)  # accumulate onto ones
    dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
    ws = torch.empty(2 * 2048 * C, device=dev)
    # GEMM-operand copy of the finished dx: per-sample scale, Swin window order (the other map)
    cwin = (16, 16, 8, 4) if not win[2] else None
    sc = torch.tensor([0.5, 2.0], device=dev)
    cp = torch.zeros(M, ld, device=dev, dtype=DT[dtype])
    H.layernorm_bwd(xd, ld, dy.to(dev, DT[dtype]), ld, gamma.to(dev), mean, rstd, dx, ld, True, dg, db, False, ws, M, C, win,
                    copy=H.copy_desc(cp, rowscale=sc, rows_per_scale=256, win=cwin))
    torch.cuda.synchronize()
    assert rel_err(dx[:, :C] - 1, xr.grad) < TOL[dtype][0]
    want = dx.cpu() * sc.cpu().repeat_interleave(256)[:, None]
    if cwin:
        want = want[win_perm(2, 16, 16, 8, 4)]
    assert rel_err(cp[:, :C].float(), want[:, :C]) < TOL[dtype][0] / 4
    assert rel_err(dg, gm.grad) < TOL[dtype][0]
    assert rel_err(db, bt.grad) < TOL[dtype][0]


def _attn_ref(q, k, v, table, nh, shift, Hh, Ww, scale):
    """q,k,v [nWin, nh, 64, hd] fp32 -> O [nWin, 64, nh, hd] and grads helper"""
    idx = relative_position_index(8)
    bias = table[idx.view(-1)].view(64, 64, nh).permute(2, 0, 1)
    s = (q * scale) @ k.transpose(-2, -1) + bias
    if shift:
        mask = shift_region_mask(Hh, Ww, 8, shift)
        nW = mask.shape[0]
        s = (s.view(-1, nW, nh, 64, 64) + mask[None, :, None]).view(-1, nh, 64, 64)
    return torch.softmax(s, -1) @ v


@pytest.mark.parametrize("dtype", [H.F32, H.BF16])
@pytest.mark.parametrize("shift", [0, 4])
def test_window_attention_fwd_bwd(dtype, shift):
    B, Hh, Ww, nh, hd = 2, 16, 24, 6, 30
    nWin = B * (Hh // 8) * (Ww // 8)
    scale = hd ** -0.5
    g = torch.Generator().manual_seed(19)
    q = torch.randn(nWin, nh, 64, hd, generator=g)
    k = torch.randn(nWin, nh, 64, hd, generator=g)
    v = torch.randn(nWin, nh, 64, hd, generator=g)
    table = torch.randn(225, nh, generator=g) * 0.5
    if dtype == H.BF16:  # compare on the bf16-rounded inputs
        q, k, v = (t.bfloat16().float() for t in (q, k, v))
    qr, kr, vr, tr = (t.clone().requires_grad_(True) for t in (q, k, v, table))
    o = _attn_ref(qr, kr, vr, tr, nh, shift, Hh, Ww, scale)
    go = torch.randn(o.shape, generator=g)
    if dtype == H.BF16:
        go = go.bfloat16().float()
    o.backward(go)
    # pack into the head-blocked padded layout [3][nWin][nh][64][32]
    qkv = torch.zeros(3, nWin, nh, 64, 32)
    qkv[0, ..., :hd], qkv[1, ..., :hd], qkv[2, ..., :hd] = q, k, v
    qkv_d = qkv.to(dev, DT[dtype]).contiguous()
    O = torch.empty(nWin * 64, nh * 32, device=dev, dtype=DT[dtype])
    lse = torch.empty(nWin, nh, 64, device=dev)
    H.window_attn_fwd(qkv_d, table.to(dev), O, nh * 32, lse, nWin, nh, hd, scale, Hh, Ww, shift)
    torch.cuda.synchronize()
    got = O.float().cpu().view(nWin, 64, nh, 32)[..., :hd].permute(0, 2, 1, 3)
    tol = 2e-5 if dtype == H.F32 else 1.5e-2
    assert rel_err(got, o.detach()) < tol
    assert O.float().cpu().view(nWin, 64, nh, 32)[..., hd:].abs().max() == 0
    dO = torch.zeros(nWin, 64, nh, 32)
    dO[..., :hd] = go.permute(0, 2, 1, 3)
    dqkv = torch.empty_like(qkv_d)
    dtab = torch.empty(225, nh, device=dev)
    ws = torch.empty(H.window_attn_bwd_ws(nWin, nh), device=dev)
    H.window_attn_bwd(qkv_d, O, nh * 32, dO.view(nWin * 64, nh * 32).to(dev, DT[dtype]), nh * 32, table.to(dev), lse,
                      dqkv, dtab, False, ws, nWin, nh, hd, scale, Hh, Ww, shift)
    torch.cuda.synchronize()
    d = dqkv.float().cpu()
    tolb = 5e-5 if dtype == H.F32 else 3e-2
    assert rel_err(d[0, ..., :hd], qr.grad) < tolb
    assert rel_err(d[1, ..., :hd], kr.grad) < tolb
    assert rel_err(d[2, ..., :hd], vr.grad) < tolb
    assert rel_err(dtab, tr.grad) < tolb
    if dtype == H.BF16:   # token-row dqkv layout [nWin*64][3*nh*32] (kair_window_attn_bwd_ex): the same bits
        dr = torch.empty(nWin * 64, 3 * nh * 32, device=dev, dtype=torch.bfloat16)
        H.window_attn_bwd(qkv_d, O, nh * 32, dO.view(nWin * 64, nh * 32).to(dev, DT[dtype]), nh * 32, table.to(dev),
                          lse, dr, dtab, False, ws, nWin, nh, hd, scale, Hh, Ww, shift, dqkv_rows=True)
        torch.cuda.synchronize()
        blocked = dqkv.cpu().permute(1, 3, 0, 2, 4).reshape(nWin * 64, 3 * nh * 32)   # [win][tok][part][h][d]
        assert torch.equal(dr.cpu(), blocked)


@pytest.mark.parametrize("hd", [10, 15, 16])
@pytest.mark.parametrize("shift", [0, 4])
def test_window_attention_head_pad16(hd, shift):
    """bf16, head pad 16 (kair_window_attn_fwd_ex / _bwd_ex head_pad=16; SwinIR-lightweight's head dim 10,
    network_swinir.py:85): against the fp32 autograd reference at the bf16 bars of the pad-32 test, and bit-equal
    to the pad-32 kernels on the same values (the pad-32 tiles' columns 16..31 are zeros, so both contract the
    same products in the same order).  The ones column (proj bias gradient) lands in the pad."""
    B, Hh, Ww, nh = 2, 16, 24, 6
    nWin = B * (Hh // 8) * (Ww // 8)
    scale = hd ** -0.5
    g = torch.Generator().manual_seed(23)
    q, k, v = (torch.randn(nWin, nh, 64, hd, generator=g).bfloat16().float() for _ in range(3))
    table = torch.randn(225, nh, generator=g) * 0.5
    qr, kr, vr, tr = (t.clone().requires_grad_(True) for t in (q, k, v, table))
    o = _attn_ref(qr, kr, vr, tr, nh, shift, Hh, Ww, scale)
    go = torch.randn(o.shape, generator=g).bfloat16().float()
    o.backward(go)
    ones = hd if hd < 16 else -1
    res = {}
    for hp in (16, 32):
        qkv = torch.zeros(3, nWin, nh, 64, hp)
        qkv[0, ..., :hd], qkv[1, ..., :hd], qkv[2, ..., :hd] = q, k, v
        qkv_d = qkv.to(dev, torch.bfloat16).contiguous()
        O = torch.full((nWin * 64, nh * hp), float("nan"), device=dev, dtype=torch.bfloat16)
        lse = torch.empty(nWin, nh, 64, device=dev)
        H.window_attn_fwd(qkv_d, table.to(dev), O, nh * hp, lse, nWin, nh, hd, scale, Hh, Ww, shift, ones_col=ones,
                          head_pad=hp)
        dO = torch.zeros(nWin, 64, nh, hp)
        dO[..., :hd] = go.permute(0, 2, 1, 3)
        dO_d = dO.view(nWin * 64, nh * hp).to(dev, torch.bfloat16)
        dqkv = torch.full_like(qkv_d, float("nan"))
        dr = torch.full((nWin * 64, 3 * nh * hp), float("nan"), device=dev, dtype=torch.bfloat16)
        dtab = torch.empty(225, nh, device=dev)
        ws = torch.empty(H.window_attn_bwd_ws(nWin, nh), device=dev)
        H.window_attn_bwd(qkv_d, O, nh * hp, dO_d, nh * hp, table.to(dev), lse, dqkv, dtab, False, ws, nWin, nh, hd,
                          scale, Hh, Ww, shift, head_pad=hp)
        dtab1 = dtab.clone()
        H.window_attn_bwd(qkv_d, O, nh * hp, dO_d, nh * hp, table.to(dev), lse, dr, dtab, False, ws, nWin, nh, hd,
                          scale, Hh, Ww, shift, dqkv_rows=True, head_pad=hp)
        torch.cuda.synchronize()
        Ov = O.cpu().view(nWin, 64, nh, hp)
        res[hp] = (Ov[..., :hd], lse.cpu(), dqkv.cpu()[..., :hd], dtab1.cpu(),
                   dr.cpu().view(nWin, 64, 3, nh, hp)[..., :hd])
        if hp == 16:
            got = Ov[..., :hd].float().permute(0, 2, 1, 3)
            assert rel_err(got, o.detach()) < 1.5e-2
            if ones >= 0:   # pad columns: the ones column of head 0, zeros elsewhere
                pad = Ov[..., hd:].float()
                assert pad[:, :, 0, 0].eq(1).all() and pad[:, :, 0, 1:].eq(0).all() and pad[:, :, 1:].eq(0).all()
            d = dqkv.float().cpu()
            for i, ref in enumerate((qr.grad, kr.grad, vr.grad)):
                assert rel_err(d[i, ..., :hd], ref) < 3e-2
            assert rel_err(dtab1.cpu(), tr.grad) < 3e-2
            blocked = dqkv.cpu().permute(1, 3, 0, 2, 4)   # [win][tok][part][h][d]
            assert torch.equal(dr.cpu().view(nWin, 64, 3, nh, hp), blocked)
    for a, b in zip(res[16], res[32]):
        assert torch.equal(a, b)


def test_window_attention_head_pad_checks():
    """head_pad 16 is a bf16 layout; the head dim must fit the pad."""
    nWin, nh = 2, 2
    qkv = torch.zeros(3 * nWin * nh * 64 * 16, device=dev)
    O = torch.zeros(nWin * 64, nh * 16, device=dev)
    lse = torch.empty(nWin * nh * 64, device=dev)
    tab = torch.zeros(225, nh, device=dev)
    with pytest.raises(RuntimeError, match="head pad"):
        H.window_attn_fwd(qkv, tab, O, nh * 16, lse, nWin, nh, 10, 0.3, 8, 16, 0, head_pad=16)
    qb, Ob = qkv.bfloat16(), O.bfloat16()
    with pytest.raises(RuntimeError, match="head_dim"):
        H.window_attn_fwd(qb, tab, Ob, nh * 16, lse, nWin, nh, 20, 0.3, 8, 16, 0, head_pad=16)


@pytest.mark.parametrize("charb", [False, True])
def test_pixel_loss_bf16_rows(charb):
    """The training step's loss layout (bf16 dE rows of 16 slots, r = 1: kair_l1_loss's pixel-per-thread
    kernel): loss value, gradient (bf16 of torch's) and zero pad slots, L1 and Charbonnier."""
    g = torch.Generator().manual_seed(29)
    B, C, Hh, Ww = 3, 3, 40, 24
    E = torch.rand(B, C, Hh, Ww, generator=g)
    Ht = torch.rand(B, C, Hh, Ww, generator=g)
    Ht[:, :, :4] = E[:, :, :4]   # exact zeros of d
    Er = E.clone().requires_grad_(True)
    d = Er - Ht
    eps = 1e-3
    ref = (torch.sqrt(d * d + eps) if charb else d.abs()).mean()
    ref.backward()
    out = torch.empty(1, device=dev)
    dE = torch.full((B * Hh * Ww, 16), float("nan"), device=dev, dtype=torch.bfloat16)
    ws = torch.empty(1024, device=dev)
    H.l1_loss(E.to(dev), Ht.to(dev), out, dE, 16, 1.0, B, C, Hh, Ww, ws, **({"charb_eps": eps} if charb else {}))
    torch.cuda.synchronize()
    assert abs(out.item() - ref.item()) < 1e-5 * ref.item()
    got = dE.float().cpu().view(B, Hh, Ww, 16)
    gg = got[..., :C].permute(0, 3, 1, 2)
    if charb:   # bf16 of a differently-ordered fp32 expression: within one bf16 ulp
        assert (gg - Er.grad).abs().max().item() <= 2 ** -8 * Er.grad.abs().max().item()
    else:       # +-1 / numel or 0: exact
        assert torch.equal(gg, Er.grad.bfloat16().float())
    assert (got[..., C:] == 0).all()


def test_l1_and_adam():
    g = torch.Generator().manual_seed(23)
    E = torch.rand(2, 3, 8, 8, generator=g)
    Hh = torch.rand(2, 3, 8, 8, generator=g)
    Er = E.clone().requires_grad_(True)
    loss = torch.nn.functional.l1_loss(Er, Hh)
    loss.backward()
    out = torch.empty(1, device=dev)
    dE = torch.empty(2 * 64, 16, device=dev)
    ws = torch.empty(1024, device=dev)
    H.l1_loss(E.to(dev), Hh.to(dev), out, dE, 16, 1.0, 2, 3, 8, 8, ws)
    torch.cuda.synchronize()
    assert abs(out.item() - loss.item()) < 1e-6
    assert rel_err(dE.cpu().view(2, 8, 8, 16)[..., :3].permute(0, 3, 1, 2), Er.grad) < 1e-6
    # Adam + EMA against torch.optim.Adam (single tensor) for 3 steps
    p = torch.randn(1000, generator=g)
    pt = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=2e-4, betas=(0.9, 0.999), foreach=False)
    ema_ref = p.clone()
    pd, md, vd = p.to(dev), torch.zeros(1000, device=dev), torch.zeros(1000, device=dev)
    ed = p.to(dev)
    for t in range(1, 4):
        grad = torch.randn(1000, generator=g)
        pt.grad = grad.clone()
        opt.step()
        with torch.no_grad():
            ema_ref.mul_(0.999).add_(pt, alpha=0.001)
        lr_t = torch.tensor([2e-4 / (1 - 0.9 ** t), math.sqrt(1 - 0.999 ** t)], device=dev)
        H.adam_ema(pd, grad.to(dev), md, vd, ed, 1000, lr_t, 0.9, 0.999, 1e-8, 0.0, 0.999)
    torch.cuda.synchronize()
    assert rel_err(pd, pt.detach()) < 1e-6
    assert rel_err(ed, ema_ref) < 1e-6


@pytest.mark.parametrize("a_dtype", [H.F32, H.BF16])
def test_gemm_stream_epilogues(a_dtype):
    """bf16 compute, N > 64: the streaming kernel — fp32/bf16 A, gelu' gate, DropPath rowscale +
    residual (rows_per_scale), and the head-blocked q/k/v output layout."""
    B, Hh, Ww, nh = 2, 16, 16, 6
    M, C, Np = B * Hh * Ww, 192, 576
    g = torch.Generator().manual_seed(11)
    x = torch.randn(M, C, generator=g)
    w = torch.randn(384, C, generator=g) * 0.1
    gate = torch.randn(M, 384, generator=g)
    res = torch.randn(M, 384, generator=g)
    scale = torch.tensor([0.5, 2.0])
    out = torch.empty(M, 384, device=dev)
    A = x.to(dev, DT[a_dtype])
    H.gemm_nt(H.rows(A), H.rows(w.to(dev, torch.bfloat16)),
              H.epilogue(out, resid=res.to(dev), rowscale=scale.to(dev), rows_per_scale=Hh * Ww,
                         gate=gate.to(dev, torch.bfloat16), gate_kind=1), M, 384, C, H.BF16)
    xa = A.float().cpu().double()
    y = xa @ w.to(torch.bfloat16).double().T
    gb = gate.to(torch.bfloat16).double()
    cdf = 0.5 * (1 + torch.erf(gb / 2 ** 0.5))
    y = y * (cdf + gb * torch.exp(-0.5 * gb * gb) / (2 * torch.pi) ** 0.5)
    s = scale.double().repeat_interleave(Hh * Ww)[:, None]
    ref = res.double() + s * y
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 1e-2
    # q/k/v head-blocked output [3][M/64][nh][64][32] from a window-mapped A
    wq = torch.randn(Np, C, generator=g) * 0.1
    bq = torch.randn(Np, generator=g)
    qkv = torch.empty(3 * M * nh * 32, device=dev, dtype=torch.bfloat16)
    win = (Hh, Ww, 8, 4)
    H.gemm_nt(H.rows(A, win=win), H.rows(wq.to(dev, torch.bfloat16)),
              H.epilogue(qkv, mode=H.OUT_QKVBLK, ldo=0, bias=bq.to(dev), qkv=(nh, 32, 64)), M, Np, C, H.BF16)
    perm = win_perm(B, Hh, Ww, 8, 4)
    yq = xa[perm] @ wq.to(torch.bfloat16).double().T + bq.double()      # [M(window order), 576]
    refq = yq.view(M // 64, 64, 3, nh, 32).permute(2, 0, 3, 1, 4).reshape(-1)
    torch.cuda.synchronize()
    assert rel_err(qkv.float(), refq) < 1e-2


@pytest.mark.parametrize("N,K,epi", [(64, 128, "resid"), (64, 64, "plain"), (128, 64, "gate"), (128, 64, "gelu"),
                                     (96, 64, "resid"), (64, 256, "plain"), (64, 96, "resid"), (128, 96, "gelu"),
                                     (96, 40, "plain"), (192, 168, "plain")])
def test_gemm_ring_narrow_n(N, K, epi):
    """bf16 NT GEMMs on the LDS-DMA ring kernel, N <= 128 in ONE N tile (gemm.hip ring_bn_of: 64 / 96 / 128 wide) and
    K % 64 != 0 (a partial last chunk: zero-line pieces past K, a zero B slice there): the SwinIR-lightweight block
    shapes (Cp = 64, Hdp = 128, 6 heads x 16 = 96) -- residual + DropPath row scale, GELU with its derivative stored
    and a ones column, the GELU' gate -- at M >= one 128-row tile per CU, ragged last tile.  A is allocated with
    exactly K columns, so a piece read past K on the last row would leave the buffer."""
    B, Hh, Ww = 3, 104, 128
    M = B * Hh * Ww   # 39,936 rows: 312 full 128-row tiles, and a ragged 39,899
    for m in (M, M - 37):
        g = torch.Generator().manual_seed(N + K + m)
        a = torch.randn(m, K, generator=g).bfloat16()
        w = (torch.randn(N, K, generator=g) * 0.1).bfloat16()
        bias = torch.randn(N, generator=g)
        y = a.double() @ w.double().T + bias.double()
        out = torch.full((m, N), float("nan"), device=dev)
        kw = {}
        if epi == "resid":
            res = torch.randn(m, N, generator=g)
            scale = torch.tensor([0.5, 2.0, 1.25])
            rps = (m + 2) // 3
            kw = dict(resid=res.to(dev), rowscale=scale.to(dev), rows_per_scale=rps)
            ref = res.double() + scale.double().repeat_interleave(rps)[:m, None] * y
        elif epi == "gate":
            gate = torch.randn(m, N, generator=g).bfloat16()
            kw = dict(gate=gate.to(dev), gate_kind=4)
            ref = y * gate.double()
        elif epi == "gelu":
            pre = torch.empty(m, N, device=dev, dtype=torch.bfloat16)
            kw = dict(act=H.ACT_GELU, pre=pre, pre_grad=True, ones_col=N - 3)
            ref = torch.nn.functional.gelu(y)
            ref[:, N - 3] = 1.0
        else:
            ref = y
        A_d, W_d, E_d = H.rows(a.to(dev)), H.rows(w.to(dev)), H.epilogue(out, bias=bias.to(dev), **kw)
        torch.cuda.synchronize()
        H.ktime_begin(8)
        try:
            H.gemm_nt(A_d, W_d, E_d, m, N, K, H.BF16)
        finally:
            n = H.ktime_end()
        torch.cuda.synchronize()
        assert n == 1 and "gemm_nt_ring" in H.ktime_read(0)[1], H.ktime_read(0)[1]
        assert torch.isfinite(out).all()
        assert rel_err(out, ref) < (5e-3 if epi == "gelu" else 1e-5)
        if epi == "gelu":   # GELU'(y), bf16
            t = y.clone()
            t.requires_grad_(True)
            torch.nn.functional.gelu(t).sum().backward()
            dref = t.grad
            dref[:, N - 3] = pre.double().cpu()[:, N - 3]   # the ones column's pre value is not specified
            assert rel_err(pre, dref) < 1e-2


def test_gemm_qkvblk_A_operand():
    """A read from the head-blocked q/k/v layout (the q/k/v input-gradient GEMM), K = 576."""
    nWin, nh, tok, hdp = 12, 6, 64, 32
    M, N, K = nWin * tok, 192, 3 * nh * hdp
    g = torch.Generator().manual_seed(13)
    blk = torch.randn(3, nWin, nh, tok, hdp, generator=g)
    w = torch.randn(N, K, generator=g) * 0.05
    out = torch.empty(M, N, device=dev)
    H.gemm_nt(H.qkvblk(blk.to(dev, torch.bfloat16).reshape(-1), nh), H.rows(w.to(dev, torch.bfloat16)), H.epilogue(out),
              M, N, K, H.BF16)
    a = blk.to(torch.bfloat16).double().permute(1, 3, 0, 2, 4).reshape(M, K)   # row m=(win,t), col=(part,h,d)
    ref = a @ w.to(torch.bfloat16).double().T
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 1e-2


def test_gemm_qkvblk_A_ring_head_pad16():
    """The q/k/v input-gradient GEMM of the 16-wide head layout on the ring: A head-blocked [3][nWin][6][64][16],
    K = 288 (4.5 chunks of 64: a partial last chunk), N = Cp = 64, M = 600 windows x 64 tokens."""
    nWin, nh, tok, hdp = 600, 6, 64, 16
    M, N, K = nWin * tok, 64, 3 * nh * hdp
    g = torch.Generator().manual_seed(14)
    blk = torch.randn(3, nWin, nh, tok, hdp, generator=g).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.05).bfloat16()
    out = torch.full((M, N), float("nan"), device=dev)
    A_d, W_d, E_d = H.qkvblk(blk.to(dev).reshape(-1), nh, hdp=hdp), H.rows(w.to(dev)), H.epilogue(out)
    torch.cuda.synchronize()
    H.ktime_begin(8)
    try:
        H.gemm_nt(A_d, W_d, E_d, M, N, K, H.BF16)
    finally:
        n = H.ktime_end()
    torch.cuda.synchronize()
    assert n == 1 and "gemm_nt_ring" in H.ktime_read(0)[1], H.ktime_read(0)[1]
    a = blk.double().permute(1, 3, 0, 2, 4).reshape(M, K)
    assert rel_err(out, a @ w.double().T) < 1e-5


@pytest.mark.parametrize("M", [3001, 40000])
def test_wgrad_grouped_narrow_bf16(M):
    """kair_wgrad_grouped (bf16 TN ring, one launch) over a SwinIR-lightweight block's linears -- Cp = 64, Hdp = 128,
    6 heads x 16: fc2 (64 x 128), fc1 (128 x 64), proj (64 x 96, A = the token rows of O), qkv (288 x 64, A head-blocked
    [3][M/64][6][64][16]) -- with the bias ones columns in the data, against float64 on the bf16 operands."""
    g = torch.Generator().manual_seed(31)
    M = M // 64 * 64
    C, Cp, Hd, Hdp, nh, hd, hp = 60, 64, 120, 128, 6, 10, 16
    jobs, refs, keep = [], [], []
    # (Np, Kp, N, K, n_grp, k_grp, qkv-blocked A)
    for Np, Kp, N, K, ng, kg, blk in [(Cp, Hdp, C, Hd, (1, C, Cp), (1, Hd, Hdp), False),
                                      (Hdp, Cp, Hd, C, (1, Hd, Hdp), (1, C, Cp), False),
                                      (Cp, nh * hp, C, C, (1, C, Cp), (nh, hd, hp), False),
                                      (3 * nh * hp, Cp, 3 * C, C, (3 * nh, hd, hp), (1, C, Cp), True)]:
        dy = torch.zeros(M, Np)
        cols = torch.tensor([i // ng[1] * ng[2] + i % ng[1] for i in range(N)])
        dy[:, cols] = torch.randn(M, N, generator=g).bfloat16().float()
        x = torch.zeros(M, Kp)
        kcols = torch.tensor([i // kg[1] * kg[2] + i % kg[1] for i in range(K)])
        x[:, kcols] = torch.randn(M, K, generator=g).bfloat16().float()
        ones = int(kcols[-1]) + 1   # the first pad column after the last real one
        x[:, ones] = 1.0
        if blk:   # head-blocked [3][nWin][nh][64][hp] of the token-row gradient [M][3 nh hp]
            a = dy.view(M // 64, 64, 3, nh, hp).permute(2, 0, 3, 1, 4).contiguous().to(dev, torch.bfloat16).reshape(-1)
            A = H.qkvblk(a, nh, hdp=hp)
        else:
            a = dy.to(dev, torch.bfloat16)
            A = H.rows(a)
        b = x.to(dev, torch.bfloat16)
        Bop = H.rows(b, ones_col=ones, ones_in_data=True)
        m = H.wmap(0, N, K, ng, kg)
        gw, gb = torch.full((N, K), 7.0, device=dev), torch.full((N,), 7.0, device=dev)
        jobs.append((A, Bop, Np, Kp, m, gw, gb, ones))
        keep += [a, b]
        refs.append((gw, gb, dy[:, cols].double().T @ x[:, kcols].double(), dy[:, cols].double().sum(0)))
    grp = H.WgradGroup(jobs, M)
    ws = torch.empty(grp.ws_floats, device=dev)
    grp.run(ws)
    torch.cuda.synchronize()
    for gw, gb, rw, rb in refs:
        assert rel_err(gw, rw) < 1e-5 and rel_err(gb, rb) < 1e-5


@pytest.mark.parametrize("dtype", [H.F32, H.BF16])
def test_row_copy(dtype):
    M, C, ld = 512, 192, 200
    g = torch.Generator().manual_seed(19)
    src = torch.randn(M, ld, generator=g)
    sc = torch.tensor([3.0, -1.0])
    out = torch.empty(M, C, device=dev, dtype=DT[dtype])
    H.row_copy(src.to(dev), ld, M, C, H.copy_desc(out, rowscale=sc.to(dev), rows_per_scale=256, win=(16, 16, 8, 4)))
    want = (src[:, :C] * sc.repeat_interleave(256)[:, None])[win_perm(2, 16, 16, 8, 4)]
    torch.cuda.synchronize()
    assert rel_err(out.float(), want) < TOL[dtype][0] / 4


def test_gemm_tn_ring_qkvblk_A():
    """Weight gradient of the q/k/v projection: A read from the head-blocked layout (ring kernel)."""
    nWin, nh, tok, hdp = 40, 6, 64, 32
    M, N, K = nWin * tok, 3 * nh * hdp, 192
    g = torch.Generator().manual_seed(23)
    blk = torch.randn(3, nWin, nh, tok, hdp, generator=g).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    x[:, 180] = 1.0
    S = H.wgrad_splits(M, N, K)
    ws = torch.empty(S, N, K, device=dev)
    H.gemm_tn(H.qkvblk(blk.to(dev).reshape(-1), nh), H.rows(x.to(dev), ones_col=180, ones_in_data=True), ws, S, M, N, K,
              H.BF16)
    a = blk.double().permute(1, 3, 0, 2, 4).reshape(M, N)
    ref = a.T @ x.double()
    torch.cuda.synchronize()
    assert rel_err(ws.sum(0).cpu(), ref) < 1e-2


@pytest.mark.parametrize("B,Hh,Ww,Cout", [(2, 24, 24, 256), (1, 96, 96, 256), (3, 10, 12, 96)])
def test_conv_wgrad_tap3_ring(B, Hh, Ww, Cout):
    """The reconstruction tail's 64-channel conv weight gradients (network_swinir.py:597-600 Upsample,
    conv 64 -> 4*64) on the ring with three taps per 192-wide K tile (gemm.hip BM_TAP3), against
    float64 conv2d backward on the same bf16 values."""
    C = 64
    g = torch.Generator().manual_seed(19)
    x = torch.randn(B, C, Hh, Ww, generator=g).to(torch.bfloat16).double().requires_grad_(True)
    w = torch.randn(Cout, C, 3, 3, generator=g, dtype=torch.float64, requires_grad=True)
    y = torch.nn.functional.conv2d(x, w, padding=1)
    gy = torch.randn(y.shape, generator=g).to(torch.bfloat16).double()
    y.backward(gy)
    M = B * Hh * Ww
    dy = gy.permute(0, 2, 3, 1).reshape(M, Cout).to(torch.bfloat16)
    xin = x.detach().permute(0, 2, 3, 1).reshape(M, C).to(torch.bfloat16)
    K = 9 * C
    S = H.wgrad_splits(M, Cout, K)
    ws = torch.full((S, Cout, K), float("nan"), device=dev)
    H.gemm_tn(H.rows(dy.contiguous().to(dev)), H.im2col(xin.contiguous().to(dev), Hh, Ww, C), ws, S, M, Cout, K, H.BF16)
    grad = torch.empty(Cout, C, 3, 3, device=dev)
    H.wgrad_finalize(ws, S, H.wmap(1, Cout, C), grad)
    torch.cuda.synchronize()
    assert rel_err(grad, w.grad) < 1e-5
