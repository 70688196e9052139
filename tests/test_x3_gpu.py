"""The fp16-pair ("fp32x3") path: every contraction as hi.hi + hi.lo + lo.hi of hi/lo fp16 pairs of power-of-2
scaled operands (x 2^e: weights 2^12, activations 2^4, data gradients 2^(log2 numel + 4)), the fp32 reference's
arithmetic on the 16-bit matrix cores (the reference trains SwinIR classical x4 in fp32: models/model_plain.py:31-36,
options/swinir/train_swinir_sr_classical.json has no amp_enabled).

Kernels are checked against float64 torch references at the fp32 engine's tolerances (2e-5 .. 5e-5
relative); the whole classical x4 network against the CPU oracle at SURVEY.md §8d's fp32 bar (outputs < 1e-5
relative), gradients < 1e-3, PSNR < 1e-3 dB; the 3-step ModelPlain trajectory < 1e-4.  The range guard that
keeps the fixed exponents safe: tests/test_x3_range_gpu.py."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from conftest import load_golden, sub_grads, sub_state  # noqa: E402
from kair_amd import _hip as H  # noqa: E402
from kair_amd.engine.trainer import FusedTrainer  # noqa: E402
from kair_amd.models.network_swinir import SwinIR  # noqa: E402
from oracle import image as oimg  # noqa: E402
from oracle import swinir as osw  # noqa: E402
from test_kernels_gpu import _attn_ref  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def hilo(x, e=0):
    """The fp16 pair planes of x * 2^e: [2, *x.shape] (hi = f16(x 2^e), lo = f16(x 2^e - hi))."""
    w = x * 2.0 ** e
    hi = w.to(torch.float16)
    lo = (w - hi.float()).to(torch.float16)
    return torch.stack([hi, lo])


@pytest.mark.parametrize("kind,base", [(17, 0), (18, 2), (19, 3)])
def test_split_pack_kinds(kind, base):
    """Pack kinds 17 / 18 / 19: fp16 pairs of w 2^KAIR_X3_WEXP for kinds 0 / 2 / 3, interleaved per 64 columns;
    (hi + lo) 2^-KAIR_X3_WEXP reproduces the plain fp32 form to ~2^-21 relative."""
    g = torch.Generator().manual_seed(3)
    if base == 2:
        N, K = 72, 40
        w = torch.randn(N, K, 3, 3, generator=g)
        m, mb = H.wmap(kind, N, K, (1, N, 80), (1, K, 48)), H.wmap(base, N, K, (1, N, 80), (1, K, 48))
        rows, rowlen = 48, 9 * 80
    else:
        N, K = 100, 70
        w = torch.randn(N, K, generator=g)
        m, mb = H.wmap(kind, N, K, (1, N, 104), (1, K, 72)), H.wmap(base, N, K, (1, N, 104), (1, K, 72))
        rows, rowlen = (104, 72) if base == 0 else (72, 104)
    wd = w.to(dev)
    plain = torch.empty(rows, rowlen, device=dev)
    H.pack_weight(wd, plain, mb)
    KS = 2 * (-(-rowlen // 64)) * 64
    sp = torch.full((rows, KS), float("nan"), device=dev, dtype=torch.float16)
    H.pack_weight(wd, sp, m)
    torch.cuda.synchronize()
    s = sp.double().cpu().view(rows, KS // 128, 2, 64) * 2.0 ** -H.X3_WEXP
    recon = (s[:, :, 0] + s[:, :, 1]).reshape(rows, -1)[:, :rowlen]
    assert torch.isfinite(s).all()
    assert rel(recon, plain) < 1e-6
    assert (s[:, :, 0].reshape(rows, -1)[:, rowlen:] == 0).all()


@pytest.mark.parametrize("a_bf, b_bf, b_im2col", [(False, False, False), (True, True, False), (False, True, False),
                                                  (False, False, True), (True, False, True)])
@pytest.mark.parametrize("M,N,K", [(3000, 576, 192), (777, 64, 40), (2304, 192, 384)])
def test_gemm_tn_x3(a_bf, b_bf, b_im2col, M, N, K):
    """kair_gemm_tn compute KAIR_COMPUTE_X3: fp32 operands split in the kernel (with an exponent), or fp16 pair
    planes carrying one; the bias column injected (ones_col) -- against float64, tighter than the fp32 path."""
    g = torch.Generator().manual_seed(5)
    dy = torch.randn(M, N, generator=g) * 1e-6   # a gradient-sized operand, exponent 24
    if b_im2col:
        if M % 16:
            pytest.skip("im2col case needs M = 16 * W")
        Cin = 32 if K >= 288 else 8
        B_, Hh, Ww = 1, 16, M // 16
        x = torch.randn(M, Cin, generator=g)
        xi = x.view(B_, Hh, Ww, Cin).permute(0, 3, 1, 2)
        cols = torch.nn.functional.unfold(xi.double(), 3, padding=1)   # [1, Cin*9, HW], c-major taps
        cols = cols.view(Cin, 9, M).permute(2, 1, 0).reshape(M, 9 * Cin)   # k = tap*Cin + c
        K = 9 * Cin
        ref = dy.double().T @ cols
        Bsrc = x
    else:
        x = torch.randn(M, K, generator=g)
        ones = K - 3
        xr = x.clone()
        xr[:, ones] = 1.0
        ref = dy.double().T @ xr.double()
        Bsrc = x
    S = H.wgrad_splits(M, N, K)
    ws = torch.empty(S, N, K, device=dev)
    if a_bf:
        ap = hilo(dy.to(dev), 24)
        A = H.with_lo(H.rows(ap[0]), ap[1])
    else:
        A = H.rows(dy.to(dev))
    A.x3_exp = 24
    if b_bf:
        bp = hilo(Bsrc.to(dev), 4)
        Bop = H.rows(bp[0], ones_col=K - 3) if not b_im2col else H.im2col(bp[0], Hh, Ww, Bsrc.shape[1])
        Bop = H.with_lo(Bop, bp[1])
    else:
        Bop = H.rows(Bsrc.to(dev), ones_col=K - 3) if not b_im2col else H.im2col(Bsrc.to(dev), Hh, Ww, Bsrc.shape[1])
    Bop.x3_exp = 4
    H.gemm_tn(A, Bop, ws, S, M, N, K, H.X3)
    torch.cuda.synchronize()
    assert rel(ws.sum(0), ref) < 2e-6


@pytest.mark.parametrize("N,K", [(576, 192), (192, 384), (384, 192), (192, 192)])
def test_gemm_tn_x3_ring_pairs(N, K):
    """The TN ring on fp16-pair operands (the fp32x3 block weight gradients: A = the gradient pair at its exponent,
    B = the activation pair with the bias ones column in its data): transposed LDS reads, no split -- against float64
    over ragged splits (M not a multiple of the 32-row chunk)."""
    g = torch.Generator().manual_seed(15)
    M = 3001
    dy = torch.randn(M, N, generator=g) * 1e-6
    x = torch.randn(M, K, generator=g)
    x[:, K - 3] = 1.0
    ref = dy.double().T @ x.double()
    S = H.wgrad_splits(M, N, K)
    ws = torch.empty(S, N, K, device=dev)
    ap, bp = hilo(dy.to(dev), 24), hilo(x.to(dev), 4)
    A = H.with_lo(H.rows(ap[0]), ap[1])
    A.x3_exp = 24
    Bop = H.with_lo(H.rows(bp[0], ones_col=K - 3, ones_in_data=True), bp[1])
    Bop.x3_exp = 4
    H.gemm_tn(A, Bop, ws, S, M, N, K, H.X3)
    torch.cuda.synchronize()
    assert rel(ws.sum(0), ref) < 2e-6


@pytest.mark.parametrize("M, max_ctas", [(3001, 192), (9216, 192), (9216, 0)])
def test_wgrad_grouped_x3_pairs(M, max_ctas):
    """kair_wgrad_grouped on fp16-pair jobs (the fp32x3 engine's per-RSTB grouped block weight gradients: one TN-ring
    launch over a Swin block's qkv / proj / fc1 / fc2 shapes + one grouped finalize into the reference-layout
    gradients and biases) against float64, the side stream's workgroup cap and ragged row splits included."""
    g = torch.Generator().manual_seed(23)
    C, Cp, Hd, Hdp = 180, 192, 360, 384
    shapes = [(Cp, Hdp, C, Hd), (Hdp, Cp, Hd, C), (Cp, Cp, C, C), (576, Cp, 540, C)]   # (Np, Kp, N, K): fc2 fc1 proj qkv
    jobs, refs, keep = [], [], []
    for Np, Kp, N, K in shapes:
        dy = torch.zeros(M, Np)
        dy[:, :N] = torch.randn(M, N, generator=g) * 1e-5
        x = torch.zeros(M, Kp)
        x[:, :K] = torch.randn(M, K, generator=g)
        x[:, K] = 1.0   # the bias ones column, in the data
        ap, bp = hilo(dy.to(dev), 20), hilo(x.to(dev), 4)
        A = H.with_lo(H.rows(ap[0]), ap[1])
        A.x3_exp = 20
        Bop = H.with_lo(H.rows(bp[0], ones_col=K, ones_in_data=True), bp[1])
        Bop.x3_exp = 4
        m = H.wmap(0, N, K, (1, N, Np), (1, K, Kp))
        gw, gb = torch.full((N, K), 7.0, device=dev), torch.full((N,), 7.0, device=dev)
        jobs.append((A, Bop, Np, Kp, m, gw, gb, K))
        keep += [ap, bp]
        refs.append((gw, gb, dy[:, :N].double().T @ x[:, :K].double(), dy[:, :N].double().sum(0)))
    grp = H.WgradGroup(jobs, M)
    ws = torch.empty(grp.ws_floats, device=dev)
    grp.run(ws, max_ctas=max_ctas)
    torch.cuda.synchronize()
    for gw, gb, rw, rb in refs:
        assert rel(gw, rw) < 2e-6 and rel(gb, rb) < 2e-6


def test_layernorm_x3_pair_forms():
    """kair_layernorm_fwd_x3 (window-ordered fp16-pair output with the ones column at 2^e), and the pair forms of
    the GEMM-operand copies (kair_copy_desc dtype F16: kair_layernorm_bwd's copy, kair_row_copy) -- (hi + lo) 2^-e
    against float64 to ~2^-21."""
    g = torch.Generator().manual_seed(19)
    Bn, Hh, Ww, C, Cp = 2, 16, 16, 180, 192
    M = Bn * Hh * Ww
    x = torch.zeros(M, Cp)
    x[:, :C] = torch.randn(M, C, generator=g) * 3 + 0.5
    gam, bet = 1 + 0.1 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    y = torch.empty(2, M, Cp, device=dev, dtype=torch.float16)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    win = (Hh, Ww, 8, 4)
    H.layernorm_fwd_x3(x.to(dev), Cp, y, Cp, gam.to(dev), bet.to(dev), mean, rstd, M, C, 1e-5, win, one_col=C, x3_exp=4)
    xd = x[:, :C].double()
    ref = (xd - xd.mean(1, keepdim=True)) / torch.sqrt(xd.var(1, unbiased=False, keepdim=True) + 1e-5) * gam.double() + bet.double()
    # window order: output row r holds token win_to_token(r): compare through the fp32 kernel's own map
    y32 = torch.empty(M, Cp, device=dev)
    H.layernorm_fwd(x.to(dev), Cp, y32, Cp, gam.to(dev), bet.to(dev), mean, rstd, M, C, 1e-5, win, one_col=C)
    torch.cuda.synchronize()
    rec = (y[0].double() + y[1].double()).cpu() / 16
    assert rel(rec, y32) < 1e-6 and (rec[:, C] == 1).all() and (rec[:, C + 1:] == 0).all()
    tok = torch.sort(y32[:, 0].double().cpu())[0]
    assert rel(tok, torch.sort(ref[:, 0])[0]) < 1e-6
    # pair copies: row_copy (row scale per image) and the LayerNorm backward's operand copy, gradient-sized values
    src = torch.randn(M, Cp, generator=g) * 1e-5
    sc = torch.tensor([0.5, 2.0])
    cp = torch.zeros(2, M, Cp, device=dev, dtype=torch.float16)
    H.row_copy(src.to(dev), Cp, M, Cp, H.copy_desc(cp, rowscale=sc.to(dev), rows_per_scale=Hh * Ww, x3_exp=20))
    torch.cuda.synchronize()
    want = src.double() * sc.double().repeat_interleave(Hh * Ww)[:, None]
    assert rel((cp[0].double() + cp[1].double()).cpu() * 2.0 ** -20, want) < 1e-6
    dy = torch.randn(M, Cp, generator=g) * 1e-5
    dx = torch.zeros(M, Cp, device=dev)
    ws = torch.empty(2 * 2048 * Cp, device=dev)
    cp2 = torch.zeros(2, M, Cp, device=dev, dtype=torch.float16)
    cp32 = torch.zeros(M, Cp, device=dev)
    for out, e in ((cp2, 20), (cp32, 0)):
        dx.zero_()
        H.layernorm_bwd(x.to(dev), Cp, dy.to(dev), Cp, gam.to(dev), mean, rstd, dx, Cp, False, None, None, False, ws, M, C,
                        win, copy=H.copy_desc(out, rowscale=sc.to(dev), rows_per_scale=Hh * Ww, win=win, x3_exp=e))
    torch.cuda.synchronize()
    assert rel((cp2[0].double() + cp2[1].double()).cpu() * 2.0 ** -20, cp32) < 1e-6


def test_gemm_nt_x3_rows_and_qkvblk():
    """kair_gemm_nt as the fp32x3 engine calls it (compute KAIR_COMPUTE_X3): fp32 A and an fp16 pair A, split-packed
    fp16 weights (kind 17), ROWS fp32 and head-blocked q/k/v fp16-pair outputs (with an output exponent)."""
    g = torch.Generator().manual_seed(7)
    M, N, K, C = 4 * 64, 3 * 6 * 32, 192, 180
    x = torch.zeros(M, K)
    x[:, :C] = torch.randn(M, C, generator=g)
    w = torch.randn(3 * 180, C, generator=g) * 0.05
    b = torch.randn(3 * 180, generator=g) * 0.1
    grp_n, grp_k = (18, 30, 32), (1, C, K)
    Wp = torch.empty(N, 2 * 192, device=dev, dtype=torch.float16)
    H.pack_weight(w.to(dev), Wp, H.wmap(17, 540, C, grp_n, grp_k))
    bp = torch.empty(N, device=dev)
    H.pack_weight(b.to(dev), bp, H.wmap(4, 540, 0, grp_n, (1, 1, 1)))
    ref = x[:, :C].double() @ w.double().T + b.double()   # [M][540], column (part, h, d)
    refp = torch.zeros(M, 18, 32, dtype=torch.float64)
    refp[..., :30] = ref.view(M, 18, 30)
    def wop():
        o = H.rows(Wp)
        o.x3_exp = H.X3_WEXP
        return o
    for a_mode in ("f32", "pair"):
        def aop():
            if a_mode == "f32":
                o = H.rows(x.to(dev))
            else:
                xp = hilo(x.to(dev), 4)
                o = H.with_lo(H.rows(xp[0]), xp[1])
            o.x3_exp = 4
            return o
        out = torch.empty(M, N, device=dev)
        H.gemm_nt(aop(), wop(), H.epilogue(out, bias=bp), M, N, K, H.X3)
        qkv = torch.empty(2, 3 * M * 6 * 32, device=dev, dtype=torch.float16)
        E = H.epilogue(qkv[0], mode=H.OUT_QKVBLK, ldo=0, bias=bp, qkv=(6, 32, 64), out_lo=qkv[1])
        E.x3_out_exp = 2
        H.gemm_nt(aop(), wop(), E, M, N, K, H.X3)
        torch.cuda.synchronize()
        assert rel(out.view(M, 18, 32), refp) < 2e-6
        blk = (qkv[0].double() + qkv[1].double()).cpu().view(3, M // 64, 6, 64, 32).permute(1, 3, 0, 2, 4).reshape(M, 18, 32)
        assert rel(blk / 4, refp) < 2e-6


def _wsplit(w):
    """kind-17 split pack of a [N][K] weight (fp16 pairs of w 2^KAIR_X3_WEXP) and its operand."""
    N, K = w.shape
    Wp = torch.empty(N, 2 * (-(-K // 64)) * 64, device=dev, dtype=torch.float16)
    H.pack_weight(w.to(dev), Wp, H.wmap(17, N, K))
    o = H.rows(Wp)
    o.x3_exp = H.X3_WEXP
    return o, Wp


@pytest.mark.parametrize("M, win, with_copy", [(1000, False, True), (3 * 16 * 16, True, True), (2 * 24 * 24, True, False)])
def test_gemm_nt_x3_lnbwd_fused(M, win, with_copy):
    """kair_gemm_nt_x3_lnbwd (the q/k/v or fc1 input-gradient GEMM fused with the LayerNorm backward in front of it)
    against float64: D += LN'(A W^T) over token rows (GEMM rows in window order when win), the fp16-pair operand copy
    of D (row-scaled, window order), and the dgamma / dbeta partial rows reduced by ln_param_reduce_grouped; ragged M,
    padded channels (C = 180 of 192)."""
    g = torch.Generator().manual_seed(37)
    C, Cp, K = 180, 192, 384
    geo = (16, 16, 8, 4) if M == 768 else ((24, 24, 8, 0) if win else (0, 0, 0, 0))
    HW = geo[0] * geo[1] if win else M
    dy = torch.randn(M, K, generator=g) * 1e-5
    w = torch.zeros(Cp, K)
    w[:C] = torch.randn(C, K, generator=g) * 0.05
    x = torch.zeros(M, Cp)
    x[:, :C] = torch.randn(M, C, generator=g) * 2 + 0.3
    gam = 1 + 0.1 * torch.randn(C, generator=g)
    D0 = torch.zeros(M, Cp)
    D0[:, :C] = torch.randn(M, C, generator=g) * 1e-5
    mu = x[:, :C].double().mean(1)
    rs = 1 / torch.sqrt(x[:, :C].double().var(1, unbiased=False) + 1e-5)
    Wo, keep = _wsplit(w)
    dp = hilo(dy.to(dev), 20)
    A = H.with_lo(H.rows(dp[0]), dp[1])   # GEMM rows = dy rows (window order when win)
    A.x3_exp = 20
    D = D0.to(dev)
    nb = H.gemm_nt_lnbwd_parts(M, Cp)
    part = torch.full((nb * 2 * C,), float("nan"), device=dev)
    nimg = -(-M // HW)
    sc = torch.rand(nimg, generator=g) + 0.5
    cp = torch.zeros(2, M, Cp, device=dev, dtype=torch.float16)
    desc = H.copy_desc(cp, rowscale=sc.to(dev), rows_per_scale=HW, win=geo if win else None, x3_exp=20) if with_copy else None
    H.gemm_nt_lnbwd(A, Wo, M, Cp, K, x.to(dev), Cp, gam.to(dev), mu.float().to(dev), rs.float().to(dev), C, D, Cp, part,
                    win=geo if win else (0, 0, 0, 0), copy=desc)
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    H.ln_param_reduce_grouped([(part, M, C, dg, db, False, nb)])
    torch.cuda.synchronize()
    # float64 reference, token order: GEMM row r is token win_to_token(r)
    dxn_r = dy.double() @ w.double().T                       # [M][Cp] in GEMM-row order
    if win:
        ref32 = torch.empty(M, Cp, device=dev)
        tok = torch.empty(M, 8, device=dev)
        H.row_copy(torch.arange(M, dtype=torch.float32, device=dev)[:, None].repeat(1, 8).contiguous(), 8, M, 8,
                   H.copy_desc(tok, win=geo))   # tok[token_to_win(t)] = t
        perm = tok[:, 0].long().cpu()                      # GEMM row r holds token perm[r]
        dxn = torch.empty_like(dxn_r)
        dxn[perm] = dxn_r
    else:
        perm = torch.arange(M)
        dxn = dxn_r
    xh = (x[:, :C].double() - mu[:, None]) * rs[:, None]
    gy = dxn[:, :C] * gam.double()
    dx = rs[:, None] * (gy - gy.mean(1, keepdim=True) - xh * (gy * xh).mean(1, keepdim=True))
    Dref = D0.double().clone()
    Dref[:, :C] += dx
    assert rel(D[:, :C], Dref[:, :C]) < 1e-6 and (D[:, C:] == 0).all()
    assert rel(dg, (dxn[:, :C] * xh).sum(0)) < 1e-5 and rel(db, dxn[:, :C].sum(0)) < 1e-5
    if with_copy:
        want = Dref * sc.double().repeat_interleave(HW)[:M, None]
        got = (cp[0].double() + cp[1].double()).cpu() * 2.0 ** -20
        if win:
            got_tok = torch.empty_like(got)
            got_tok[perm] = got   # copy row r (window order) holds token perm[r]
            got = got_tok
        assert rel(got[:, :C], want[:, :C]) < 1e-6


@pytest.mark.parametrize("C", [64, 256])
def test_gemm_nt_x3_im2col_generic(C):
    """The generic x3 NT kernel on a flipped 3x3 im2col of a C-channel map (the upsampling convs' input gradients)
    against float64 over ragged tiles (N = 48 of a 64-column tile, M not a multiple of 128)."""
    g = torch.Generator().manual_seed(41)
    Bn, Hh, Ww, N = 2, 10, 18, 48
    M, K = Bn * Hh * Ww, 9 * C
    x, w = torch.randn(M, C, generator=g), torch.randn(N, K, generator=g) * 0.05
    Wo, keep = _wsplit(w)
    A = H.im2col(x.to(dev), Hh, Ww, C, flip=True)
    A.x3_exp = 4
    out = torch.empty(M, N, device=dev)
    H.gemm_nt(A, Wo, H.epilogue(out), M, N, K, H.X3)
    cols = torch.nn.functional.unfold(x.view(Bn, Hh, Ww, C).permute(0, 3, 1, 2).double(), 3, padding=1)
    cols = cols.view(Bn, C, 9, Hh * Ww).permute(0, 3, 2, 1).reshape(M, 9, C).flip(1).reshape(M, K)
    torch.cuda.synchronize()
    assert rel(out, cols @ w.double().T) < 2e-6


def test_gemm_nt_x3_ring_epilogues():
    """The persistent LDS-DMA ring form of kair_gemm_nt x3 (N % 192 == 0, K % 32 == 0): ragged M with a GELU +
    GELU' epilogue, window-ordered rows of an fp16 pair A with a DropPath-scaled residual, and a flipped 3x3
    im2col of an fp32 map with a multiplicative gate -- each against float64."""
    g = torch.Generator().manual_seed(11)
    # (a) fp32 rows, M not a multiple of the 128-row tile, 7 k-chunks, two N-tiles
    M, N, K = 1000, 384, 224
    x, w, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05, torch.randn(N, generator=g) * 0.1
    Wo, keep = _wsplit(w)
    A = H.rows(x.to(dev))
    A.x3_exp = 4
    out, pre = torch.empty(M, N, device=dev), torch.empty(M, N, device=dev)
    H.gemm_nt(A, Wo, H.epilogue(out, bias=b.to(dev), act=H.ACT_GELU, pre=pre, pre_grad=True), M, N, K, H.X3)
    h = x.double() @ w.double().T + b.double()
    cdf = 0.5 * (1 + torch.erf(h / 2 ** 0.5))
    torch.cuda.synchronize()
    assert rel(out, h * cdf) < 2e-6
    assert rel(pre, cdf + h * torch.exp(-h * h / 2) / (2 * torch.pi) ** 0.5) < 2e-6
    # (b) fp16 pair rows read and written through the Swin window map (shift 4), residual + per-image scale
    Bn, Hh, Ww, N, K = 3, 16, 16, 192, 192
    M = Bn * Hh * Ww
    x, w = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05
    r, s = torch.randn(M, N, generator=g), torch.tensor([0.5, 1.25, 2.0])
    Wo, keep = _wsplit(w)
    xp = hilo(x.to(dev), 4)
    A = H.with_lo(H.rows(xp[0], win=(Hh, Ww, 8, 4)), xp[1])
    A.x3_exp = 4
    out = torch.empty(M, N, device=dev)
    H.gemm_nt(A, Wo, H.epilogue(out, win=(Hh, Ww, 8, 4), resid=r.to(dev), rowscale=s.to(dev), rows_per_scale=Hh * Ww),
              M, N, K, H.X3)
    ref = r.double() + s.double().repeat_interleave(Hh * Ww)[:, None] * (x.double() @ w.double().T)
    torch.cuda.synchronize()
    assert rel(out, ref) < 2e-6
    # (c) flipped 3x3 im2col of a 64-channel fp32 map (the conv input gradient), gated
    Bn, Hh, Ww, C, N = 2, 12, 20, 64, 192
    M, K = Bn * Hh * Ww, 9 * C
    x, w, gt = torch.randn(M, C, generator=g), torch.randn(N, K, generator=g) * 0.05, torch.randn(M, N, generator=g)
    Wo, keep = _wsplit(w)
    A = H.im2col(x.to(dev), Hh, Ww, C, flip=True)
    A.x3_exp = 4
    out = torch.empty(M, N, device=dev)
    H.gemm_nt(A, Wo, H.epilogue(out, gate=gt.to(dev), gate_kind=4), M, N, K, H.X3)
    cols = torch.nn.functional.unfold(x.view(Bn, Hh, Ww, C).permute(0, 3, 1, 2).double(), 3, padding=1)
    cols = cols.view(Bn, C, 9, Hh * Ww).permute(0, 3, 2, 1).reshape(M, 9, C).flip(1).reshape(M, K)
    torch.cuda.synchronize()
    assert rel(out, (cols @ w.double().T) * gt.double()) < 2e-6
    # (d) fp16-pair rows out with GELU and its fp32 GELU' (the fc1 forward of the pair engine), ones column at 2^e
    M, N, K = 1000, 384, 192
    x, w, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05, torch.randn(N, generator=g) * 0.1
    Wo, keep = _wsplit(w)
    xp = hilo(x.to(dev), 4)
    A = H.with_lo(H.rows(xp[0]), xp[1])
    A.x3_exp = 4
    hp, pre = torch.empty(2, M, N, device=dev, dtype=torch.float16), torch.empty(M, N, device=dev)
    E = H.epilogue(hp[0], out_lo=hp[1], bias=b.to(dev), act=H.ACT_GELU, pre=pre, pre_grad=True, ones_col=N - 20)
    E.x3_out_exp = 4
    H.gemm_nt(A, Wo, E, M, N, K, H.X3)
    h = x.double() @ w.double().T + b.double()
    cdf = 0.5 * (1 + torch.erf(h / 2 ** 0.5))
    want = h * cdf
    want[:, N - 20] = 1.0
    torch.cuda.synchronize()
    assert rel((hp[0].double() + hp[1].double()).cpu() / 16, want) < 2e-6
    pw = cdf + h * torch.exp(-h * h / 2) / (2 * torch.pi) ** 0.5
    keepc = [c for c in range(N) if c != N - 20]
    assert rel(pre[:, keepc], pw[:, keepc]) < 2e-6
    # (e) fp16-pair A (a gradient pair) -> fp16-pair rows out through the fp32 multiply gate (the fc2 input gradient)
    M, N, K = 777, 384, 192
    dy, w, gt = torch.randn(M, K, generator=g) * 1e-5, torch.randn(N, K, generator=g) * 0.05, torch.rand(M, N, generator=g)
    Wo, keep = _wsplit(w)
    dp = hilo(dy.to(dev), 20)
    A = H.with_lo(H.rows(dp[0]), dp[1])
    A.x3_exp = 20
    up = torch.empty(2, M, N, device=dev, dtype=torch.float16)
    E = H.epilogue(up[0], out_lo=up[1], gate=gt.to(dev), gate_kind=4)
    E.x3_out_exp = 20
    H.gemm_nt(A, Wo, E, M, N, K, H.X3)
    torch.cuda.synchronize()
    assert rel((up[0].double() + up[1].double()).cpu() * 2.0 ** -20, (dy.double() @ w.double().T) * gt.double()) < 2e-6
    # (d) the tail's tile widths: 64 columns with LeakyReLU (conv_before_upsample), 256 plain (the x4 upsampling convs)
    for N, leaky in ((64, True), (256, False)):
        M, K = 700, 576
        x, w, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05, torch.randn(N, generator=g)
        Wo, keep = _wsplit(w)
        A = H.rows(x.to(dev))
        A.x3_exp = 4
        out = torch.empty(M, N, device=dev)
        kw = dict(act=H.ACT_LEAKY, slope=0.01) if leaky else {}
        H.gemm_nt(A, Wo, H.epilogue(out, bias=b.to(dev), **kw), M, N, K, H.X3)
        ref = x.double() @ w.double().T + b.double()
        if leaky:
            ref = torch.where(ref > 0, ref, 0.01 * ref)
        torch.cuda.synchronize()
        assert rel(out, ref) < 2e-6, N
    # (e) the upsampling convs' stores: PixelShuffle(2) sub-pixel-major (forward, 256 columns = 2 tiles of 128) and
    # PixelUnshuffle(2) into the previous conv's pre-shuffle rows (input gradient, 64 columns)
    Bn, h, w_ = 2, 6, 10
    for mode, N in ((H.OUT_PSHUF_SPM, 256), (H.OUT_PUNSHUF_SPM, 64)):
        M = Bn * h * w_ * (1 if mode == H.OUT_PSHUF_SPM else 4)
        K = 576
        x, w, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) * 0.05, torch.randn(N, generator=g)
        Wo, keep = _wsplit(w)
        A = H.rows(x.to(dev))
        A.x3_exp = 4
        y = x.double() @ w.double().T + b.double()
        out = torch.full((Bn * h * w_ * 4, 64) if mode == H.OUT_PSHUF_SPM else (Bn * h * w_, 256), float("nan"), device=dev)
        H.gemm_nt(A, Wo, H.epilogue(out, mode=mode, ldo=out.shape[1], bias=b.to(dev), ps=(2, h, w_)), M, N, K, H.X3)
        if mode == H.OUT_PSHUF_SPM:   # row (b, y, x), column (i 2 + j) 64 + c -> pixel (b, 2y + i, 2x + j), channel c
            ref = y.view(Bn, h, w_, 2, 2, 64).permute(0, 1, 3, 2, 4, 5).reshape(-1, 64)
        else:                         # pixel (b, 2y + i, 2x + j), channel c -> row (b, y, x), column (i 2 + j) 64 + c
            ref = y.view(Bn, h, 2, w_, 2, 64).permute(0, 1, 3, 2, 4, 5).reshape(-1, 256)
        torch.cuda.synchronize()
        assert rel(out, ref) < 2e-6, mode


@pytest.mark.parametrize("conv", [None, "c192", "c64"])
def test_gemm_tn_x3_ring(conv):
    """The LDS-DMA ring form of kair_gemm_tn x3 (fp32 operands, 192 x 192 tiles): ragged splits over 3 N-tiles with
    the bias ones column carried in B's data, and the per-lane-tap im2col of a C-channel map (conv weight gradient,
    K = 9 C: the 192-channel RSTB convs, one tap per K tile; the 64-channel upsampling convs with N = 256, three
    taps per K tile and a partial N tile; an injected bias ones column) -- the split partial planes summed
    against float64."""
    g = torch.Generator().manual_seed(13)
    if conv:
        Bn, Hh, Ww, C, N = (2, 12, 20, 192, 192) if conv == "c192" else (2, 16, 40, 64, 256)
        M, K = Bn * Hh * Ww, 9 * C
        x = torch.randn(M, C, generator=g)
        cols = torch.nn.functional.unfold(x.view(Bn, Hh, Ww, C).permute(0, 3, 1, 2).double(), 3, padding=1)
        ref_b = cols.view(Bn, C, 9, Hh * Ww).permute(0, 3, 2, 1).reshape(M, K)
        oc = C + 7   # an injected bias ones column (tap 1: halo rows included)
        ref_b[:, oc] = 1.0
        Bop = H.im2col(x.to(dev), Hh, Ww, C, ones_col=oc)
    else:
        M, N, K = 3000, 576, 192
        x = torch.randn(M, K, generator=g)
        x[:, K - 12] = 1.0
        ref_b = x.double()
        Bop = H.rows(x.to(dev), ones_col=K - 12, ones_in_data=True)
    dy = torch.randn(M, N, generator=g) * 1e-6
    A = H.rows(dy.to(dev))
    A.x3_exp, Bop.x3_exp = 24, 4
    S = H.wgrad_splits(M, N, K)
    ws = torch.empty(S, N, K, device=dev)
    H.gemm_tn(A, Bop, ws, S, M, N, K, H.X3)
    torch.cuda.synchronize()
    assert rel(ws.sum(0), dy.double().T @ ref_b) < 2e-6


@pytest.mark.parametrize("f32_out", [False, True])
@pytest.mark.parametrize("shift", [0, 4])
def test_window_attention_x3(shift, f32_out):
    """kair_window_attn_fwd_x3 / _bwd_x3 against float64 autograd of WindowAttention (network_swinir.py:114-145)
    at the fp32 kernels' tolerances (fwd 2e-5, bwd 5e-5); dq/dk/dv as token rows; O and dq/dk/dv as fp16 pairs or
    (f32_out, the engine's form) fp32 in natural units."""
    B, Hh, Ww, nh, hd = 2, 16, 24, 6, 30
    nWin = B * (Hh // 8) * (Ww // 8)
    scale = hd ** -0.5
    g = torch.Generator().manual_seed(19)
    q, k, v = (torch.randn(nWin, nh, 64, hd, generator=g) for _ in range(3))
    table = torch.randn(225, nh, generator=g) * 0.5
    qr, kr, vr, tr = (t.double().clone().requires_grad_(True) for t in (q, k, v, table))
    o = _attn_ref(qr, kr, vr, tr, nh, shift, Hh, Ww, scale)
    go = torch.randn(o.shape, generator=g, dtype=torch.float64)
    o.backward(go)
    qkv = torch.zeros(3, nWin, nh, 64, 32)
    qkv[0, ..., :hd], qkv[1, ..., :hd], qkv[2, ..., :hd] = q, k, v
    e_act, e_grad = 4, 26    # exponents of the stored pairs: q/k/v / O and the gradients (dO ~ 1e-7 below)
    qkv_p = hilo(qkv.view(-1).to(dev), e_act)
    if f32_out:
        O = torch.full((nWin * 64, nh * 32), float("nan"), device=dev)
    else:
        O = torch.empty(2, nWin * 64, nh * 32, device=dev, dtype=torch.float16)
    lse = torch.empty(nWin, nh, 64, device=dev)
    H.window_attn_fwd_x3(qkv_p, table.to(dev), O, nh * 32, lse, nWin, nh, hd, scale, Hh, Ww, shift, e_in=e_act, e_out=e_act)
    torch.cuda.synchronize()
    if f32_out:
        Of = O.double().cpu().view(nWin, 64, nh, 32)
    else:
        Of = (O[0].double() + O[1].double()).cpu().view(nWin, 64, nh, 32) * 2.0 ** -e_act
    assert rel(Of[..., :hd].permute(0, 2, 1, 3), o.detach()) < 2e-6
    assert Of[..., hd:].abs().max() == 0
    dO = torch.zeros(nWin, 64, nh, 32)
    dO[..., :hd] = go.float().permute(0, 2, 1, 3) * 1e-7
    dO_p = hilo(dO.view(nWin * 64, nh * 32).to(dev), e_grad)
    if f32_out:
        dqkv = torch.full((nWin * 64, 3 * nh * 32), float("nan"), device=dev)
    else:
        dqkv = torch.empty(2, nWin * 64, 3 * nh * 32, device=dev, dtype=torch.float16)
    dtab = torch.empty(225, nh, device=dev)
    ws = torch.empty(H.window_attn_bwd_ws(nWin, nh), device=dev)
    H.window_attn_bwd_x3(qkv_p, O, nh * 32, dO_p, nh * 32, table.to(dev), lse, dqkv, dtab, False, ws, nWin, nh, hd, scale,
                         Hh, Ww, shift, e_act=e_act, e_grad=e_grad)
    torch.cuda.synchronize()
    if f32_out:
        d = dqkv.double().cpu().view(nWin, 64, 3, nh, 32)[..., :hd].permute(2, 0, 3, 1, 4) * 1e7
    else:
        d = (dqkv[0].double() + dqkv[1].double()).cpu().view(nWin, 64, 3, nh, 32)[..., :hd].permute(2, 0, 3, 1, 4)
        d = d * 2.0 ** -e_grad * 1e7
    assert rel(d[0], qr.grad) < 5e-6
    assert rel(d[1], kr.grad) < 5e-6
    assert rel(d[2], vr.grad) < 5e-6
    assert rel(dtab * 1e7, tr.grad) < 5e-6


def small(ups, sc, dt):
    return SwinIR(upscale=sc, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2, 2], embed_dim=60,
                  num_heads=[6, 6], mlp_ratio=2, upsampler=ups, resi_connection="1conv", drop_path_rate=0.0,
                  compute_dtype=dt)


@pytest.mark.parametrize("tag,ups,sc", [("classical", "pixelshuffle", 4), ("light", "pixelshuffledirect", 2)])
def test_swinir_small_x3_vs_golden(tag, ups, sc):
    """The fp32 engine's golden bars (tests/test_swinir_gpu.py::test_swinir_small_vs_golden, fp32 row)."""
    z = load_golden("swinir_small")
    pre = tag + "."
    net = small(ups, sc, "fp32x3")
    net.load_state_dict(sub_state(z, pre), strict=True)
    net = net.to(dev).train()
    L = torch.from_numpy(z[pre + "L"]).to(dev)
    Hh = torch.from_numpy(z[pre + "H"]).to(dev)
    E = net(L)
    assert rel(E, torch.from_numpy(z[pre + "E"])) < 1e-4
    loss = torch.nn.functional.l1_loss(E, Hh)
    loss.backward()
    g = sub_grads(z, pre)
    worst = max((rel(p.grad, g[k]), k) for k, p in net.named_parameters())
    assert worst[0] < 2e-3, worst


def test_swinir_classical_full_x3_vs_oracle():
    """The full classical x4 network on the fp16-pair engine vs the CPU oracle: outputs within SURVEY.md §8d's fp32
    bar (1e-5 relative; measured ~1e-6), PSNR float / uint8 within 1e-3 dB, every gradient within 1e-3."""
    from test_swinir_gpu import classical_x4, synth_batch
    net = classical_x4("fp32x3")
    ref = osw.SwinIR(4, 3, 48, 8, 1.0, [6] * 6, 180, [6] * 6, 2, "pixelshuffle")
    ref.load_state_dict(net.state_dict(), strict=True)
    L, Hh = synth_batch(2)
    Er = ref(L)
    torch.nn.functional.l1_loss(Er, Hh).backward()
    net = net.to(dev).train()
    E = net(L.to(dev))
    print("classical x4 fp32x3: output rel", rel(E, Er))
    assert rel(E, Er) < 1e-5
    for i in range(2):
        pf_gpu, pf_cpu = oimg.psnr_float(E[i].cpu(), Hh[i]), oimg.psnr_float(Er[i].detach(), Hh[i])
        assert abs(pf_gpu - pf_cpu) < 1e-3
        pu_gpu = oimg.calculate_psnr(oimg.tensor2uint(E[i].cpu()), oimg.tensor2uint(Hh[i]), border=4)
        pu_cpu = oimg.calculate_psnr(oimg.tensor2uint(Er[i].detach()), oimg.tensor2uint(Hh[i]), border=4)
        assert abs(pu_gpu - pu_cpu) < 1e-3
    torch.nn.functional.l1_loss(E, Hh.to(dev)).backward()
    gref = dict(ref.named_parameters())
    worst = max((rel(p.grad, gref[k].grad), k) for k, p in net.named_parameters())
    print("classical x4 fp32x3: worst gradient rel", worst)
    assert worst[0] < 1e-3, worst


def test_swinir_x3_lnfuse_engine(monkeypatch):
    """The opt-in fused LayerNorm backward (KAIR_X3_LNFUSE=1: kair_gemm_nt_x3_lnbwd at both LayerNorms of every Swin
    block) against the CPU oracle at the fp32 bars: 2 RSTBs of embed 180 (the one-tile C <= 192 the fused epilogue
    needs), output and every gradient."""
    monkeypatch.setenv("KAIR_X3_LNFUSE", "1")
    torch.manual_seed(5)
    kw = dict(upscale=2, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2, 2], embed_dim=180,
              num_heads=[6, 6], mlp_ratio=2, upsampler="pixelshuffle", resi_connection="1conv")
    net = SwinIR(drop_path_rate=0.0, compute_dtype="fp32x3", **kw)
    ref = osw.SwinIR(2, 3, 16, 8, 1.0, [2, 2], 180, [6, 6], 2, "pixelshuffle")
    ref.load_state_dict(net.state_dict(), strict=True)
    g = torch.Generator().manual_seed(6)
    L, Hh = torch.rand(2, 3, 16, 16, generator=g), torch.rand(2, 3, 32, 32, generator=g)
    Er = ref(L)
    torch.nn.functional.l1_loss(Er, Hh).backward()
    net = net.to(dev).train()
    assert net.engine().x3_lnfuse
    E = net(L.to(dev))
    torch.nn.functional.l1_loss(E, Hh.to(dev)).backward()
    assert rel(E, Er) < 1e-5
    gref = dict(ref.named_parameters())
    worst = max((rel(p.grad, gref[k].grad), k) for k, p in net.named_parameters())
    print("lnfuse: worst gradient rel", worst)
    assert worst[0] < 1e-3, worst


@pytest.mark.parametrize("use_graph", [False, True])
def test_trainer_x3_matches_reference_trajectory(use_graph):
    """3 fused-trainer steps on the fp16-pair engine against the reference ModelPlain trajectory (1e-4)."""
    z = load_golden("train_trajectory")
    mk = lambda: SwinIR(upscale=4, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2, 2], embed_dim=60,
                        num_heads=[6, 6], mlp_ratio=2, upsampler="pixelshuffle", drop_path_rate=0.0,
                        compute_dtype="fp32x3")
    net, ema = mk(), mk()
    net.load_state_dict(sub_state(z, "init."), strict=True)
    ema.load_state_dict(sub_state(z, "init."), strict=True)
    net, ema = net.to(dev).train(), ema.to(dev).eval()
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999, use_graph=use_graph)
    milestones, lr0 = [2, 100], 2e-4
    losses = []
    for s in range(1, 4):
        tr.lr = lr0 * 0.5 ** sum(1 for m in milestones if m <= s)
        loss = tr.step(torch.from_numpy(z[f"step{s}.L"]).to(dev), torch.from_numpy(z[f"step{s}.H"]).to(dev))
        losses.append(loss.item())
    np.testing.assert_allclose(losses, z["losses"], rtol=1e-4)
    fg, fe = sub_state(z, "final.G."), sub_state(z, "final.E.")
    for k, v in net.state_dict().items():
        assert rel(v.float(), fg[k].float()) < 1e-4, k
    for k, v in ema.state_dict().items():
        assert rel(v.float(), fe[k].float()) < 1e-4, k


def test_droppath_injected_masks_x3_vs_oracle():
    """DropPath with the same keep masks in the fp16-pair engine and the oracle (fwd + every gradient)."""
    torch.manual_seed(4)
    net = SwinIR(upscale=2, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2, 2], embed_dim=60,
                 num_heads=[6, 6], mlp_ratio=2, upsampler="pixelshuffle", drop_path_rate=0.3, compute_dtype="fp32x3")
    ref = osw.SwinIR(2, 3, 16, 8, 1.0, [2, 2], 60, [6, 6], 2, "pixelshuffle")
    ref.load_state_dict(net.state_dict(), strict=True)
    B = 3
    keep = torch.tensor([1.0 - b.drop_path_rate for l in net.layers for b in l.residual_group.blocks])
    g = torch.Generator().manual_seed(9)
    D = (torch.rand(len(keep), 2, B, generator=g) < 0.6).float() / keep.view(-1, 1, 1)
    D[1, 0, 0] = 0.0
    D[1, 1, 0] = 1.0 / keep[1]
    L = torch.rand(B, 3, 16, 16, generator=g)
    gE = torch.randn(B, 3, 32, 32, generator=g)
    keeps = [(D[i, 0].view(B, 1, 1), D[i, 1].view(B, 1, 1)) for i in range(len(keep))]
    Er = ref(L, keeps)
    Er.backward(gE)
    net = net.to(dev).train()
    eng = net.engine()
    E = eng.forward(L.to(dev), D.to(dev)).clone()
    params = list(net.parameters())
    flat = torch.zeros(sum(p.numel() for p in params), device=dev)
    grads, off = {}, 0
    for p in params:
        grads[p] = flat[off:off + p.numel()].view_as(p)
        off += p.numel()
    eng.backward_from_grad(gE.to(dev), grads)
    assert rel(E, Er.detach()) < 1e-4
    gref = dict(ref.named_parameters())
    worst = max((rel(grads[p], gref[k].grad), k) for k, p in net.named_parameters())
    assert worst[0] < 2e-3, worst
