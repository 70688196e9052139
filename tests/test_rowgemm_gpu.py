"""kair_rowgemm_{store,gate,lnbwd} (csrc/rowgemm.hip) against a float64 torch restatement of the same
products: the Swin-block input gradients (nn.Linear backward, network_swinir.py:19-20, 105, 107)
with the LayerNorm backward (norm1 / norm2, :199, :205; ln_bwd_kernel maths) fused into the epilogue.

Shapes are the classical x4 block's (C = 180 -> 192 padded, hidden 360 -> 384, q/k/v 3 x 6 x 32),
at sizes that need several persistent passes per workgroup and rows past M."""
import pytest
import torch

from kair_amd import _hip as H

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)
C, CP, HD, HDP, NH = 180, 192, 360, 384, 6


def _lin(N, K, n_grp, k_grp, seed):
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(N, K, generator=g) * 0.05).to(dev)
    Np, Kp = n_grp[0] * n_grp[2], k_grp[0] * k_grp[2]
    frag = torch.empty(Kp, Np, device=dev, dtype=torch.bfloat16)        # kind 13: [Kp/32][Np/16][64][8]
    H.pack_weight(w, frag, H.wmap(13, N, K, n_grp, k_grp))
    plain = torch.empty(Np, Kp, device=dev, dtype=torch.bfloat16)       # kind 0: [Np][Kp] (padded), same rounding
    H.pack_weight(w, plain, H.wmap(0, N, K, n_grp, k_grp))
    return frag, plain


LINEARS = {   # dgrad contraction K (= the linear's padded N), output N (= the linear's padded K)
    "proj": (lambda s: _lin(C, C, (1, C, CP), (NH, C // NH, 32), s), CP, CP),
    "fc1": (lambda s: _lin(HD, C, (1, HD, HDP), (1, C, CP), s), HDP, CP),
    "qkv": (lambda s: _lin(3 * C, C, (3 * NH, C // NH, 32), (1, C, CP), s), 3 * NH * 32, CP),
    "fc2": (lambda s: _lin(C, HD, (1, C, CP), (1, HD, HDP), s), CP, HDP),
}


def _rows(M, K, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(M, K, generator=g)).to(dev, torch.bfloat16)


@pytest.mark.parametrize("name", ["proj", "fc1", "qkv", "fc2"])
@pytest.mark.parametrize("M", [4608, 4600, 37])
def test_rowgemm_store_and_gate(name, M):
    make, K, N = LINEARS[name]
    frag, plain = make(1)
    A = _rows(M, K, 2)
    ref = A.double() @ plain.double()                                    # [M, N]
    out = torch.full((M, N), 7.0, device=dev, dtype=torch.bfloat16)
    H.rowgemm_store(A, M, K, frag, N, out)
    torch.cuda.synchronize()
    err = (out.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 8e-3, err                                               # bf16 output rounding
    g = torch.rand(M, N, device=dev).to(torch.bfloat16)
    out2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    H.rowgemm_gate(A, M, K, frag, N, g, out2)
    ref2 = ref * g.double()
    err2 = (out2.double() - ref2).abs().max().item() / ref2.abs().max().item()
    assert err2 < 8e-3, err2


def _win_perm(B, Hh, Ww, shift):
    """perm[r] = token read by window-order row r (roll(-shift) + window_partition, network_swinir.py:250-256)."""
    idx = torch.arange(B * Hh * Ww).view(B, Hh, Ww)
    if shift:
        idx = torch.roll(idx, (-shift, -shift), (1, 2))
    return idx.view(B, Hh // 8, 8, Ww // 8, 8).permute(0, 1, 3, 2, 4).reshape(-1)


@pytest.mark.parametrize("name,shift,cshift", [("qkv", 4, 0), ("qkv", 0, 0), ("fc1", 0, 4), ("fc1", 0, 0)])
def test_rowgemm_lnbwd(name, shift, cshift):
    """D += LN-backward(A . W^T) for GEMM rows in window order `shift` (qkv -> LN1) or token order
    (fc1 -> LN2), the copy in window order `cshift` scaled per sample, and the dgamma / dbeta partials."""
    make, K, N = LINEARS[name]
    B, Hh, Ww = 3, 48, 40
    M = B * Hh * Ww
    frag, plain = make(3)
    A = _rows(M, K, 4)
    g = torch.Generator().manual_seed(5)
    x = torch.zeros(M, CP)
    x[:, :C] = torch.randn(M, C, generator=g) * 2 + 0.5
    gamma = torch.randn(C, generator=g)
    D0 = torch.zeros(M, CP)
    D0[:, :C] = torch.randn(M, C, generator=g)
    mu = x[:, :C].mean(1)
    rstd = 1.0 / torch.sqrt(x[:, :C].var(1, unbiased=False) + 1e-5)
    scale = torch.tensor([1.0, 0.0, 1.25])
    xd, Dd = x.to(dev), D0.to(dev).clone()
    copy = torch.zeros(M, CP, device=dev, dtype=torch.bfloat16)
    nb = H.rowgemm_ln_blocks(M, K)
    part = torch.empty(nb * 2 * C, device=dev)
    win = (Hh, Ww, 8, shift) if shift or name == "qkv" else (0, 0, 0, 0)
    cwin = (Hh, Ww, 8, cshift) if name == "fc1" else None
    cd = H.copy_desc(copy, rowscale=scale.to(dev), rows_per_scale=Hh * Ww, win=cwin)
    H.rowgemm_lnbwd(A, M, K, frag, xd, gamma.to(dev), mu.to(dev), rstd.to(dev), C, Dd, part, win=win, copy=cd)
    dgam = torch.empty(C, device=dev)
    dbet = torch.empty(C, device=dev)
    H.ln_param_reduce_grouped([(part, M, C, dgam, dbet, False, nb)])
    torch.cuda.synchronize()

    # float64 restatement
    Y = A.double().cpu() @ plain.double().cpu()                          # [M (GEMM rows), 192]
    perm = _win_perm(B, Hh, Ww, win[3]) if win[2] else torch.arange(M)
    dy = torch.zeros(M, CP, dtype=torch.float64)
    dy[perm] = Y                                                         # token rows
    dy = dy[:, :C]
    xh = (x[:, :C].double() - mu.double()[:, None]) * rstd.double()[:, None]
    gy = dy * gamma.double()
    dx = rstd.double()[:, None] * (gy - gy.mean(1, keepdim=True) - xh * (gy * xh).mean(1, keepdim=True))
    Dref = D0.double().clone()
    Dref[:, :C] += dx
    err = (Dd.double().cpu() - Dref).abs().max().item() / Dref.abs().max().item()
    assert err < 2e-5, err
    assert Dd[:, C:].abs().max().item() == 0.0                           # pad columns untouched
    sc = scale.double().repeat_interleave(Hh * Ww)[:, None]
    cref = torch.zeros(M, CP, dtype=torch.float64)
    crow = torch.argsort(_win_perm(B, Hh, Ww, cwin[3])) if cwin else torch.arange(M)
    cref[crow] = Dref * sc
    errc = (copy.double().cpu() - cref).abs().max().item() / cref.abs().max().item()
    assert errc < 8e-3, errc
    dg_ref, db_ref = (dy * xh).sum(0), dy.sum(0)
    assert (dgam.double().cpu() - dg_ref).abs().max().item() / dg_ref.abs().max().item() < 2e-5
    assert (dbet.double().cpu() - db_ref).abs().max().item() / db_ref.abs().max().item() < 2e-5


def test_rowgemm_rejects_bad_shapes():
    A = torch.zeros(64, 200, device=dev, dtype=torch.bfloat16)
    W = torch.zeros(192 * 200, device=dev, dtype=torch.bfloat16)
    out = torch.zeros(64, 192, device=dev, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        H.rowgemm_store(A, 64, 200, W, 192, out)   # K must be 192 / 384 / 576
