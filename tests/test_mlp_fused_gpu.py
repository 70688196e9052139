"""kair_swin_mlp_fwd (csrc/swin_fused.hip, the weight-resident kernel) against a float64 torch
restatement of the MLP half of a Swin block on the same bf16 operands:

    out = x + s * fc2(GELU(fc1(LN2(x))))      network_swinir.py:274-276, Mlp.forward :24-30

with the tensors it saves for backward (ln2 with 1.0 at column C, mean / rstd, GELU'(u), GELU(u)
with 1.0 at column hd).  Shapes are the classical x4 block's (C 180 -> 192, hidden 360 -> 384), at
sizes with one tile per workgroup (M = 1152) and several persistent passes (M = 73,728 / 8)."""
import pytest
import torch

from kair_amd import _hip as H

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)
C, CP, HD, HDP = 180, 192, 360, 384


def _pack(w, kind, n_grp, k_grp):
    Np, Kp = n_grp[0] * n_grp[2], k_grp[0] * k_grp[2]
    out = torch.empty(Np, Kp, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w, out, H.wmap(kind, w.shape[0], w.shape[1], n_grp, k_grp))
    return out


@pytest.mark.parametrize("M,rows_per_scale", [(1152, 576), (9216, 2304), (73728 // 8, 2304)])
def test_swin_mlp_fwd_vs_float64(M, rows_per_scale):
    g = torch.Generator().manual_seed(3)
    x = torch.zeros(M, CP)
    x[:, :C] = torch.randn(M, C, generator=g) * 1.5 + 0.3
    gamma, beta = 1 + 0.2 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    w1, b1 = 0.05 * torch.randn(HD, C, generator=g), 0.05 * torch.randn(HD, generator=g)
    w2, b2 = 0.05 * torch.randn(C, HD, generator=g), 0.05 * torch.randn(C, generator=g)
    nsc = M // rows_per_scale
    scale = torch.tensor([1.0, 0.0, 1.25, 0.8] * nsc)[:nsc]
    W1 = _pack(w1.to(dev), 10, (1, HD, HDP), (1, C, CP))
    W2 = _pack(w2.to(dev), 14, (1, C, CP), (1, HD, HDP))
    b1p = torch.zeros(HDP); b1p[:HD] = b1
    b2p = torch.zeros(CP); b2p[:C] = b2
    xd = x.to(dev)
    ln = torch.empty(M, CP, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    u = torch.empty(M, HDP, device=dev, dtype=torch.bfloat16)
    h = torch.empty(M, HDP, device=dev, dtype=torch.bfloat16)
    out = torch.full((M, CP), 7.0, device=dev)
    H.swin_mlp_fwd(xd, CP, gamma.to(dev), beta.to(dev), 1e-5, C, ln, CP, mean, rstd, W1, b1p.to(dev), u, h, HDP, HD, W2,
                   b2p.to(dev), scale.to(dev), rows_per_scale, out, CP, M, CP, HDP)
    torch.cuda.synchronize()

    xd64 = x[:, :C].double()
    mu = xd64.mean(1)
    rs = 1.0 / torch.sqrt(xd64.var(1, unbiased=False) + 1e-5)
    assert (mean.cpu().double() - mu).abs().max().item() < 1e-5
    assert ((rstd.cpu().double() - rs).abs() / rs).max().item() < 1e-5
    lnr = (xd64 - mu[:, None]) * rs[:, None] * gamma.double() + beta.double()
    lng = ln.cpu().double()
    assert (lng[:, :C] - lnr).abs().max().item() < 2e-2 * lnr.abs().max().item()   # bf16 rounding
    assert (lng[:, C] == 1).all() and (lng[:, C + 1:] == 0).all()
    # the rest of the chain from the kernel's own bf16 LN output and bf16 weights (products in fp64)
    w1b = w1.to(torch.bfloat16).double()
    w2b = w2.to(torch.bfloat16).double()
    uu = lng[:, :C] @ w1b.t() + b1.double()
    cdf = 0.5 * (1 + torch.erf(uu / 2 ** 0.5))
    hr = uu * cdf
    gr = cdf + uu * torch.exp(-0.5 * uu * uu) / (2 * torch.pi) ** 0.5
    hg, ug = h.cpu().double(), u.cpu().double()
    assert (hg[:, :HD] - hr).abs().max().item() < 1e-2 * hr.abs().max().item() + 1e-3
    assert (ug[:, :HD] - gr).abs().max().item() < 1e-2
    assert (hg[:, HD] == 1).all() and (hg[:, HD + 1:] == 0).all()
    y = hg[:, :HD] @ w2b.t() + b2.double()
    s = scale.double().repeat_interleave(rows_per_scale)[:, None]
    ref = x.double().clone()
    ref[:, :C] += s * y
    err = (out.cpu().double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-4, err


@pytest.mark.parametrize("N,K,n_grp,k_grp", [
    (540, 180, (18, 30, 32), (1, 180, 192)),   # qkv: head-padded rows
    (180, 180, (1, 180, 192), (6, 30, 32)),    # proj: head-padded contraction
    (360, 180, (1, 360, 384), (1, 180, 192)),  # fc1
    (180, 360, (1, 180, 192), (1, 360, 384)),  # fc2
])
def test_batched_pack_matches_elementwise(N, K, n_grp, k_grp):
    """kair_pack_weights (one launch; the bf16 linear forms 0 / 10 / 13 / 14 packed 8 elements per
    thread in source-row order) == kair_pack_weight (one thread per packed element), bit for bit."""
    g = torch.Generator().manual_seed(N + K)
    w = torch.randn(N, K, generator=g).to(dev)
    Np, Kp = n_grp[0] * n_grp[2], k_grp[0] * k_grp[2]
    jobs, refs = [], []
    for kind in (0, 3, 10, 13, 14):
        m = H.wmap(kind, N, K, n_grp, k_grp)
        shape = (Kp, Np) if kind in (3, 13) else (Np, Kp)
        ref = torch.empty(shape, device=dev, dtype=torch.bfloat16)
        H.pack_weight(w, ref, m)
        dst = torch.full(shape, 3.0, device=dev, dtype=torch.bfloat16)
        jobs.append((w, dst, m))
        refs.append(ref)
    t = H.PackTable(jobs)
    t.run()
    torch.cuda.synchronize()
    for (_, dst, m), ref in zip(jobs, refs):
        assert torch.equal(dst, ref), m.kind


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N, K, n_grp, k_grp", [
    (180, 180, (1, 180, 192), (6, 30, 32)),    # Swin proj / RSTB conv: padded groups
    (540, 180, (1, 540, 576), (1, 180, 192)),  # qkv
    (64, 180, (1, 64, 64), (1, 180, 192)),     # conv_before_upsample-like widths
])
def test_batched_pair_pack_matches_elementwise(dt, N, K, n_grp, k_grp):
    """kair_pack_weights on the split pair forms (kinds 9 / 17 / 18 / 19: the fp32x3 engine's fp16 pairs of w 2^12,
    or bf16 hi / lo; 8 columns of one packed row per thread) == kair_pack_weight (one thread per packed element),
    bit for bit."""
    g = torch.Generator().manual_seed(N + 3 * K)
    w_lin = torch.randn(N, K, generator=g).to(dev)
    w_conv = torch.randn(N, K, 3, 3, generator=g).to(dev)
    Np, Kp = n_grp[0] * n_grp[2], k_grp[0] * k_grp[2]
    r64 = lambda n: 2 * ((n + 63) // 64) * 64
    shapes = {9: (Np, r64(9 * Kp)), 17: (Np, r64(Kp)), 18: (Kp, r64(9 * Np)), 19: (Kp, r64(Np))}
    jobs, refs = [], []
    for kind, shape in shapes.items():
        w = w_conv if kind in (9, 18) else w_lin
        m = H.wmap(kind, N, K, n_grp, k_grp)
        ref = torch.empty(shape, device=dev, dtype=dt)
        H.pack_weight(w, ref, m)
        dst = torch.full(shape, 3.0, device=dev, dtype=dt)
        jobs.append((w, dst, m))
        refs.append(ref)
    t = H.PackTable(jobs)
    t.run()
    torch.cuda.synchronize()
    for (_, dst, m), ref in zip(jobs, refs):
        assert torch.equal(dst, ref), m.kind
