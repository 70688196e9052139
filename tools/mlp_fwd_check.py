"""Repeated kair_swin_mlp_fwd runs checked element by element against float64 (h, GELU', output):
the check that found the buffer-store data hazard (common.h buf_st*).  python tools/mlp_fwd_check.py [lib.so]"""
import sys, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
from kair_amd import _hip as H
import test_mlp_fused_gpu as TM
dev = TM.dev
C, CP, HD, HDP = TM.C, TM.CP, TM.HD, TM.HDP
import os
if len(sys.argv) > 1: H.LIB_PATH = os.path.abspath(sys.argv[1])
print("lib", H.LIB_PATH)
for rep in range(2):
    M, rps = 1152, 576
    g = torch.Generator().manual_seed(3)
    x = torch.zeros(M, CP); x[:, :C] = torch.randn(M, C, generator=g) * 1.5 + 0.3
    gamma, beta = 1 + 0.2 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    w1, b1 = 0.05 * torch.randn(HD, C, generator=g), 0.05 * torch.randn(HD, generator=g)
    w2, b2 = 0.05 * torch.randn(C, HD, generator=g), 0.05 * torch.randn(C, generator=g)
    W1 = TM._pack(w1.to(dev), 10, (1, HD, HDP), (1, C, CP)); W2 = TM._pack(w2.to(dev), 14, (1, C, CP), (1, HD, HDP))
    b1p = torch.zeros(HDP); b1p[:HD] = b1
    b2p = torch.zeros(CP); b2p[:C] = b2
    ln = torch.full((M, CP), 3.0, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.full((M,), -5.0, device=dev), torch.full((M,), -5.0, device=dev)
    u = torch.full((M, HDP), 3.0, device=dev, dtype=torch.bfloat16); h = torch.full_like(u, 3.0)
    out = torch.full((M, CP), 7.0, device=dev)
    H.swin_mlp_fwd(x.to(dev), CP, gamma.to(dev), beta.to(dev), 1e-5, C, ln, CP, mean, rstd, W1, b1p.to(dev), u, h, HDP, HD, W2,
                   b2p.to(dev), None, 0, out, CP, M, CP, HDP)
    torch.cuda.synchronize()
    lng = ln.cpu().double()
    w1b = w1.to(torch.bfloat16).double()
    uu = lng[:, :C] @ w1b.t() + b1.double()
    cdf = 0.5 * (1 + torch.erf(uu / 2 ** 0.5))
    hr = uu * cdf
    gr = cdf + uu * torch.exp(-0.5 * uu * uu) / (2 * torch.pi) ** 0.5
    hg, ug = h.cpu().double(), u.cpu().double()
    dh = (hg[:, :HD] - hr).abs(); du = (ug[:, :HD] - gr).abs()
    bh = (dh > 0.02).nonzero(); bu = (du > 0.02).nonzero()
    print("rep", rep, "ln pad ok", bool((lng[:, C] == 1).all()), bool((lng[:, C+1:] == 0).all()), "h pad", bool((hg[:, HD] == 1).all()), bool((hg[:, HD+1:] == 0).all()))
    print("  h bad", bh.shape[0], bh[:6].tolist(), " u bad", bu.shape[0], bu[:6].tolist())
    if bh.shape[0]: r, c = bh[0].tolist(); print("   h", r, c, hg[r, c].item(), hr[r, c].item())
    if bu.shape[0]: r, c = bu[0].tolist(); print("   u", r, c, ug[r, c].item(), gr[r, c].item())
    y = hg[:, :HD] @ w2.to(torch.bfloat16).double().t() + b2.double()
    ref = x.double().clone(); ref[:, :C] += y
    print("  out err", ((out.cpu().double() - ref).abs().max() / ref.abs().max()).item())
