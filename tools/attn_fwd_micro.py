"""Isolated launch time of the fused attention half (kair_swin_attn_fwd) at B = 32 and B = 4 (48x48
LQ, C 180, 6 heads), graph-timed.  With a --debug-ablations library, KAIR_ATTN_DBG=1 drops the q/k/v
stores, =2 the end-of-window stores (perf investigation only).   python tools/attn_fwd_micro.py [lib.so]"""
import os
import sys
import torch
sys.path.insert(0, "/root/repo")
from kair_amd import _hip as H
if len(sys.argv) > 1:
    import ctypes
    H.LIB_PATH = os.path.abspath(sys.argv[1])
    _probe = ctypes.CDLL(H.LIB_PATH)   # an older variant may lack newer debug entry points
    H._SIGS = {k: v for k, v in H._SIGS.items() if hasattr(_probe, k)}
dev = torch.device("cuda", 0)
C, CP, NH = 180, 192, 6


def timeit(f, reps=40):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay(); torch.cuda.synchronize()
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000


def pack(w, kind, n_grp, k_grp):
    out = torch.empty(n_grp[0] * n_grp[2], k_grp[0] * k_grp[2], device=dev, dtype=torch.bfloat16)
    H.pack_weight(w, out, H.wmap(kind, w.shape[0], w.shape[1], n_grp, k_grp))
    return out


g = torch.Generator().manual_seed(0)
wq = pack((0.05 * torch.randn(3 * C, C, generator=g)).to(dev), 10, (3 * NH, C // NH, 32), (1, C, CP))
wp = pack((0.05 * torch.randn(C, C, generator=g)).to(dev), 10, (1, C, CP), (NH, C // NH, 32))
bq, bp = torch.zeros(3 * NH * 32, device=dev), torch.zeros(CP, device=dev)
table = (0.1 * torch.randn(225, NH, generator=g)).to(dev)
gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
dbg = os.environ.get("KAIR_ATTN_DBG", "0")
for B in (32, 4):
    Hh = Ww = 48
    M = B * Hh * Ww
    nWin = M // 64
    x = torch.randn(M, CP, device=dev); x[:, C:] = 0
    ln = torch.empty(M, CP, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    qkv = torch.empty(3 * M * NH * 32, device=dev, dtype=torch.bfloat16)
    O = torch.empty(M, NH * 32, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(nWin * NH * 64, device=dev)
    out = torch.empty(M, CP, device=dev)
    for shift in (0, 4):
        t = timeit(lambda: H.swin_attn_fwd(x, CP, gamma, beta, 1e-5, C, ln, CP, mean, rstd, wq, bq, qkv, table, 30 ** -0.5, O,
                                           NH * 32, C // NH, lse, wp, bp, None, 0, out, CP, nWin, NH, Hh, Ww, shift))
        print("dbg %s B %2d shift %d: %7.1f us  (%.2f TB/s algorithmic)" % (dbg, B, shift, t, nWin * 209408 / t / 1e6), flush=True)
