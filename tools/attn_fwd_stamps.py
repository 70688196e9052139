"""Phase timing of the fused attention half (kair_swin_attn_fwd, a --debug-ablations library with
KAIR_ATTN_DBG bit 8): median s_memtime cycles per phase of each workgroup's last window, per wave, at
B = 32 and B = 4 (48x48 LQ, C 180, 6 heads).   KAIR_ATTN_DBG=8 python tools/attn_fwd_stamps.py lib.so"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402

if len(sys.argv) > 1:
    H.LIB_PATH = os.path.abspath(sys.argv[1])
dev = torch.device("cuda", 0)
C, CP, NH = 180, 192, 6
NAMES = ["LN+row map", "QKV mfma", "q/k/v stores", "S+softmax", "PV+O tile", "proj mfma", "out stores+barrier"]


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
        H.debug_fused_stamps()   # clears
        for _ in range(3):
            H.swin_attn_fwd(x, CP, gamma, beta, 1e-5, C, ln, CP, mean, rstd, wq, bq, qkv, table, 30 ** -0.5, O,
                            NH * 32, C // NH, lse, wp, bp, None, 0, out, CP, nWin, NH, Hh, Ww, shift)
        torch.cuda.synchronize()
        a = np.array(H.debug_fused_stamps(), dtype=np.uint64).reshape(-1, 8).astype(np.int64)
        a = a[a[:, 0] > 0]
        simd = (a[:, 0] >> 56) & 3
        a[:, 0] &= (1 << 56) - 1
        d = np.diff(a, axis=1)
        tot = a[:, 7] - a[:, 0]
        res = {"B": B, "shift": shift, "waves": int(len(a)),
               "phase_cycles_median": {k: float(np.median(d[:, i])) for i, k in enumerate(NAMES)},
               "window_median": float(np.median(tot)), "window_p90": float(np.percentile(tot, 90)),
               "simd_of_wave_in_wg": [int(np.bincount(simd[w::6], minlength=4).argmax()) for w in range(6)]}
        print(json.dumps(res), flush=True)
