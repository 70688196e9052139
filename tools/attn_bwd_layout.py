"""Isolated timing of the bf16 attention backward at B = 32 (1152 windows, 6 heads): dq/dk/dv
head-blocked vs token rows (kair_window_attn_bwd_ex)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
for B in (32, 4):
    nWin, nh, hd, Hh, Ww = B * 36, 6, 30, 48, 48
    qkv = (torch.randn(3, nWin, nh, 64, 32, device=dev) * 0.5).to(bf)
    O = torch.randn(nWin * 64, nh * 32, device=dev).to(bf)
    dO = torch.randn(nWin * 64, nh * 32, device=dev).to(bf)
    lse = torch.randn(nWin, nh, 64, device=dev).abs() + 3
    table = torch.randn(225, nh, device=dev)
    ws = torch.empty(H.window_attn_bwd_ws(nWin, nh), device=dev)
    d_blk = torch.empty(3 * nWin * nh * 64 * 32, device=dev, dtype=bf)
    d_row = torch.empty(nWin * 64, 3 * nh * 32, device=dev, dtype=bf)
    for name, d, rows in (("blocked", d_blk, False), ("rows", d_row, True)):
        f = lambda: H.window_attn_bwd(qkv, O, nh * 32, dO, nh * 32, table, lse, d, None, False, ws, nWin, nh, hd,
                                      hd ** -0.5, Hh, Ww, 4, dqkv_rows=rows)
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(f"B={B} {name}: {e0.elapsed_time(e1) * 1e3 / 20:.1f} us", flush=True)
