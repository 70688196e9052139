"""Micro-benchmark of the split-fp16 (x3) GEMMs at the SwinIR classical x4 block shapes (B = 32, M = 73,728
tokens): every Swin-block linear forward / input gradient (kair_gemm_nt compute X3) and weight gradient
(kair_gemm_tn compute X3), timed with HIP events over R launches captured in one graph.  Printed per case:
us per launch, issued TFLOP/s (3 fp16 products per multiply-add) and its fraction of the dense fp16 MFMA peak,
and algorithmic GB/s (operands read once, outputs written once, fp32 4 B / fp16 pair 4 B per element).

    python tools/x3_micro.py [substring] [--reps R]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402
from tools.gemm_micro import timeit  # noqa: E402

dev = torch.device("cuda")
M = int(os.environ.get("X3_MICRO_B", "32")) * 48 * 48   # X3_MICRO_B: the per-GPU batch (B = 4: the 8-GPU shape)
PEAK_F16 = 2500.0


def pair(x, e):
    w = x * 2.0 ** e
    hi = w.to(torch.float16)
    return torch.stack([hi, (w - hi.float()).to(torch.float16)])


def wpack(N, K):
    w = torch.randn(N, K, device=dev) * 0.05
    Wp = torch.empty(N, 2 * (-(-K // 64)) * 64, device=dev, dtype=torch.float16)
    H.pack_weight(w, Wp, H.wmap(17, N, K))
    return Wp


def nt_case(N, K, a_pair, out_pair, epi):
    A = torch.randn(M, K, device=dev)
    Ap = pair(A, 4) if a_pair else None
    Wp = wpack(N, K)
    out = torch.empty(2, M, N, device=dev, dtype=torch.float16) if out_pair else torch.empty(M, N, device=dev)
    extra = {}
    if epi == "resid":
        extra["resid"] = torch.randn(M, N, device=dev)
    elif epi == "gate":
        extra["gate"], extra["gate_kind"] = torch.randn(M, N, device=dev), 4
    elif epi == "gelu":
        extra["act"], extra["pre"], extra["pre_grad"] = H.ACT_GELU, torch.empty(M, N, device=dev), True

    def run():
        a = H.with_lo(H.rows(Ap[0]), Ap[1]) if a_pair else H.rows(A)
        a.x3_exp = 4
        b = H.rows(Wp)
        b.x3_exp = H.X3_WEXP
        e = H.epilogue(out[0] if out_pair else out, out_lo=out[1] if out_pair else None, **extra)
        if out_pair:
            e.x3_out_exp = 4
        H.gemm_nt(a, b, e, M, N, K, H.X3)
    nb = 4 * M * K + 4 * M * N + sum(4 * M * N for k in ("resid", "gate", "pre") if k in extra)
    return run, 2.0 * 3 * M * N * K, nb


def tn_case(N, K, a_pair, b_pair, conv=False):
    A = torch.randn(M, N, device=dev) * 1e-6
    Bm = torch.randn(M, 192 if conv else K, device=dev)
    Ap, Bp = pair(A, 24) if a_pair else None, pair(Bm, 4) if b_pair else None
    S = H.wgrad_splits(M, N, K)
    ws = torch.empty(S, N, K, device=dev)

    def run():
        a = H.with_lo(H.rows(Ap[0]), Ap[1]) if a_pair else H.rows(A)
        if conv:
            b = H.im2col(Bm, 48, 48, 192)
        else:
            b = H.with_lo(H.rows(Bp[0]), Bp[1]) if b_pair else H.rows(Bm)
        a.x3_exp, b.x3_exp = 24, 4
        H.gemm_tn(a, b, ws, S, M, N, K, H.X3)
    return run, 2.0 * 3 * M * N * K, 4 * M * (N + (192 if conv else K)) + 4 * S * N * K


def nt_conv():
    x = torch.randn(M, 192, device=dev)
    Wp = wpack(192, 1728)
    out = torch.empty(M, 192, device=dev)

    def run():
        a = H.im2col(x, 48, 48, 192)
        a.x3_exp = 4
        b = H.rows(Wp)
        b.x3_exp = H.X3_WEXP
        H.gemm_nt(a, b, H.epilogue(out), M, 192, 1728, H.X3)
    return run, 2.0 * 3 * M * 192 * 1728, 4 * M * 192 * 2


def attn_case(bwd):
    """The split window attention at C4's block shape: 1152 windows x 6 heads (head dim 30), shift 4."""
    nWin, nh, hd = M // 64, 6, 30
    qkv = pair(torch.randn(3 * M * nh * 32, device=dev), 4)
    table = torch.randn(225, nh, device=dev) * 0.5
    O = torch.empty(M, nh * 32, device=dev)
    lse = torch.empty(nWin * nh * 64, device=dev)
    H.window_attn_fwd_x3(qkv, table, O, nh * 32, lse, nWin, nh, hd, hd ** -0.5, 48, 48, 4, ones_col=hd, e_in=4, e_out=4)
    dO = pair(torch.randn(M, nh * 32, device=dev) * 1e-6, 24)
    dqkv = torch.empty(M, 3 * nh * 32, device=dev)
    ws = torch.empty(H.window_attn_bwd_ws(nWin, nh), device=dev)

    def run():
        if bwd:
            H.window_attn_bwd_x3(qkv, O, nh * 32, dO, nh * 32, table, lse, dqkv, None, False, ws, nWin, nh, hd, hd ** -0.5,
                                 48, 48, 4, e_act=4, e_grad=24)
        else:
            H.window_attn_fwd_x3(qkv, table, O, nh * 32, lse, nWin, nh, hd, hd ** -0.5, 48, 48, 4, ones_col=hd, e_in=4,
                                 e_out=4)
    fl = nWin * nh * (5 if bwd else 2) * 2 * 64 * 64 * hd
    nb = M * nh * ((8 if bwd else 4) * hd * 4 + 4)
    return run, 3.0 * fl, nb


def cases():
    return {   # the pair engine's forms (round 6: every block operand an fp16 pair) and, *_f32, the fp32-operand forms
        "nt_qkv_fwd": nt_case(576, 192, True, True, None),
        "nt_proj_fwd": nt_case(192, 192, True, False, "resid"),
        "nt_fc1_fwd": nt_case(384, 192, True, True, "gelu"),
        "nt_fc1_fwd_f32": nt_case(384, 192, False, False, "gelu"),
        "nt_fc2_fwd": nt_case(192, 384, True, False, "resid"),
        "nt_fc2_dgrad": nt_case(384, 192, True, True, "gate"),
        "nt_fc2_dgrad_f32": nt_case(384, 192, False, False, "gate"),
        "nt_fc1_dgrad": nt_case(192, 384, True, False, None),
        "nt_proj_dgrad": nt_case(192, 192, True, True, None),
        "nt_qkv_dgrad": nt_case(192, 576, True, False, None),
        "tn_qkv": tn_case(576, 192, True, True),
        "tn_proj": tn_case(192, 192, True, True),
        "tn_fc1": tn_case(384, 192, True, True),
        "tn_fc2": tn_case(192, 384, True, True),
        "tn_qkv_f32": tn_case(576, 192, False, False),
        "tn_proj_f32": tn_case(192, 192, False, False),
        "nt_conv_fwd": nt_conv(),
        "tn_conv_tap": tn_case(192, 1728, False, False, conv=True),
        "attn_fwd": attn_case(False),
        "attn_bwd": attn_case(True),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("filter", nargs="?", default="")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    tot = 0.0
    for name, (run, fl, nb) in cases().items():
        if a.filter not in name:
            continue
        us = timeit(run, a.reps)
        tot += us
        tf = fl / (us * 1e-6) / 1e12
        print(f"{name:16s} {us:8.1f} us  {tf:7.1f} TFLOP/s issued  {tf / PEAK_F16:6.3f} of fp16 MFMA  "
              f"{nb / (us * 1e-6) / 1e9:7.0f} GB/s alg")
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
