"""Micro-benchmark of the libkair_hip GEMMs at the SwinIR classical x4 (B=32) shapes.

    python tools/gemm_micro.py            (on the GPU box)

Times each kernel with HIP events over R launches and prints us / TFLOP/s; torch.matmul (hipBLASLt)
on the same plain shapes is printed beside it purely as a yardstick (it is never used by kair_amd).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402

dev = torch.device("cuda")


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    B, Hh, Ww, Cp = 32, 48, 48, 192
    M = B * Hh * Ww
    bf = torch.bfloat16
    res = []
    a = torch.randn(M, Cp, device=dev).to(bf)
    for name, N, K, mode in [("qkv_fwd", 576, 192, H.OUT_QKVBLK), ("proj_fwd", 192, 192, H.OUT_ROWS),
                             ("fc1_fwd", 384, 192, H.OUT_ROWS), ("fc2_fwd", 192, 384, H.OUT_ROWS)]:
        A = torch.randn(M, K, device=dev).to(bf)
        W = torch.randn(N, K, device=dev).to(bf) * 0.05
        out = torch.empty(M * N, device=dev, dtype=bf)
        ep = H.epilogue(out.view(M, N), mode=mode, ldo=0 if mode == H.OUT_QKVBLK else N, qkv=(6, 32, 64))
        us = timeit(lambda: H.gemm_nt(H.rows(A), H.rows(W), ep, M, N, K, H.BF16))
        ref = timeit(lambda: torch.matmul(A, W.T))
        fl = 2.0 * M * N * K
        res.append((name, us, fl / us / 1e6, ref, fl / ref / 1e6))
    # conv 3x3 180->180 (fp32 residual-stream input)
    x = torch.randn(M, Cp, device=dev)
    Wc = torch.randn(Cp, 9 * Cp, device=dev).to(bf) * 0.02
    oc = torch.empty(M, Cp, device=dev)
    us = timeit(lambda: H.gemm_nt(H.im2col(x, Hh, Ww, Cp), H.rows(Wc), H.epilogue(oc), M, Cp, 9 * Cp, H.BF16))
    fl = 2.0 * M * Cp * 9 * Cp
    xb = torch.randn(B, Cp, Hh, Ww, device=dev, dtype=bf)
    wb = torch.randn(Cp, Cp, 3, 3, device=dev, dtype=bf)
    ref = timeit(lambda: torch.nn.functional.conv2d(xb, wb, padding=1))
    res.append(("conv3x3_fwd", us, fl / us / 1e6, ref, fl / ref / 1e6))
    # wgrad (TN)
    for name, N, K in [("fc1_wgrad", 384, 192), ("qkv_wgrad", 576, 192)]:
        G = torch.randn(M, N, device=dev).to(bf)
        X = torch.randn(M, K, device=dev).to(bf)
        S = H.wgrad_splits(M, N, K)
        ws = torch.empty(S, N, K, device=dev)
        us = timeit(lambda: H.gemm_tn(H.rows(G), H.rows(X, ones_col=K - 1), ws, S, M, N, K, H.BF16))
        ref = timeit(lambda: torch.matmul(G.T, X))
        fl = 2.0 * M * N * K
        res.append((name + f"(S={S})", us, fl / us / 1e6, ref, fl / ref / 1e6))
    print(f"{'kernel':22s} {'kair us':>9s} {'TF/s':>7s} {'torch us':>9s} {'TF/s':>7s}")
    for r in res:
        print(f"{r[0]:22s} {r[1]:9.1f} {r[2]:7.1f} {r[3]:9.1f} {r[4]:7.1f}")


if __name__ == "__main__":
    main()
