"""Micro-benchmark of the libkair_hip GEMMs at the SwinIR classical x4 (B=32) shapes.

    python tools/gemm_micro.py [substring] [--no-torch] [--reps R]     (on the GPU box)

Times each kernel with HIP events over R launches and prints us / TFLOP/s / algorithmic GB/s;
torch.matmul (hipBLASLt) on the same plain shapes is printed beside it purely as a yardstick (it is
never used by kair_amd).  KAIR_GEMM_STREAM=0 selects the tiled NT kernel for A/B comparisons.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
B_, HH, WW, CP = 32, 48, 48, 192
M = B_ * HH * WW


def timeit(fn, reps):
    """Average us per launch of `reps` launches captured in one HIP graph (host launch cost of the
    Python wrappers excluded, as in the graph-replayed training step)."""
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin()
        for _ in range(reps):
            fn()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def nbytes(*ts):
    return sum(t.numel() * t.element_size() for t in ts)


def cases():
    """name -> (launch, torch yardstick or None, flops, algorithmic bytes)"""
    out = {}
    for name, N, K, mode in [("qkv_fwd", 576, 192, H.OUT_QKVBLK), ("proj_fwd", 192, 192, H.OUT_ROWS),
                             ("fc1_fwd", 384, 192, H.OUT_ROWS), ("fc2_fwd", 192, 384, H.OUT_ROWS)]:
        A = torch.randn(M, K, device=dev).to(bf)
        W = torch.randn(N, K, device=dev).to(bf) * 0.05
        o = torch.empty(M * N, device=dev, dtype=bf)
        ep = H.epilogue(o.view(M, N), mode=mode, ldo=0 if mode == H.OUT_QKVBLK else N, qkv=(6, 32, 64))
        out[name] = (lambda A=A, W=W, ep=ep, N=N, K=K: H.gemm_nt(H.rows(A), H.rows(W), ep, M, N, K, H.BF16),
                     lambda A=A, W=W: torch.matmul(A, W.T), 2.0 * M * N * K, nbytes(A, W, o))
    A = torch.randn(M, 192, device=dev).to(bf)
    W = torch.randn(384, 192, device=dev).to(bf) * 0.05
    o = torch.empty(M, 384, device=dev, dtype=bf)
    pre = torch.empty(M, 384, device=dev, dtype=bf)
    bias = torch.randn(384, device=dev)
    out["fc1_fwd_gelu_pre"] = (lambda: H.gemm_nt(H.rows(A), H.rows(W), H.epilogue(o, bias=bias, act=H.ACT_GELU, pre=pre),
                                                 M, 384, 192, H.BF16), None, 2.0 * M * 384 * 192, nbytes(A, W, o, pre))
    D = torch.randn(M, 192, device=dev)
    gate = torch.randn(M, 384, device=dev).to(bf)
    o2 = torch.empty(M, 384, device=dev, dtype=bf)
    out["fc2_dgrad_f32A_gate"] = (lambda: H.gemm_nt(H.rows(D), H.rows(W), H.epilogue(o2, gate=gate, gate_kind=1),
                                                    M, 384, 192, H.BF16), None, 2.0 * M * 384 * 192,
                                  nbytes(D, W, gate, o2))
    R = torch.randn(M, 192, device=dev)
    W3 = torch.randn(192, 192, device=dev).to(bf) * 0.05
    o3 = torch.empty(M, 192, device=dev)
    out["f32A_resid_192"] = (lambda: H.gemm_nt(H.rows(D), H.rows(W3), H.epilogue(o3, resid=R), M, 192, 192, H.BF16),
                             None, 2.0 * M * 192 * 192, nbytes(D, W3, R, o3))
    Db = torch.randn(M, 192, device=dev).to(bf)
    o4 = torch.empty(M, 384, device=dev, dtype=bf)
    out["fc2_dgrad_gate"] = (lambda: H.gemm_nt(H.rows(Db), H.rows(W), H.epilogue(o4, gate=gate, gate_kind=1),
                                               M, 384, 192, H.BF16), None, 2.0 * M * 384 * 192, nbytes(Db, W, gate, o4))
    sc = torch.rand(B_, device=dev) + 0.5
    o5 = torch.empty(M, 192, device=dev)
    out["proj_fwd_full"] = (lambda: H.gemm_nt(H.rows(Db), H.rows(W3), H.epilogue(o5, win=(HH, WW, 8, 4), resid=R, rowscale=sc,
                                                                                rows_per_scale=HH * WW), M, 192, 192, H.BF16),
                            None, 2.0 * M * 192 * 192, nbytes(Db, W3, R, o5))
    x = torch.randn(M, CP, device=dev)
    Wc = torch.randn(CP, 9 * CP, device=dev).to(bf) * 0.02
    oc = torch.empty(M, CP, device=dev)
    xb = torch.randn(B_, CP, HH, WW, device=dev, dtype=bf)
    wb = torch.randn(CP, CP, 3, 3, device=dev, dtype=bf)
    out["conv3x3_fwd"] = (lambda: H.gemm_nt(H.im2col(x, HH, WW, CP), H.rows(Wc), H.epilogue(oc), M, CP, 9 * CP, H.BF16),
                          lambda: torch.nn.functional.conv2d(xb, wb, padding=1), 2.0 * M * CP * 9 * CP,
                          nbytes(x, Wc, oc))
    for name, N, K in [("fc1_wgrad", 384, 192), ("qkv_wgrad", 576, 192), ("proj_wgrad", 192, 192), ("fc2_wgrad", 192, 384)]:
        G = torch.randn(M, N, device=dev).to(bf)
        X = torch.randn(M, K, device=dev).to(bf)
        X[:, K - 1] = 1.0
        S = H.wgrad_splits(M, N, K)
        ws = torch.empty(S, N, K, device=dev)
        out[name + f"(S={S})"] = (lambda G=G, X=X, ws=ws, S=S, N=N, K=K:
                                  H.gemm_tn(H.rows(G), H.rows(X, ones_col=K - 1, ones_in_data=True), ws, S, M, N, K, H.BF16),
                                  lambda G=G, X=X: torch.matmul(G.T, X), 2.0 * M * N * K, nbytes(G, X, ws))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("only", nargs="?", default=None)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    print(f"{'kernel':22s} {'kair us':>9s} {'TF/s':>7s} {'GB/s':>7s} {'torch us':>9s} {'TF/s':>7s}")
    for name, (fn, ref, fl, by) in cases().items():
        if a.only and a.only not in name:
            continue
        us = timeit(fn, a.reps)
        rus = timeit(ref, a.reps) if (ref is not None and not a.no_torch) else float("nan")
        print(f"{name:22s} {us:9.1f} {fl / us / 1e6:7.1f} {by / us / 1e3:7.0f} {rus:9.1f} {fl / rus / 1e6:7.1f}")


if __name__ == "__main__":
    main()
