"""B=4 (M = 9216 tokens) block input-gradient GEMMs: libkair_hip vs torch.matmul (hipBLASLt, a
yardstick only) in graph-captured loops -- where the 16 us per launch of the register-staged NT
kernel goes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for M in (9216, 73728):
    for N, K, gate in ((384, 192, True), (192, 384, False), (192, 192, False)):
        A = torch.randn(M, K, device=dev).to(bf)
        W = torch.randn(N, K, device=dev).to(bf)
        out = torch.empty(M, N, device=dev, dtype=bf)
        G = torch.randn(M, N, device=dev).to(bf)
        ep = H.epilogue(out, gate=G, gate_kind=4) if gate else H.epilogue(out)
        t = timeit(lambda: H.gemm_nt(H.rows(A), H.rows(W), ep, M, N, K, H.BF16))
        tt = timeit(lambda: torch.matmul(A, W.t(), out=out))
        z = torch.empty(1, device=dev)
        t0 = timeit(lambda: z.add_(1.0))
        by = (M * K + N * K + M * N * (2 if gate else 1)) * 2
        print(f"M {M} N {N} K {K} gate {gate}: kair {t:7.1f} us ({by / t / 1e3:6.0f} GB/s)  "
              f"torch.matmul {tt:7.1f} us  tiny-kernel floor {t0:5.1f} us", flush=True)
