"""Ring-GEMM cost model sweep: us per launch vs M-tiles per CTA (graph-captured, 50 launches), for
the proj (N=K=192) and fc1 (N=384, K=192) shapes.  Run under KAIR_RING_DBG=<bits> for ablations.

    python tools/ring_sweep.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402
from tools.gemm_micro import timeit  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
for name, N, K in [("proj", 192, 192), ("fc1", 384, 192), ("fc2", 192, 384)]:
    for tpc in [1, 2, 3, 6, 12]:
        tilesN = (N + 191) // 192 if K <= 192 else (N + 95) // 96
        M = 128 * tpc * (256 // tilesN)
        A = torch.randn(M, K, device=dev).to(bf)
        W = torch.randn(N, K, device=dev).to(bf) * 0.05
        o = torch.empty(M, N, device=dev, dtype=bf)
        ep = H.epilogue(o)
        us = timeit(lambda: H.gemm_nt(H.rows(A), H.rows(W), ep, M, N, K, H.BF16), 50)
        gb = (A.numel() + o.numel()) * 2 / us / 1e3
        print(f"{name:5s} tiles/CTA {tpc:3d}  M {M:7d}  {us:8.2f} us  {gb:7.0f} GB/s", flush=True)
