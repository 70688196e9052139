"""Isolated launch times of the per-block kernels at small per-GPU batches (B = 4 is M = 9216 rows):
fused MLP forward, the four row GEMMs.  Rows are varied around 256 tiles of 32 to show the cost of
the second-tile tail vs the per-tile chain.  python tools/b4_micro.py"""
import sys
import torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
from kair_amd import _hip as H
import test_mlp_fused_gpu as TM
dev = torch.device("cuda", 0)
C, CP, HD, HDP = 180, 192, 360, 384


def timeit(f, reps=50):
    for _ in range(5):
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


Mmax = 73728
x = torch.randn(Mmax, CP, device=dev); x[:, C:] = 0
gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
W1 = TM._pack(0.05 * torch.randn(HD, C, device=dev), 10, (1, HD, HDP), (1, C, CP))
W2 = TM._pack(0.05 * torch.randn(C, HD, device=dev), 14, (1, C, CP), (1, HD, HDP))
b1, b2 = torch.zeros(HDP, device=dev), torch.zeros(CP, device=dev)
ln = torch.empty(Mmax, CP, device=dev, dtype=torch.bfloat16)
mean, rstd = torch.empty(Mmax, device=dev), torch.empty(Mmax, device=dev)
u = torch.empty(Mmax, HDP, device=dev, dtype=torch.bfloat16); h = torch.empty_like(u)
out = torch.empty(Mmax, CP, device=dev)
Wt = {K: torch.randn(K * (384 if K == 192 else 192), device=dev).to(torch.bfloat16) for K in (192, 384, 576)}
A = torch.randn(Mmax, 576, device=dev).to(torch.bfloat16)
gate = torch.rand(Mmax, 384, device=dev).to(torch.bfloat16)
o384 = torch.empty(Mmax, 384, device=dev, dtype=torch.bfloat16)
o192 = torch.empty(Mmax, 192, device=dev, dtype=torch.bfloat16)
D = torch.zeros(Mmax, CP, device=dev)
part = torch.empty(4096 * 2 * C, device=dev)
print("%8s %8s %8s %8s %8s %8s %8s" % ("M", "tiles", "mlp", "gate", "fc1ln", "qkvln", "proj"))
for M in (4096, 8192, 9216, 16384, 73728):
    t_mlp = timeit(lambda: H.swin_mlp_fwd(x, CP, gamma, beta, 1e-5, C, ln, CP, mean, rstd, W1, b1, u, h, HDP, HD, W2, b2,
                                          None, 0, out, CP, M, CP, HDP))
    t_gate = timeit(lambda: H.rowgemm_gate(A[:M, :192], M, 192, Wt[192], 384, gate[:M], o384[:M]))
    t_fc1 = timeit(lambda: H.rowgemm_lnbwd(A[:M, :384], M, 384, Wt[384], x[:M], gamma, mean, rstd, C, D[:M], part))
    t_qkv = timeit(lambda: H.rowgemm_lnbwd(A[:M], M, 576, Wt[576], x[:M], gamma, mean, rstd, C, D[:M], part))
    t_proj = timeit(lambda: H.rowgemm_store(A[:M, :192], M, 192, Wt[192][:192 * 192], 192, o192[:M]))
    print("%8d %8d %8.1f %8.1f %8.1f %8.1f %8.1f" % (M, M // 32, t_mlp, t_gate, t_fc1, t_qkv, t_proj))
