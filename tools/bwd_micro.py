"""Micro-timings of the Swin block backward launches at B=32 (block 0 operands after one real
forward + backward), HIP-event timed; variants isolate epilogue ALU cost (GELU' gate vs a plain
ReLU-style gate) and ring-kernel ablations (KAIR_RING_DBG set by the caller).

    python tools/bwd_micro.py [B] [reps]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402
from kair_amd.models.network_swinir import SwinIR  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1000.0, 2)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda")
    torch.manual_seed(0)
    net = SwinIR(upscale=4, in_chans=3, img_size=48, window_size=8, img_range=1.0, depths=[2], embed_dim=180,
                 num_heads=[6], mlp_ratio=2, upsampler="pixelshuffle", drop_path_rate=0.1).to(dev).train()
    eng = net.engine()
    x = torch.rand(B, 3, 48, 48, device=dev)
    D = torch.ones(len(eng.blocks), 2, B, device=dev)
    eng.forward(x, D)
    P = eng.cur
    params = list(net.parameters())
    grads = {p: torch.zeros_like(p) for p in params}
    eng.backward_from_grad(torch.randn(B, 3, 192, 192, device=dev), grads)
    blk, S = eng.blocks[0], P["blocks"][0]
    M, Cp, Hdp, nh, cd = P["M"], eng.Cp, eng.Hdp, eng.nh, eng.cd
    Dc = P["Dc"]
    out = {"B": B, "dbg": os.environ.get("KAIR_RING_DBG", "0")}
    fc2, fc1, proj, qkv = blk.fc2, blk.fc1, blk.proj, blk.qkv
    out["fc2_dgrad_gelu_gate"] = timeit(lambda: H.gemm_nt(H.rows(Dc), H.rows(fc2.Wt), H.epilogue(P["dU"], gate=S["u"], gate_kind=1),
                                                          M, Hdp, Cp, cd), reps)
    out["fc2_dgrad_mul_gate"] = timeit(lambda: H.gemm_nt(H.rows(Dc), H.rows(fc2.Wt), H.epilogue(P["dU"], gate=S["u"], gate_kind=4),
                                                         M, Hdp, Cp, cd), reps)
    out["fc2_dgrad_relu_gate"] = timeit(lambda: H.gemm_nt(H.rows(Dc), H.rows(fc2.Wt), H.epilogue(P["dU"], gate=S["u"], gate_kind=0),
                                                          M, Hdp, Cp, cd), reps)
    out["fc2_dgrad_no_gate"] = timeit(lambda: H.gemm_nt(H.rows(Dc), H.rows(fc2.Wt), H.epilogue(P["dU"]), M, Hdp, Cp, cd), reps)
    out["fc1_dgrad"] = timeit(lambda: H.gemm_nt(H.rows(P["dU"]), H.rows(fc1.Wt), H.epilogue(P["dxn"]), M, Cp, Hdp, cd), reps)
    out["proj_dgrad"] = timeit(lambda: H.gemm_nt(H.rows(Dc), H.rows(proj.Wt), H.epilogue(P["dO"]), M, nh * 32, Cp, cd), reps)
    out["qkv_dgrad"] = timeit(lambda: H.gemm_nt(H.qkvblk(P["dqkv"], nh), H.rows(qkv.Wt), H.epilogue(P["dxn"]), M, Cp, qkv.Np, cd),
                              reps)
    out["attn_bwd"] = timeit(lambda: H.window_attn_bwd(S["qkv"], S["O"], nh * 32, P["dO"], nh * 32, blk.table, S["lse"], P["dqkv"],
                                                       grads[blk.table], False, P["attn_ws"], P["nWin"], nh, eng.C // nh,
                                                       blk.scale, 48, 48, blk.shift), reps)
    n = blk.n2
    out["ln_bwd"] = timeit(lambda: H.layernorm_bwd(S["mid"], Cp, P["dxn"], Cp, n.weight, S["m2"], S["r2"], P["D"], Cp, True,
                                                   grads[n.weight], grads[n.bias], False, P["ln_ws"], M, eng.C,
                                                   copy=H.copy_desc(Dc, rowscale=None, rows_per_scale=48 * 48,
                                                                    win=(48, 48, 8, 0))), reps)
    g = lambda p: grads[p]
    out["fc2_wgrad+fin"] = timeit(lambda: eng._wgrad(P, H.rows(Dc), H.rows(S["h"], ones_col=fc2.K, ones_in_data=True), M, Cp,
                                                     Hdp, fc2.map, g(fc2.w), g(fc2.b), fc2.K), reps)
    out["wgrad_splits_fc2"] = H.wgrad_splits(M, Cp, Hdp)
    out["qkv_wgrad+fin"] = timeit(lambda: eng._wgrad(P, H.qkvblk(P["dqkv"], nh), H.rows(S["ln1"], ones_col=eng.C, ones_in_data=True),
                                                     M, qkv.Np, Cp, qkv.map, g(qkv.w), g(qkv.b), eng.C), reps)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
