"""Fused MLP-half backward (kair_swin_mlp_bwd) vs the launches it replaces (fc2 / fc1 input
gradients + LayerNorm-2 backward), block 0 of the classical x4 network at batch B, HIP-event timed.

    python tools/mlpbwd_micro.py [B] [reps]
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
    grads = {p: torch.zeros_like(p) for p in net.parameters()}
    eng.backward_from_grad(torch.randn(B, 3, 192, 192, device=dev), grads)
    blk, S = eng.blocks[0], P["blocks"][0]
    M, Cp, Hdp, cd = P["M"], eng.Cp, eng.Hdp, eng.cd
    fc2, fc1, n = blk.fc2, blk.fc1, blk.n2
    Dc, Dg = P["Dc"], P["D"]
    out = {"B": B, "dbg": os.environ.get("KAIR_MLPB_DBG", "0")}
    if eng.fused_mlp_bwd:
        out["fused_mlp_bwd_us"] = timeit(lambda: H.swin_mlp_bwd(
            Dc, S["u"], fc2.Wgt, fc1.Wgt, P["dU"], S["mid"], n.weight, S["m2"], S["r2"], eng.C, Dg, P["Dc2"], D[0, 0],
            48 * 48, 48, 48, 0, grads[n.weight], grads[n.bias], P["mlp_ws"], M, Cp, Hdp), reps)

    def unfused():
        H.gemm_nt(H.rows(Dc), H.rows(fc2.Wt), H.epilogue(P["dU"], gate=S["u"], gate_kind=4), M, Hdp, Cp, cd)
        H.gemm_nt(H.rows(P["dU"]), H.rows(fc1.Wt), H.epilogue(P["dxn"]), M, Cp, Hdp, cd)
        H.layernorm_bwd(S["mid"], Cp, P["dxn"], Cp, n.weight, S["m2"], S["r2"], Dg, Cp, True, grads[n.weight],
                        grads[n.bias], False, P["ln_ws"], M, eng.C,
                        copy=H.copy_desc(P["Dc2"], rowscale=D[0, 0], rows_per_scale=48 * 48, win=(48, 48, 8, 0)))
    out["unfused_us"] = timeit(unfused, reps)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
