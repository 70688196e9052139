"""Micro-benchmark of the Swin-block attention half: the fused kernel (kair_swin_attn_fwd) against
the four launches it replaces (LayerNorm, QKV GEMM, window attention, proj GEMM), one block of the
classical x4 network at per-GPU batch B, HIP-event timed on the current stream.

    python tools/fused_micro.py [B] [reps]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402
from kair_amd.models.network_swinir import SwinIR  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda")
    torch.manual_seed(0)
    split = os.environ.get("KAIR_SPLIT", "1") == "1"
    net = SwinIR(upscale=4, in_chans=3, img_size=48, window_size=8, img_range=1.0, depths=[2], embed_dim=180,
                 num_heads=[6], mlp_ratio=2, upsampler="pixelshuffle", drop_path_rate=0.1,
                 split_conv=split).to(dev).train()
    eng = net.engine()
    x = torch.rand(B, 3, 48, 48, device=dev)
    D = torch.ones(len(eng.blocks), 2, B, device=dev)
    eng.forward(x, D)
    P = eng.cur
    out = {}
    for bi in (0, 1):
        blk, S = eng.blocks[bi], P["blocks"][bi]
        xin = P["s0"]
        res = {}
        for fused in (True, False):
            eng.fused_attn = fused
            eng.fused_mlp = fused and blk.fc1.Wg is not None
            run = lambda: eng._block_fwd(blk, P, S, xin, bi)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            res["fused" if fused else "unfused"] = e0.elapsed_time(e1) / reps * 1000.0
        out[f"block{bi}_shift{blk.shift}"] = res
    # the attention half alone: fused kernel by itself
    eng.fused_attn = True
    blk, S = eng.blocks[0], P["blocks"][0]
    Cp, nh = eng.Cp, eng.nh
    HW = 48 * 48

    def attn_only():
        H.swin_attn_fwd(P["s0"], Cp, blk.n1.weight, blk.n1.bias, blk.n1.eps, eng.C, S["ln1"], Cp, S["m1"], S["r1"],
                        blk.qkv.Wg, blk.qkv.bp, S["qkv"], blk.table, blk.scale, S["O"], nh * 32, eng.C // nh, S["lse"],
                        blk.proj.Wg, blk.proj.bp, D[0, 0], HW, S["mid"], Cp, P["nWin"], nh, 48, 48, 0, w_split=blk.qkv.split)
    for _ in range(3):
        attn_only()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        attn_only()
    e1.record()
    torch.cuda.synchronize()
    out["fused_attn_kernel_us"] = e0.elapsed_time(e1) / reps * 1000.0

    def mlp_only():
        f1, f2 = blk.fc1, blk.fc2
        H.swin_mlp_fwd(S["mid"], Cp, blk.n2.weight, blk.n2.bias, blk.n2.eps, eng.C, S["ln2"], Cp, S["m2"], S["r2"],
                       f1.Wg, f1.bp, S["u"], S["h"], eng.Hdp, f1.N, f2.Wg, f2.bp, D[0, 1], HW, S["out"], Cp, P["M"], Cp,
                       eng.Hdp, w_split=f1.split)
    if blk.fc1.Wg is not None:   # the MLP-half kernel is packed only when enabled (KAIR_FUSED_MLP=1)
        for _ in range(3):
            mlp_only()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            mlp_only()
        e1.record()
        torch.cuda.synchronize()
        out["fused_mlp_kernel_us"] = e0.elapsed_time(e1) / reps * 1000.0
    out["split"] = bool(blk.qkv.split)
    out["B"] = B
    print(json.dumps(out))


if __name__ == "__main__":
    main()
