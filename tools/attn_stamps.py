"""Phase timing of the bf16 attention backward (KAIR_ATTN_STAMP=1): median cycles per phase of one
window per wave, over all waves, at B=32.

    python tools/attn_stamps.py [B]
"""
import json
import os
import sys

os.environ["KAIR_ATTN_STAMP"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402
from kair_amd.models.network_swinir import SwinIR  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    dev = torch.device("cuda")
    torch.manual_seed(0)
    net = SwinIR(upscale=4, in_chans=3, img_size=48, window_size=8, img_range=1.0, depths=[2], embed_dim=180,
                 num_heads=[6], mlp_ratio=2, upsampler="pixelshuffle", drop_path_rate=0.1, compute_dtype="bf16").to(dev).train()
    eng = net.engine()
    x = torch.rand(B, 3, 48, 48, device=dev)
    eng.forward(x, torch.ones(len(eng.blocks), 2, B, device=dev))
    P = eng.cur
    grads = {p: torch.zeros_like(p) for p in net.parameters()}
    eng.backward_from_grad(torch.randn(B, 3, 192, 192, device=dev), grads)
    blk, S = eng.blocks[1], P["blocks"][1]
    nh = eng.nh
    for _ in range(2):
        H.window_attn_bwd(S["qkv"], S["O"], nh * 32, P["dO"], nh * 32, blk.table, S["lse"], P["dqkv"], grads[blk.table],
                          False, P["attn_ws"], P["nWin"], nh, eng.C // nh, blk.scale, 48, 48, blk.shift)
    torch.cuda.synchronize()
    a = np.array(H.debug_attn_stamps(), dtype=np.uint64).reshape(-1, 8).astype(np.int64)
    a = a[a[:, 0] > 0]
    d = np.diff(a[:, :7], axis=1)
    names = ["lds_writes+delta", "S,dP mfma+next loads", "P,dS elementwise", "dV,dK mfma+stores", "dS to LDS", "dQ mfma+stores"]
    out = {"waves": int(len(a)), "windows_per_wave": int(np.median(a[:, 7])),
           "phase_cycles_median": {k: float(np.median(d[:, i])) for i, k in enumerate(names)},
           "window_total_median": float(np.median(a[:, 6] - a[:, 0])),
           "window_total_p90": float(np.percentile(a[:, 6] - a[:, 0], 90))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
