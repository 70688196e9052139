"""PSNR deviation of bf16 engine variants from the fp32 engine on the same trained weights, over
several training realizations (seeds): how much of the bench's psnr.bf16_delta_db is weight
rounding (removed by hi/lo split weights) and how much is activation rounding.

    python tools/parity_seeds.py [n_seeds] [steps]
Prints one JSON line per (seed, variant): float / uint8-border-4 PSNR deltas on the bench's one
evaluation patch (seed 7) and the mean per-image delta over 8 held-out patches.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import build_net  # noqa: E402
from kair_amd.engine.swinir_engine import SwinIREngine  # noqa: E402
from kair_amd.engine.trainer import FusedTrainer  # noqa: E402
from kair_amd.utils import utils_image as U  # noqa: E402

VARIANTS = {
    "split_conv_only": dict(split_linear=False, fused_mlp=False),
    "split_conv+attn_linears": dict(split_linear=True, fused_mlp=False),
    "split_all(fused mlp)": dict(split_linear=True, fused_mlp=True),
    "no_split": dict(split_conv=False, split_linear=False, fused_mlp=False),
}


def main():
    n_seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    dev = torch.device("cuda", 0)
    L1, H1 = U.synth_sr_batch(1, 48, 4, seed=7)
    L8, H8 = U.synth_sr_batch(8, 48, 4, seed=77)
    for seed in range(n_seeds):
        net = build_net("bf16", 0.1, seed=seed).to(dev).train()
        ema = build_net("bf16", 0.1, seed=seed).to(dev).eval()
        ema.load_state_dict(net.state_dict())
        tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999)
        L, Hh = U.synth_sr_batch(32, 48, 4, seed=1000 + seed, device=dev)
        for _ in range(steps):
            tr.step(L, Hh)
        torch.cuda.synchronize()
        sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
        del tr, net, ema

        def run(dtype, kw):
            n = build_net(dtype, 0.0).to(dev).eval()
            n.load_state_dict(sd, strict=True)
            if kw is not None:
                n._engine = SwinIREngine(n, dtype, **{"split_conv": True, "fused_blocks": True, **kw})
            with torch.no_grad():
                return n(L1.to(dev)).float().cpu(), n(L8.to(dev)).float().cpu()

        E1r, E8r = run("fp32", None)

        def metrics(E1, E8):
            d1 = U.psnr_float(E1, H1) - U.psnr_float(E1r, H1)
            u1 = (U.calculate_psnr(U.tensor2uint(E1), U.tensor2uint(H1), border=4) -
                  U.calculate_psnr(U.tensor2uint(E1r), U.tensor2uint(H1), border=4))
            d8 = sum(U.psnr_float(E8[i:i + 1], H8[i:i + 1]) - U.psnr_float(E8r[i:i + 1], H8[i:i + 1]) for i in range(8)) / 8
            u8 = sum(U.calculate_psnr(U.tensor2uint(E8[i]), U.tensor2uint(H8[i]), border=4) -
                     U.calculate_psnr(U.tensor2uint(E8r[i]), U.tensor2uint(H8[i]), border=4) for i in range(8)) / 8
            return {"d1": round(d1, 6), "u1": round(u1, 6), "d8": round(d8, 6), "u8": round(u8, 6)}

        for name, kw in VARIANTS.items():
            print(json.dumps({"seed": seed, "variant": name, **metrics(*run("bf16", kw))}), flush=True)


if __name__ == "__main__":
    main()
