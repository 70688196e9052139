"""Attribute the bf16 engine's PSNR deviation (bench.py psnr leg) to weight rounding vs activation
rounding, layer group by layer group.

Trains the bench network (bf16, drop_path 0.1) for --steps fused steps, then evaluates on the bench's
PSNR batch:  the fp32 engine on the exact weights (reference, = oracle to 1e-7 dB), the bf16 engine,
and the fp32 engine with the weights of one group rounded to bf16 (what the bf16 engine's packed
GEMM weights are).  Prints one JSON line per variant.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import build_net  # noqa: E402
from kair_amd.engine.trainer import FusedTrainer  # noqa: E402
from kair_amd.utils import utils_image as U  # noqa: E402


def groups(net):
    tail = ["conv_after_body", "conv_before_upsample", "upsample", "conv_last"]
    g = {"all": lambda k: True,
         "tail": lambda k: any(k.startswith(t) for t in tail),
         "conv_last": lambda k: k.startswith("conv_last"),
         "upsample": lambda k: k.startswith("upsample"),
         "cbu+cab": lambda k: k.startswith("conv_before_upsample") or k.startswith("conv_after_body"),
         "body_linear": lambda k: k.startswith("layers") and (".qkv." in k or ".proj." in k or ".fc1." in k or ".fc2." in k),
         "body_conv": lambda k: k.startswith("layers") and ".conv." in k,
         "conv_first": lambda k: k.startswith("conv_first")}
    return g


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 25
    dev = torch.device("cuda", 0)
    net = build_net("bf16", 0.1).to(dev).train()
    ema = build_net("bf16", 0.1).to(dev).eval()
    ema.load_state_dict(net.state_dict())
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999)
    L, Hh = U.synth_sr_batch(32, 48, 4, seed=1000, device=dev)
    for _ in range(steps):
        tr.step(L, Hh)
    torch.cuda.synchronize()
    sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
    Le, He = U.synth_sr_batch(1, 48, 4, seed=7)
    hu = U.tensor2uint(He)

    def run(dtype, state, split=True):
        n = build_net(dtype, 0.0)
        n.split_conv = split
        n = n.to(dev).eval()
        n.load_state_dict(state, strict=True)
        with torch.no_grad():
            E = n(Le.to(dev)).float().cpu()
        return E

    E32 = run("fp32", sd)
    p32 = U.psnr_float(E32, He)
    u32 = U.calculate_psnr(U.tensor2uint(E32), hu, border=4)

    def report(name, E):
        pf = U.psnr_float(E, He)
        uf = U.calculate_psnr(U.tensor2uint(E), hu, border=4)
        d = (E - E32)
        print(json.dumps({"variant": name, "d_db": round(pf - p32, 6), "d_u8_db": round(uf - u32, 6),
                          "max_abs": float(d.abs().max()), "rms": float(d.pow(2).mean().sqrt()),
                          "mean": [round(float(d[:, c].mean()), 7) for c in range(3)]}), flush=True)

    report("bf16_engine(split conv)", run("bf16", sd))

    # body / tail attribution: run both engines, then swap P['fb'] and re-run one tail
    def engine_of(dtype, fused=True):
        n = build_net(dtype, 0.0)
        n.fused_blocks = fused
        n = n.to(dev).eval()
        n.load_state_dict(sd, strict=True)
        return n, n.engine()
    x = Le.to(dev)
    with torch.no_grad():
        n32, e32 = engine_of("fp32")
        n16, e16 = engine_of("bf16")
        e32.forward(x)
        P32 = e32.cur
        fb32 = P32["fb"].clone()
        e16.forward(x)
        P16 = e16.cur
        fb16 = P16["fb"].clone()
        P16["fb"].copy_(fb32)
        report("bf16 tail on fp32 body", e16._forward_tail(P16).float().cpu())
        P32["fb"].copy_(fb16)
        report("fp32 tail on bf16 body", e32._forward_tail(P32).float().cpu())
        print(json.dumps({"fb_rel_rms(bf16 body)": float((fb16 - fb32).pow(2).mean().sqrt() / fb32.pow(2).mean().sqrt())}))
        nu, eu = engine_of("bf16", fused=False)
        report("bf16_engine(unfused blocks)", nu(x).float().cpu())
    report("bf16_engine(no split)", run("bf16", sd, split=False))
    for name, sel in groups(net).items():
        st = {k: (v.to(torch.bfloat16).float() if (sel(k) and k.endswith("weight") and v.dim() >= 2) else v)
              for k, v in sd.items()}
        report("fp32_w_bf16:" + name, run("fp32", st))
    print(json.dumps({"ref_psnr": p32, "ref_u8": u32}))


if __name__ == "__main__":
    main()
