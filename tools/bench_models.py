"""Training throughput of the other BASELINE.json configs on one MI355X (the headline SwinIR
classical x4 line is bench.py's).  One JSON line per config:

    python tools/bench_models.py [dncnn|swinir_light|rrdbnet|usrnet ...] [--steps K] [--warmup W]

C1 DnCNN sigma 25, 40x40, batch 64 (BN, fused trainer)        network_dncnn.py, options/train_dncnn.json
C2 SwinIR-lightweight x2, 64-px LQ, batch 64 (fused trainer)   options/swinir/train_swinir_sr_lightweight.json
C5 RRDBNet x4, 32-px LQ, batch 16 (fused trainer)              options/train_rrdb_psnr.json
C3 USRNet x4, 128-px LQ (512^2 HR), batch 48, n_iter 6         options/train_usrnet.json (ModelPlain4 step:
                                                                fused trainer with (k, sf, sigma) inputs, no EMA)
Synthetic seeded inputs resident in HBM; bf16 MFMA operands, fp32 accumulation.
FLOP/patch from BASELINE.md (FlopCounterMode, GEMM + conv only; USRNet FFTs not counted).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_BF16_TFLOPS = 2500.0
TRAIN_GFLOP = {"dncnn": 5.32, "swinir_light": 25.68, "rrdbnet": 110.14, "usrnet": 577.25}


def timed(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, out


def run(name, steps, warmup, dev, dtype="bf16", head_pad=None, grouped_wgrad=None, side_ctas=None):
    """dtype: the engine's compute dtype -- "bf16" (bf16 MFMA, fp32 accumulation), "fp32" (exact fp32 MFMA: the
    reference's arithmetic for the fp32 option files, C3 / C5) or "fp32x3" where the engine has it.
    head_pad (SwinIR): the engine's q/k/v head pad (None: its choice -- 16 for C2's head dim 10; 32: A/B)."""
    from kair_amd.engine.trainer import FusedTrainer
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(1)
    if name == "dncnn":
        from kair_amd.models.network_dncnn import DnCNN
        mk = lambda: DnCNN(1, 1, 64, 17, "BR", compute_dtype=dtype)   # noqa: E731
        B, shp, sc = 64, (1, 40, 40), 1
    elif name == "swinir_light":
        from kair_amd.models.network_swinir import SwinIR
        mk = lambda: SwinIR(upscale=2, in_chans=3, img_size=64, window_size=8, img_range=1.0, depths=[6] * 4,   # noqa: E731
                            embed_dim=60, num_heads=[6] * 4, mlp_ratio=2, upsampler="pixelshuffledirect",
                            resi_connection="1conv", compute_dtype=dtype)
        B, shp, sc = 64, (3, 64, 64), 2
    elif name == "rrdbnet":
        from kair_amd.models.network_rrdbnet import RRDBNet
        mk = lambda: RRDBNet(3, 3, 64, 23, 32, 4, compute_dtype=dtype)   # noqa: E731
        B, shp, sc = 16, (3, 32, 32), 4
    elif name == "usrnet":
        return run_usrnet(steps, warmup, dev, dtype)
    else:
        raise SystemExit(f"unknown config {name}")
    net, ema = mk().to(dev).train(), mk().to(dev).eval()
    ema.load_state_dict(net.state_dict())
    if head_pad is not None or grouped_wgrad is not None or side_ctas is not None:
        from kair_amd.engine.swinir_engine import SwinIREngine
        net._engine = SwinIREngine(net, dtype, net.split_conv, net.fused_blocks, head_pad=head_pad,
                                   grouped_wgrad=grouped_wgrad, side_ctas=side_ctas)
    tr = FusedTrainer(net, ema, lr=1e-4, E_decay=0.999, use_graph=True)
    L = torch.rand(B, *shp, generator=g).to(dev)
    Hh = torch.rand(B, shp[0], shp[1] * sc, shp[2] * sc, generator=g).to(dev)
    dt, loss = timed(lambda: tr.step(L, Hh), steps, warmup)
    return B, dt, float(loss.item())


def run_usrnet(steps, warmup, dev, dtype="bf16"):
    from kair_amd.engine.trainer import FusedTrainer
    from kair_amd.models.network_usrnet import USRNet
    net = USRNet(n_iter=6, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2, compute_dtype=dtype).to(dev).train()
    tr = FusedTrainer(net, None, lr=1e-4, E_decay=0.0, use_graph=True)   # train_usrnet.json: E_decay 0
    g = torch.Generator().manual_seed(2)
    B, lq, sf = 48, 128, 4
    L = torch.rand(B, 3, lq, lq, generator=g).to(dev)
    Hh = torch.rand(B, 3, lq * sf, lq * sf, generator=g).to(dev)
    k = torch.rand(B, 1, 25, 25, generator=g)
    k = (k / k.sum((-2, -1), keepdim=True)).to(dev)
    sigma = (torch.rand(B, 1, 1, 1, generator=g) * 25 / 255).to(dev)

    # ModelPlain.optimize_parameters (model_plain.py:270-318) with ModelPlain4's forward
    dt, loss = timed(lambda: tr.step(L, Hh, k, sf, sigma), steps, warmup)
    return B, dt, float(loss.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["dncnn", "swinir_light", "rrdbnet", "usrnet"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp32x3"])
    ap.add_argument("--head-pad", type=int, default=None, choices=[16, 32])
    ap.add_argument("--no-grouped-wgrad", action="store_true", help="SwinIR: one weight-gradient launch per linear (A/B)")
    ap.add_argument("--side-ctas", type=int, default=None, help="SwinIR: side-stream workgroup cap (0: uncapped)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name in a.configs:
        B, dt, loss = run(name, a.steps, a.warmup, dev, a.dtype, a.head_pad, False if a.no_grouped_wgrad else None,
                          a.side_ctas)
        pps = B / dt
        tf = pps * TRAIN_GFLOP[name] / 1e3
        print(json.dumps({"config": name, "patches_per_s": round(pps, 2), "ms_per_step": round(dt * 1e3, 3), "batch": B,
                          "train_gflop_per_patch": TRAIN_GFLOP[name], "achieved_tflops": round(tf, 2),
                          "frac_of_bf16_peak": round(tf / PEAK_BF16_TFLOPS, 4), "loss": round(loss, 6),
                          "dtype": a.dtype, "n_gpus": 1}), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
