"""Headline benchmark: SwinIR classical x4 (48-px LQ) training patches/s on MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch 32 | --per-gpu-batch B]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

A step = ModelPlain.optimize_parameters of the reference (model_plain.py:270-318): forward, L1 loss,
backward, gradient all-reduce (N>1), Adam, EMA 0.999 — here the fused kair_amd trainer, captured in a
HIP graph.  Inputs are seeded synthetic patches already resident in HBM.  Rank 0 prints
ONE JSON line (plus roofline of the dominant kernel and the CPU-oracle baseline at N=1).
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, Chip-level parameters)
PEAK_F32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def build_net(dtype, drop_path=0.1, seed=0):
    from kair_amd.models.network_swinir import SwinIR
    torch.manual_seed(seed)
    return SwinIR(upscale=4, in_chans=3, img_size=48, window_size=8, img_range=1.0, depths=[6] * 6, embed_dim=180,
                  num_heads=[6] * 6, mlp_ratio=2, upsampler="pixelshuffle", resi_connection="1conv",
                  drop_path_rate=drop_path, compute_dtype=dtype)


def time_dominant_kernel(engine, reps=30):
    """HIP-event timing (torch's current stream = the stream the kernels launch on) of the QKV
    projection GEMM of block 0 at the step's exact arguments.

    The projection is HBM-bound at these shapes (2*K*N/(K+N) = 135 FLOP/B against the MI355X ridge
    of 2500 TFLOP/s / 8 TB/s = 312 FLOP/B), so its roofline is bytes: algorithmic bytes = the bf16
    operand M x K, the bf16 weight N x K and the bf16 q/k/v output M x N, each moved once
    (K = 180, N = 540: the unpadded layer)."""
    from kair_amd import _hip as H
    P = engine.cur
    blk, S = engine.blocks[0], P["blocks"][0]
    l = blk.qkv
    M = P["M"]

    def launch():
        H.gemm_nt(H.rows(S["ln1"]), H.rows(l.Wp), H.epilogue(S["qkv"], mode=H.OUT_QKVBLK, ldo=0, bias=l.bp,
                                                               qkv=(engine.nh, 32, 64)), M, l.Np, engine.Cp, engine.cd)
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flops = 2.0 * M * l.N * l.K
    nbytes = 2.0 * (M * l.K + l.N * l.K + M * l.N)
    return {"kernel": "gemm_nt_ring<192,5,0,1,0> (block QKV projection, network_swinir.py:121; rocprof name "
                      "_ZN..gemm_nt_ringILi192ELi5ELi0ELi1ELi0E..)",
            "rocprof_key": "gemm_nt_ring<192, 5, 0, 1, 0>",
            "ms": ms, "flops": flops, "bytes": nbytes, "M": M, "N": l.N, "K": l.K}


def pmc_traffic(key):
    """HBM bytes per launch of kernel `key` from the committed rocprofv3 PMC summary
    (profiles/r01_pmc_traffic.json, written by tools/pmc_traffic.py: FETCH_SIZE x 2 per the gfx950
    correction + WRITE_SIZE, KiB -> bytes), or None when absent."""
    path = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)
        for name, v in rec["kernels"].items():
            if key in name:
                return v["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        pass
    return None


def cpu_baseline(batch=2, steps=2):
    """The CPU oracle (fp32 restatement of ModelPlain.optimize_parameters) on the host cores."""
    from oracle import swinir as osw
    from oracle.train import OracleTrainer
    from kair_amd.utils.utils_image import synth_sr_batch
    threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    net = osw.SwinIR(4, 3, 48, 8, 1.0, [6] * 6, 180, [6] * 6, 2, "pixelshuffle")
    ema = osw.SwinIR(4, 3, 48, 8, 1.0, [6] * 6, 180, [6] * 6, 2, "pixelshuffle")
    ema.load_state_dict(net.state_dict())
    tr = OracleTrainer(net, ema, lr=2e-4, E_decay=0.999)
    L, Hh = synth_sr_batch(batch, 48, 4, seed=123)
    tr.optimize_parameters(L, Hh)          # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.optimize_parameters(L, Hh)
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 4), "unit": "patches/s", "cores": threads, "kind": "port",
            "sample": f"oracle SwinIR classical x4 fp32 train step (fwd+L1+bwd+Adam+EMA), batch {batch}, "
                      f"{steps} timed steps after 1 warm-up, torch CPU {threads} threads"}


def psnr_parity(net_gpu, device):
    """PSNR of the GPU forward vs the CPU oracle on the same (trained) weights, DropPath off (eval).

    SURVEY §8d's 1e-3 dB bar is checked on the fp32 parity engine (same weights, same kernels with
    exact-f32 MFMA); the bf16 engine's deviation from the fp32 oracle is reported beside it."""
    from oracle import swinir as osw
    from kair_amd.utils import utils_image as U
    ref = osw.SwinIR(4, 3, 48, 8, 1.0, [6] * 6, 180, [6] * 6, 2, "pixelshuffle")
    sd = {k: v.detach().float().cpu() for k, v in net_gpu.state_dict().items()}
    ref.load_state_dict(sd, strict=True)
    net32 = build_net("fp32", 0.0).to(device).eval()
    net32.load_state_dict(net_gpu.state_dict(), strict=True)
    L, Hh = U.synth_sr_batch(1, 48, 4, seed=7)
    was = net_gpu.training
    net_gpu.eval()
    with torch.no_grad():
        E = net_gpu(L.to(device)).float().cpu()
        E32 = net32(L.to(device)).float().cpu()
        Er = ref(L)
    net_gpu.train(was)
    del net32
    pf, p32, pr = U.psnr_float(E, Hh), U.psnr_float(E32, Hh), U.psnr_float(Er, Hh)
    hu = U.tensor2uint(Hh)
    uf = U.calculate_psnr(U.tensor2uint(E), hu, border=4)
    u32 = U.calculate_psnr(U.tensor2uint(E32), hu, border=4)
    ur = U.calculate_psnr(U.tensor2uint(Er), hu, border=4)
    return {"cpu_oracle_db": round(pr, 5), "fp32_gpu_db": round(p32, 5), "fp32_delta_db": round(abs(p32 - pr), 7),
            "uint8_border4_cpu_db": round(ur, 5), "uint8_border4_fp32_gpu_db": round(u32, 5),
            "uint8_fp32_delta_db": round(abs(u32 - ur), 7),
            "bf16_gpu_db": round(pf, 5), "bf16_delta_db": round(abs(pf - pr), 6),
            "uint8_border4_bf16_gpu_db": round(uf, 5), "uint8_bf16_delta_db": round(abs(uf - ur), 6),
            "max_abs_fp32_vs_oracle": float((E32 - Er).abs().max()),
            "max_abs_bf16_vs_oracle": float((E - Er).abs().max())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--global-batch", type=int, default=32)
    ap.add_argument("--per-gpu-batch", type=int, default=None, help="weak scaling: fixed batch per GPU")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--drop-path", type=float, default=0.1)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(device)

    from kair_amd.engine.trainer import FusedTrainer
    from kair_amd.engine.swinir_engine import swinir_flops
    from kair_amd.utils.utils_image import synth_sr_batch

    if args.per_gpu_batch:
        bpg, scaling = args.per_gpu_batch, "weak"
        gbatch = bpg * world
    else:
        gbatch, scaling = args.global_batch, "strong"
        if gbatch % world:
            raise SystemExit(f"global batch {gbatch} not divisible by {world} ranks")
        bpg = gbatch // world

    net = build_net(args.dtype, args.drop_path).to(device).train()
    ema = build_net(args.dtype, args.drop_path).to(device).eval()
    ema.load_state_dict(net.state_dict())
    if world > 1:   # replicas start identical (DDP construction broadcast, model_base.py:116)
        for t in list(net.state_dict().values()) + list(ema.state_dict().values()):
            dist.broadcast(t, 0)
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999, use_graph=not args.no_graph)
    L, Hh = synth_sr_batch(bpg, 48, 4, seed=1000 + rank, device=device)

    for _ in range(args.warmup):
        loss = tr.step(L, Hh)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        loss = tr.step(L, Hh)
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gpu_ms = e0.elapsed_time(e1)
    el = torch.tensor([wall], device=device, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    wall = el.item()
    final_loss = loss.item()

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    fl = swinir_flops(net, 48, 48)
    value = gbatch * args.steps / wall
    ms_step = 1000.0 * wall / args.steps
    step_tflops = fl["train"] * gbatch / (wall / args.steps) / 1e12 / world   # per GPU
    peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
    k = time_dominant_kernel(tr.engine)
    ach_gbs = k["bytes"] / (k["ms"] * 1e-3) / 1e9
    ach_tf = k["flops"] / (k["ms"] * 1e-3) / 1e12
    out = {
        "metric": "train patches/sec + PSNR, SwinIR x4 48-px LQ, at 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "patches/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
        "dtype": args.dtype, "data": "synthetic (seeded bicubic-LR / HR patches resident in HBM, SURVEY §8d)",
        "config": {"workload": "SwinIR classical x4 SR train step (fwd+L1+bwd+allreduce+Adam+EMA), 48-px LQ",
                   "global_batch": gbatch, "per_gpu_batch": bpg, "lq": 48, "hr": 192, "embed_dim": 180,
                   "depths": [6] * 6, "heads": 6, "window": 8, "drop_path_rate": args.drop_path,
                   "parallelism": f"dp{world}", "hip_graph": not args.no_graph},
        "roofline": {"bound": "hbm", "achieved": round(ach_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(ach_gbs / PEAK_HBM_GBS, 4), "traffic": pmc_traffic(k["rocprof_key"]),
                     "kernel": k["kernel"], "kernel_ms": round(k["ms"], 5), "bytes_per_launch": k["bytes"],
                     "flops_per_launch": k["flops"], "achieved_tflops": round(ach_tf, 2),
                     "mfma_frac": round(ach_tf / peak, 4), "shape_MNK": [k["M"], k["N"], k["K"]]},
        "step_roofline": {"train_flop_per_patch": fl["train"], "achieved_tflops_per_gpu": round(step_tflops, 2),
                          "frac_of_bf16_peak": round(step_tflops / peak, 4)},
        "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
        "final_loss": round(final_loss, 6),
    }
    try:
        out["psnr"] = psnr_parity(net, device)
    except Exception as e:  # noqa: BLE001
        out["psnr"] = {"error": repr(e)}
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
