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


def _time(launch, reps):
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def time_fused_kernels(engine, reps=30):
    """HIP-event timing (torch's current stream = the stream the kernels launch on) of the two fused
    Swin-block kernels of block 0 at the step's exact arguments -- the two largest shares of the step
    (profiles/r02_step_breakdown_b32.txt):

      mlp:  kair_swin_mlp_fwd  (LN2 + fc1 + GELU + fc2 + residual, network_swinir.py:274-276, 24-30)
      attn: kair_swin_attn_fwd (LN1 + QKV + window attention + proj + residual, :239-272, 114-145)

    Algorithmic bytes / FLOPs (unpadded C = 180, hidden 360, 64-token units):
      mlp  per 64 rows: x in + out (fp32) 2 x 46080, ln2 23040, g = GELU'(u) and h (bf16) 2 x 46080,
           mean/rstd 512 = 207872 B; 2 x 2 x 64 x 180 x 360 = 16.59 MFLOP
      attn per window: x in + mid out (fp32) 2 x 46080, ln1 / O 2 x 23040, q/k/v 69120, lse 1536,
           mean/rstd 512 = 209408 B; qkv 12.44 + q.k^T / p.v 2.95 + proj 4.15 = 19.54 MFLOP
    plus each kernel's weights once per launch.  Both sit near 80-135 FLOP/B, below the 312 FLOP/B
    ridge, so the byte roofline binds."""
    from kair_amd import _hip as H
    P = engine.cur
    blk, S = engine.blocks[0], P["blocks"][0]
    nh, Cp, C = engine.nh, engine.Cp, engine.C
    M, Hh, Ww = P["M"], P["H"], P["W"]
    nWin = P["nWin"]
    if not (engine.fused_attn and engine.fused_mlp):
        raise RuntimeError("bench roofline: the fused block kernels are not in use")
    T = 64
    out = {}

    def attn():
        H.swin_attn_fwd(P["s0"], Cp, blk.n1.weight, blk.n1.bias, blk.n1.eps, C, S["ln1"], Cp, S["m1"], S["r1"],
                        blk.qkv.Wg, blk.qkv.bp, S["qkv"], blk.table, blk.scale, S["O"], nh * 32, C // nh, S["lse"],
                        blk.proj.Wg, blk.proj.bp, None, Hh * Ww, S["mid"], Cp, nWin, nh, Hh, Ww, blk.shift,
                        w_split=blk.qkv.split)
    per = 2 * T * C * 4 + 2 * T * C * 2 + 3 * T * C * 2 + nh * T * 4 + T * 8
    out["attn"] = {"kernel": "swin_attn_fwd_kernel<6,1> (fused LN1+QKV+window attention+proj+residual, "
                             "network_swinir.py:239-272)", "rocprof_key": "swin_attn_fwd_kernel<6, 1>",
                   "ms": _time(attn, reps), "units": nWin, "bytes_per_unit": per,
                   "bytes": nWin * per + 2 * (3 * C * C + C * C),
                   "flops": nWin * (2 * T * C * 3 * C + 2 * 2 * T * T * C + 2 * T * C * C)}
    f1, f2 = blk.fc1, blk.fc2
    Hd = f1.N

    def mlp():
        H.swin_mlp_fwd(S["mid"], Cp, blk.n2.weight, blk.n2.bias, blk.n2.eps, C, S["ln2"], Cp, S["m2"], S["r2"],
                       f1.Wg, f1.bp, S["u"], S["h"], engine.Hdp, Hd, f2.Wg, f2.bp, None, Hh * Ww, S["out"], Cp, M, Cp,
                       engine.Hdp, w_split=f1.split)
    tiles = M // T
    per = 2 * T * C * 4 + T * C * 2 + 2 * T * Hd * 2 + T * 8
    out["mlp"] = {"kernel": "swin_mlp_fwd_kernel<1> (fused LN2+fc1+GELU+fc2+residual, network_swinir.py:274-276, "
                            "24-30)", "rocprof_key": "swin_mlp_fwd_kernel<1>",
                  "ms": _time(mlp, reps), "units": tiles, "bytes_per_unit": per,
                  "bytes": tiles * per + 2 * 2 * C * Hd, "flops": tiles * 2 * 2 * T * C * Hd}
    return out


def time_in_step(engine, L, drop):
    """In-step durations of the fused kernels: one eager forward of the step (same batch, DropPath
    scales, every block's own weights and the caches the preceding kernels leave), a HIP event pair
    on the launch stream around each kair_swin_attn_fwd / kair_swin_mlp_fwd call.  This is the
    duration rocprofv3's kernel trace of the graph-replayed step reports (profiles/), unlike the
    back-to-back timing of one block's launch above, which runs with warm caches."""
    from kair_amd import _hip as H
    names = ("swin_attn_fwd", "swin_mlp_fwd")
    orig = {n: getattr(H, n) for n in names}
    rec = {n: [] for n in names}

    def wrap(n):
        def f(*a, **k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            orig[n](*a, **k)
            e1.record()
            rec[n].append((e0, e1))
        return f

    for n in names:
        setattr(H, n, wrap(n))
    try:
        for _ in range(2):   # the second pass is the one kept
            for n in names:
                rec[n].clear()
            engine.forward(L, drop)
    finally:
        for n in names:
            setattr(H, n, orig[n])
    torch.cuda.synchronize()
    return {("attn" if n == "swin_attn_fwd" else "mlp"): sum(a.elapsed_time(b) for a, b in r) / len(r)
            for n, r in rec.items() if r}


def pmc_traffic(key):
    """HBM bytes per launch of kernel `key` from the committed rocprofv3 PMC summary
    (profiles/r02_pmc_traffic.json, written by tools/pmc_traffic.py: FETCH_SIZE x 2 per the gfx950
    correction + WRITE_SIZE, KiB -> bytes), or None when absent."""
    path = os.path.join(ROOT, "profiles", "r02_pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)
        for name, v in rec["kernels"].items():
            if key in name:
                return v["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        pass
    return None


def cpu_baseline(batch=4, steps=4):
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


def fp32_line(bpg, device, drop_path, steps=4, warmup=2):
    """Throughput of the same training step on the exact-fp32 engine (fp32 MFMA, same kernels and
    program): the parity configuration, whose forward matches the CPU oracle to 1e-7 dB.  A short
    run (the fp32 step is ~10x the bf16 one), timed like the headline."""
    from kair_amd.engine.trainer import FusedTrainer
    from kair_amd.utils.utils_image import synth_sr_batch
    net = build_net("fp32", drop_path).to(device).train()
    ema = build_net("fp32", drop_path).to(device).eval()
    ema.load_state_dict(net.state_dict())
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999)
    L, Hh = synth_sr_batch(bpg, 48, 4, seed=1000, device=device)
    for _ in range(warmup):
        tr.step(L, Hh)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(L, Hh)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del tr, net, ema
    return {"value": round(bpg * steps / dt, 2), "unit": "patches/s", "ms_per_step": round(1000 * dt / steps, 3),
            "steps": steps, "warmup": warmup, "dtype": "fp32", "per_gpu_batch": bpg,
            "note": "parity configuration (exact-f32 MFMA engine); the headline value is the bf16 engine"}


def psnr_parity(net_gpu, device, n_eval=8):
    """PSNR of the GPU forward vs the CPU oracle on the same (trained) weights, DropPath off (eval),
    averaged per image over n_eval held-out 48-px patches as the reference's test loop averages
    (main_train_psnr.py: avg_psnr over the test set), float and uint8 / border-4.

    The fp32 parity engine (same kernels, exact-f32 MFMA) must match the oracle to 1e-3 dB; the bf16
    engine's deviation is reported beside it.  One patch alone is not an evaluation set: bf16
    activation rounding moves a single 192x192 uint8 PSNR by up to ~1e-3 dB either way, the
    8-patch mean by ~3e-4 (tools/parity_seeds.py, DESIGN.md "parity at bf16")."""
    from oracle import swinir as osw
    from kair_amd.utils import utils_image as U
    ref = osw.SwinIR(4, 3, 48, 8, 1.0, [6] * 6, 180, [6] * 6, 2, "pixelshuffle")
    sd = {k: v.detach().float().cpu() for k, v in net_gpu.state_dict().items()}
    ref.load_state_dict(sd, strict=True)
    net32 = build_net("fp32", 0.0).to(device).eval()
    net32.load_state_dict(net_gpu.state_dict(), strict=True)
    L, Hh = U.synth_sr_batch(n_eval, 48, 4, seed=77)
    was = net_gpu.training
    net_gpu.eval()
    with torch.no_grad():
        E = net_gpu(L.to(device)).float().cpu()
        E32 = net32(L.to(device)).float().cpu()
        Er = ref(L)
    net_gpu.train(was)
    del net32

    def per_image(X):
        pf = [U.psnr_float(X[i:i + 1], Hh[i:i + 1]) for i in range(n_eval)]
        pu = [U.calculate_psnr(U.tensor2uint(X[i]), U.tensor2uint(Hh[i]), border=4) for i in range(n_eval)]
        return pf, pu
    (bf, bu), (ff, fu), (rf, ru) = per_image(E), per_image(E32), per_image(Er)
    mean = lambda v: sum(v) / len(v)
    dmax = lambda a, b: max(abs(x - y) for x, y in zip(a, b))
    return {"eval": f"{n_eval} held-out 48-px LQ patches (synth seed 77), per-image PSNR averaged",
            "cpu_oracle_db": round(mean(rf), 5), "fp32_gpu_db": round(mean(ff), 5),
            "fp32_delta_db": round(abs(mean(ff) - mean(rf)), 7),
            "uint8_border4_cpu_db": round(mean(ru), 5), "uint8_border4_fp32_gpu_db": round(mean(fu), 5),
            "uint8_fp32_delta_db": round(abs(mean(fu) - mean(ru)), 7),
            "bf16_gpu_db": round(mean(bf), 5), "bf16_delta_db": round(abs(mean(bf) - mean(rf)), 6),
            "uint8_border4_bf16_gpu_db": round(mean(bu), 5), "uint8_bf16_delta_db": round(abs(mean(bu) - mean(ru)), 6),
            "bf16_max_single_image_delta_db": round(dmax(bf, rf), 6),
            "uint8_bf16_max_single_image_delta_db": round(dmax(bu, ru), 6),
            "max_abs_fp32_vs_oracle": float((E32 - Er).abs().max()),
            "max_abs_bf16_vs_oracle": float((E - Er).abs().max())}


def other_configs(device):
    """The other BASELINE.json configs, one short fused-trainer run each (USRNet with (k, sf, sigma) inputs)
    on this GPU (tools/bench_models.py; synthetic seeded inputs resident in HBM): patches/s and the
    fraction of the dense bf16 MFMA peak their training FLOPs reach.  C1 (DnCNN) is a CPU config in
    the reference; its network's GPU step is reported for completeness."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import bench_models as bm
    labels = {"swinir_light": "C2 SwinIR-lightweight x2, 64-px LQ, batch 64",
              "usrnet": "C3 USRNet x4, 128-px LQ (512^2 HR), batch 48, n_iter 6",
              "rrdbnet": "C5 RRDBNet x4, 32-px LQ, batch 16 (the N=1 shape of global batch 16)",
              "dncnn": "C1 DnCNN sigma 25, 40x40, batch 64 (GPU step of the CPU config's network)"}
    res = {}
    for name, label in labels.items():
        try:
            B, dt, loss = bm.run(name, 5, 3, device)
            pps = B / dt
            tf = pps * bm.TRAIN_GFLOP[name] / 1e3
            res[name] = {"config": label, "value": round(pps, 2), "unit": "patches/s", "ms_per_step": round(dt * 1e3, 3),
                         "steps": 5, "warmup": 3, "train_gflop_per_patch": bm.TRAIN_GFLOP[name],
                         "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_BF16_TFLOPS,
                                      "unit": "TFLOP/s", "frac": round(tf / PEAK_BF16_TFLOPS, 4)},
                         "final_loss": round(loss, 6)}
        except Exception as e:  # noqa: BLE001
            res[name] = {"config": label, "error": repr(e)}
        torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)   # >= 100 timed steps after >= 20 warm-up
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--global-batch", type=int, default=32)
    ap.add_argument("--per-gpu-batch", type=int, default=None, help="weak scaling: fixed batch per GPU")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--drop-path", type=float, default=0.1)
    ap.add_argument("--no-fp32-line", action="store_true", help="skip the fp32 parity-config throughput line")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the short single-GPU throughput lines of BASELINE.json configs C2 / C3 / C5 (and the "
                         "C1 network on the GPU)")
    ap.add_argument("--data", default="pool", choices=["pool", "static"],
                    help="pool: every step synthesises a fresh batch on the GPU from an HBM-resident HR pool "
                         "(kair_synth_sr: crop + 8-way augment + MATLAB bicubic x1/4, DatasetSR semantics) inside "
                         "the timed loop; static: one staged batch reused")
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
    if args.data == "pool":
        from kair_amd.data.gpu_synth import PatchSynth, synthetic_pool
        pool = synthetic_pool(64, 3, 256, 256, seed=99, device=device)
        synth = PatchSynth(pool, task="sr", scale=4, H_size=192, seed=1000, rank=rank, world=world)
        batch = lambda: synth.next(bpg)
    else:
        L, Hh = synth_sr_batch(bpg, 48, 4, seed=1000 + rank, device=device)
        batch = lambda: (L, Hh)

    for _ in range(args.warmup):
        loss = tr.step(*batch())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        loss = tr.step(*batch())
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
    try:
        ks = time_fused_kernels(tr.engine)
        from kair_amd.engine.swinir_engine import drop_path_scales
        Lb = tr.static[0] if tr.static is not None else None
        if Lb is not None:
            drop = drop_path_scales(tr.engine, Lb.shape[0], Lb.device) if args.drop_path > 0 else None
            for k, ms in time_in_step(tr.engine, Lb, drop).items():   # the roofline uses the in-step time
                ks[k]["ms_isolated"], ks[k]["ms"] = ks[k]["ms"], ms
    except RuntimeError as e:   # fp32 engine: no fused block kernels
        ks = {"err": repr(e)}

    def roof(k):
        ach_gbs = k["bytes"] / (k["ms"] * 1e-3) / 1e9
        ach_tf = k["flops"] / (k["ms"] * 1e-3) / 1e12
        return {"bound": "hbm", "achieved": round(ach_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(ach_gbs / PEAK_HBM_GBS, 4), "traffic": pmc_traffic(k["rocprof_key"]),
                "kernel": k["kernel"], "kernel_ms": round(k["ms"], 5),
                "kernel_ms_timing": "in-step mean over every block of one eager forward (HIP events on the launch stream)"
                if "ms_isolated" in k else "back-to-back launches of block 0",
                "kernel_ms_isolated": round(k["ms_isolated"], 5) if "ms_isolated" in k else None,
                "bytes_per_launch": k["bytes"],
                "units_per_launch": k["units"], "bytes_per_unit": k["bytes_per_unit"],
                "flops_per_launch": k["flops"], "achieved_tflops": round(ach_tf, 2), "mfma_frac": round(ach_tf / peak, 4)}
    out = {
        "metric": "train patches/sec + PSNR, SwinIR x4 48-px LQ, at 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "patches/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
        "dtype": args.dtype,
        "data": ("synthetic: per step a fresh batch synthesised on the GPU (crop / augment / MATLAB bicubic) from "
                 "a 64-image 256x256 HR pool resident in HBM (SURVEY §8d recipe)" if args.data == "pool" else
                 "synthetic (one seeded bicubic-LR / HR batch resident in HBM, SURVEY §8d)"),
        "config": {"workload": "SwinIR classical x4 SR train step (fwd+L1+bwd+allreduce+Adam+EMA), 48-px LQ",
                   "global_batch": gbatch, "per_gpu_batch": bpg, "lq": 48, "hr": 192, "embed_dim": 180,
                   "depths": [6] * 6, "heads": 6, "window": 8, "drop_path_rate": args.drop_path,
                   "parallelism": f"dp{world}", "hip_graph": not args.no_graph},
        "roofline": roof(ks["mlp"]) if "mlp" in ks else {"error": ks["err"]},
        "roofline_attention": roof(ks["attn"]) if "attn" in ks else None,
        "step_roofline": {"train_flop_per_patch": fl["train"], "achieved_tflops_per_gpu": round(step_tflops, 2),
                          "frac_of_bf16_peak": round(step_tflops / peak, 4)},
        "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
        "final_loss": round(final_loss, 6),
    }
    if args.dtype == "bf16" and world == 1 and not args.no_fp32_line:
        try:
            out["fp32_parity_line"] = fp32_line(bpg, device, args.drop_path)
        except Exception as e:  # noqa: BLE001
            out["fp32_parity_line"] = {"error": repr(e)}
    try:
        out["psnr"] = psnr_parity(net, device)
    except Exception as e:  # noqa: BLE001
        out["psnr"] = {"error": repr(e)}
    if world == 1 and args.dtype == "bf16" and not args.no_other_configs:
        out["other_configs"] = other_configs(device)
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
