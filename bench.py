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
PRECISION_BF16 = ("training step: bf16 MFMA with fp32 accumulation; every forward conv multiplies hi/lo bf16 pairs of "
                  "its weights AND its input activation (~16-bit operands: the input image, RSTB / conv_after_body "
                  "inputs, the reconstruction tail), Swin-block GEMM operands bf16; fp32 master weights, residual "
                  "stream, LayerNorm statistics, softmax and Adam + EMA.  Evaluation (the psnr fields, eval-mode "
                  "forwards): the same kernels with the Swin-block linear weights as hi/lo pairs too "
                  "(SwinIR.eval_engine).  Holds the PSNR bar: "
                  "tests/test_swinir_gpu.py::test_swinir_classical_full_psnr_along_training[bf16], 160 steps")
PRECISION_X3 = ("training step at the fp32 reference's precision class: every operand x of every GEMM, conv and window-"
                "attention product is carried as an fp16 pair of x 2^e (hi = f16(x 2^e), lo = f16(x 2^e - hi), e a power "
                "of two per tensor class) and every product as hi.hi + hi.lo + lo.hi on v_mfma_f32_{16x16x32,32x32x16}_f16 "
                "with fp32 accumulation (~2^-21 per product); fp32 master weights, residual stream, LayerNorm statistics, "
                "softmax, GELU (erf), Adam + EMA.  Passes the exact-fp32 engine's oracle bars unchanged: tests/test_x3_gpu.py "
                "(classical x4 full network vs the CPU oracle: outputs < 1e-4, gradients < 1e-3, PSNR < 1e-3 dB; the "
                "3-step ModelPlain trajectory < 1e-4)")
PRECISION_F32 = "fp32 operands, exact fp32 MFMA (v_mfma_f32_16x16x4_f32)"
PRECISION = {"bf16": PRECISION_BF16, "fp32x3": PRECISION_X3, "fp32": PRECISION_F32}


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


# ---- in-step kernel timing and algorithmic bytes -------------------------------------------------
# One eager forward + loss + backward of the timed configuration with a HIP-event pair around every
# libkair launch, recorded on the stream that launch uses (torch's current stream at the call: the main
# stream, or the engine's side stream for the deferred weight-gradient work), so concurrency with the
# side stream is what the graph-replayed step sees.  A launch's role is its call site in the engine.
_REAL = {576: 540, 384: 360, 192: 180}   # padded operand width -> the reference's width (C 180, 2C, 3C)


def _alg_bytes(fn, a, kw=None):
    """Algorithmic bytes of one launch (reference-width operands read / written once, fp32 4 B, bf16 2 B),
    or None for launch kinds without a formula (never the dominant ones)."""
    T = 64
    kw = kw or {}
    if fn == "layernorm_fwd":         # x in (fp32), y out, mean / rstd
        x, y, M, C = a[0], a[2], a[8], a[9]
        return M * C * (4 + y.element_size()) + 8 * M
    if fn == "layernorm_bwd":         # x, dy in; dx out (+ in when accumulating); the operand copy; mean / rstd
        dy, acc, M, C = a[2], a[9], a[14], a[15]
        cp = kw.get("copy", a[17] if len(a) > 17 else None)
        return M * C * (4 + dy.element_size() + (8 if acc else 4) + (0 if cp is None else (4 if cp.dtype == 0 else 2))) + 8 * M
    if fn == "swin_mlp_fwd":          # x in + out (fp32), ln2, GELU' and GELU (bf16), mean / rstd; weights once
        C, hd, M = a[5], a[15], a[22]
        return (M // T) * (2 * T * C * 4 + T * C * 2 + 2 * T * hd * 2 + T * 8) + 2 * 2 * C * hd
    if fn == "swin_attn_fwd":         # x in + mid out, ln1 / O, q / k / v, lse, mean / rstd; weights once
        C, nWin, nh = a[5], a[25], a[26]
        return nWin * (2 * T * C * 4 + 2 * T * C * 2 + 3 * T * C * 2 + nh * T * 4 + T * 8) + 2 * (3 * C * C + C * C)
    if fn == "window_attn_bwd":       # q, k, v, O, dO, lse in; dq, dk, dv out
        nWin, nh, hd = a[11], a[12], a[13]
        M, Cr = nWin * T, nh * hd
        return M * (3 * Cr * 2 + 2 * Cr * 2 + nh * 4 + 3 * Cr * 2)
    if fn == "rowgemm_gate":          # A in, gate in, out
        M, K, N = a[1], a[2], a[4]
        return M * (_REAL[K] * 2 + 2 * _REAL[N] * 2)
    if fn == "rowgemm_store":
        M, K, N = a[1], a[2], a[4]
        return M * (_REAL[K] * 2 + _REAL[N] * 2)
    if fn == "rowgemm_lnbwd":         # A in, x in, D in + out, bf16 copy out, mean / rstd
        M, K, C = a[1], a[2], a[8]
        return M * (_REAL[K] * 2 + C * 4 + 2 * C * 4 + C * 2 + 8)
    if fn == "gemm_nt" and a[6] == X3:   # x3: fp32 / fp16-pair operands 4 B per element; A (an im2col: its map)
        A, E, M, N, K = a[0], a[2], a[3], a[4], a[5]   # once, the split weight once, out (+ pre, resid / gate)
        ka = A.im_C if A.mode == 1 else K
        nn = _REAL.get(N, N)
        per_row = _REAL.get(ka, ka) + nn * (1 + bool(E.out_pre) + bool(E.resid) + bool(E.gate))
        return 4 * (M * per_row + nn * _REAL.get(K, K))
    if fn == "gemm_tn" and a[7] == X3:   # x3 weight gradient: both operands once, the split partial planes out
        B, S, M, N, K = a[1], a[3], a[4], a[5], a[6]
        kb = B.im_C if B.mode == 1 else K
        return 4 * (M * (_REAL.get(N, N) + _REAL.get(kb, kb)) + S * N * K)
    if fn == "wgrad_grouped" and a and a[0]._keep[0][0].dtype == 3:   # fp32x3 grouped weight gradients (WgradGroup):
        grp = a[0]                                                     # every job's two pair operands once
        return sum(4 * grp.M * (_REAL.get(N, N) + _REAL.get(K, K)) for _, _, N, K, *_ in grp._keep)
    if fn == "window_attn_fwd_x3":    # q, k, v in (fp16 pairs), O out, lse
        nWin, nh, hd = a[5], a[6], a[7]
        M = nWin * T
        return M * nh * (4 * hd * 4 + 4)
    if fn == "window_attn_bwd_x3":    # q, k, v, O, dO, lse in; dq, dk, dv out
        nWin, nh, hd = a[11], a[12], a[13]
        M = nWin * T
        return M * nh * (8 * hd * 4 + 4)
    return None


def _alg_flops(fn, a):
    T = 64
    if fn == "swin_attn_fwd":
        C, nWin = a[5], a[25]
        return nWin * (2 * T * C * 3 * C + 2 * 2 * T * T * C + 2 * T * C * C)
    if fn == "swin_mlp_fwd":
        C, hd, M = a[5], a[15], a[22]
        return M * 2 * 2 * C * hd
    if fn == "window_attn_bwd":        # S, dP, dV, dK, dQ: five 64 x 64 x hd products per (window, head)
        nWin, nh, hd = a[11], a[12], a[13]
        return nWin * nh * 5 * 2 * T * T * hd
    if fn == "gemm_nt" and a[6] == X3:
        M, N, K = a[3], a[4], a[5]
        return 2 * M * _REAL.get(N, N) * _REAL.get(K, K) if a[0].mode != 1 else 2 * M * N * K
    if fn == "gemm_tn" and a[7] == X3:
        M, N, K = a[4], a[5], a[6]
        return 2 * M * _REAL.get(N, N) * _REAL.get(K, K) if a[1].mode != 1 else 2 * M * N * K
    if fn == "wgrad_grouped" and a and a[0]._keep[0][0].dtype == 3:
        grp = a[0]
        return sum(2 * grp.M * _REAL.get(N, N) * _REAL.get(K, K) for _, _, N, K, *_ in grp._keep)
    if fn == "window_attn_fwd_x3":
        nWin, nh, hd = a[5], a[6], a[7]
        return nWin * nh * 2 * 2 * T * T * hd
    if fn == "window_attn_bwd_x3":
        nWin, nh, hd = a[11], a[12], a[13]
        return nWin * nh * 5 * 2 * T * T * hd
    if fn in ("rowgemm_gate", "rowgemm_store", "rowgemm_lnbwd"):
        M, K = a[1], a[2]
        N = a[4] if fn != "rowgemm_lnbwd" else 192
        return 2 * M * _REAL[K] * _REAL[N]
    return None


X3 = 2   # kair_amd._hip.X3 (compute argument of the x3 GEMM launches)
_TIMED = ("gemm_nt", "gemm_tn", "wgrad_finalize", "colsum", "layernorm_fwd", "layernorm_bwd", "row_copy", "window_attn_fwd",
          "window_attn_fwd_x3", "window_attn_bwd_x3",
          "window_attn_bwd", "ln_param_reduce_grouped", "attn_dtable_grouped", "image_to_nhwc", "l1_loss", "axpy",
          "swin_attn_fwd", "swin_mlp_fwd", "rowgemm_store", "rowgemm_gate", "rowgemm_lnbwd", "image_to_nhwc_hilo",
          "conv3x3_narrow_fwd", "conv3x3_narrow_dgrad", "conv3x3_narrow_wgrad", "conv3x3_wr",
          "conv3x3_narrow_fwd_x3", "conv3x3_narrow_dgrad_x3", "conv3x3_narrow_wgrad_x3")


def _demangle(symbols):
    """Readable kernel names (template instantiation, no return type / parameters) for mangled symbols, through
    llvm-cxxfilt (a child process) when it is there; the symbol itself otherwise."""
    import shutil
    import subprocess
    tool = shutil.which("llvm-cxxfilt") or next((t for t in ("/opt/rocm/lib/llvm/bin/llvm-cxxfilt",) if os.path.exists(t)),
                                                 None) or shutil.which("c++filt")
    out = list(symbols)
    if tool and out:
        try:   # (binutils' demangler predates _Float16's DF16_: spelled as half, then renamed back)
            res = subprocess.run([tool], input="\n".join(x.replace("DF16_", "Dh") for x in out) + "\n",
                                 capture_output=True, text=True, timeout=60)
            dem = [d.replace("half", "_Float16") for d in res.stdout.splitlines()]
            if len(dem) == len(out):
                out = dem
        except (OSError, subprocess.SubprocessError):
            pass

    def short(n):
        n = n.replace("(anonymous namespace)::", "")
        if n.startswith("void "):
            n = n[5:]
        depth = 0
        for i, ch in enumerate(n):
            depth += ch == "<"
            depth -= ch == ">"
            if ch == "(" and depth == 0 and i > 0:
                return n[:i]
        return n
    return {s: short(d) for s, d in zip(symbols, out)}


def time_roles(tr, serial=False, passes=2):
    """In-step kernel durations of one fwd + loss + bwd of the timed configuration, run eagerly with its side-stream
    concurrency (serial: the engine's deferred side-stream work in place on the main stream instead) inside a kernel
    timing window (kair_ktime_begin): every libkair launch is dispatched with hipExtLaunchKernel and an event pair
    the runtime stamps with the dispatch packet's start / end -- the kernel duration rocprofv3 --kernel-trace
    reports.  The pass is queued whole behind a held wave (kair_gate_hold) and released at once, so it runs back to
    back like the graph-replayed step, not at the host's launch pace.  The last of `passes` passes is kept.

    Returns (roles, kernels):
      roles    {call site: {kernel, launches, ms_total, ms, bytes, flops}} -- a call site's launches are the libkair
               calls made there (the engine's thin helpers skipped), its time the kernels those calls dispatched;
      kernels  {kernel: {kernel, symbol, launches, ms_total, ms, bytes, flops, roles}} -- rocprofv3's grouping (one
               template instantiation); bytes / flops: the algorithmic bytes / FLOPs per launch, each call's figure
               (_alg_bytes / _alg_flops) attributed to the longest kernel it dispatched, averaged over the attributed
               launches (ms_attr: their mean duration)."""
    from kair_amd import _hip as H
    rec = []   # (role, fn, (args, kwargs), first slot, end slot)

    # the engine's thin launch helpers: a role is named by their caller (the layer's call site), not by them
    helpers = ("_nt", "_wgrad", "_wg", "_run_conv_job", "_bias_colsum")

    def site():
        fr = sys._getframe(2)
        while fr.f_back is not None and fr.f_code.co_name in helpers:
            fr = fr.f_back
        return f"{os.path.basename(fr.f_code.co_filename)}:{fr.f_lineno}"

    def wrap(name, f):
        def g(*a, **k):
            where = site()
            s0 = H.ktime_count()
            r = f(*a, **k)
            rec.append((f"{name} @ {where}", name, (a, k), s0, H.ktime_count()))
            return r
        return g

    orig = {n: getattr(H, n) for n in _TIMED}
    run0 = H.WgradGroup.run
    eng = getattr(tr, "engine", None)
    side0 = getattr(eng, "side_stream", None)
    if serial and side0 is not None:
        eng.side_stream = False

    def wg_run(self, ws, **kw):
        where = site()
        s0 = H.ktime_count()
        r = run0(self, ws, **kw)
        rec.append((f"wgrad_grouped @ {where}", "wgrad_grouped", ((self,), {}), s0, H.ktime_count()))
        return r
    for n in _TIMED:
        setattr(H, n, wrap(n, orig[n]))
    H.WgradGroup.run = wg_run
    nslot, gate = 0, []
    try:
        for _ in range(passes):
            torch.cuda.synchronize()
            H.gate_hold(5000)   # the pass is queued whole behind a held wave, then runs back to back
            rec.clear()
            H.ktime_begin(8192)
            try:
                tr._fwd_bwd(*tr.static)
            finally:
                nslot = H.ktime_end()
                H.gate_release()
            torch.cuda.synchronize()
            gate.append(H.gate_status())
    finally:
        for n in _TIMED:
            setattr(H, n, orig[n])
        H.WgradGroup.run = run0
        if serial and side0 is not None:
            eng.side_stream = side0
    if nslot >= 8192:
        raise RuntimeError("time_roles: kernel timing window full (8192 launches)")
    if gate[-1] != 1:
        raise RuntimeError("time_roles: the launch gate timed out before the pass was queued (a host sync inside "
                           "the pass?)")
    slot = {i: H.ktime_read(i) for i in range(nslot)}
    names = _demangle(sorted({sym for _, sym in slot.values()}))
    # each slot belongs to the innermost recorded call whose range holds it
    owner = {}
    for j in sorted(range(len(rec)), key=lambda j: rec[j][4] - rec[j][3]):
        for i in range(rec[j][3], rec[j][4]):
            owner.setdefault(i, j)
    roles, kernels = {}, {}
    for i, (ms, sym) in slot.items():
        kn = names.get(sym, sym)
        d = kernels.setdefault(kn, {"kernel": kn, "symbol": sym, "launches": 0, "ms_total": 0.0, "b": 0, "f": 0,
                                    "nb": 0, "nf": 0, "ms_b": 0.0, "ms_f": 0.0, "roles": set()})
        d["launches"] += 1
        d["ms_total"] += ms
        j = owner.get(i)
        role = rec[j][0] if j is not None else f"(outside the timed helpers) {kn}"
        d["roles"].add(role)
    for j, (role, fn, (a, k), s0, s1) in enumerate(rec):
        mine = [i for i in range(s0, s1) if owner.get(i) == j]
        r = roles.setdefault(role, {"launches": 0, "ms_total": 0.0, "b": 0, "f": 0, "nb": False, "nf": False, "k": {}})
        r["launches"] += 1
        if not mine:
            continue
        r["ms_total"] += sum(slot[i][0] for i in mine)
        top = max(mine, key=lambda i: slot[i][0])
        kn = names.get(slot[top][1], slot[top][1])
        r["k"][kn] = r["k"].get(kn, 0) + 1
        b, f = _alg_bytes(fn, a, k), _alg_flops(fn, a)
        d = kernels[kn]
        if b:
            r["b"] += b
            d["b"] += b
            d["nb"] += 1
            d["ms_b"] += slot[top][0]
        else:
            r["nb"] = True
        if f:
            r["f"] += f
            d["f"] += f
            d["nf"] += 1
            d["ms_f"] += slot[top][0]
        else:
            r["nf"] = True
    out_roles = {}
    for role, r in roles.items():
        n = r["launches"]
        out_roles[role] = {"kernel": max(r["k"], key=r["k"].get) if r["k"] else "(no libkair launch)", "launches": n,
                           "ms_total": r["ms_total"], "ms": r["ms_total"] / n,
                           "bytes": None if (r["nb"] or not r["b"]) else r["b"] / n,
                           "flops": None if (r["nf"] or not r["f"]) else r["f"] / n}
    for d in kernels.values():
        n = d["launches"]
        d["ms"] = d["ms_total"] / n
        d["bytes"] = d["b"] / d["nb"] if d["nb"] else None
        d["flops"] = d["f"] / d["nf"] if d["nf"] else None
        d["ms_bytes"] = d["ms_b"] / d["nb"] if d["nb"] else None   # mean duration of the launches those figures cover
        d["ms_flops"] = d["ms_f"] / d["nf"] if d["nf"] else None
        d["attributed"] = max(d["nb"], d["nf"])
        d["roles"] = len(d["roles"])
        for x in ("b", "f", "nb", "nf", "ms_b", "ms_f"):
            del d[x]
    return out_roles, kernels


def pmc_traffic(*keys):
    """HBM bytes per launch of the kernel named by any of `keys` (its symbol, its demangled name) from the newest
    committed rocprofv3 PMC summary (profiles/rNN_pmc_traffic.json, written by tools/pmc_traffic.py: FETCH_SIZE x 2
    per the gfx950 correction + WRITE_SIZE, KiB -> bytes), or None when absent."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_traffic.json")))
    try:
        with open(paths[-1]) as f:
            rec = json.load(f)
        for name, v in rec["kernels"].items():
            # rocprofv3 names: the symbol (possibly cut at 160 characters) or "void (anonymous namespace)::name(args)"
            if any(k and (k == name or k.startswith(name) or (k + "(") in name) for k in keys):
                return v["hbm_bytes_per_launch"]
    except (IndexError, OSError, KeyError, ValueError):
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


def engine_line(dtype, bpg, device, drop_path, steps, warmup, roles=True):
    """Throughput of the same training step on another engine of the same program (same batch, --steps /
    --warmup): "fp32" the exact-f32 MFMA engine (the reference's arithmetic, forward within 1e-7 dB of the
    CPU oracle), "bf16" the 16-bit engine (bf16 MFMA, hi/lo bf16 pairs on the conv inputs and weights), with
    the step's MFMA roofline (train FLOPs / step time vs the engine's dense MFMA peak) and its longest kernels."""
    from kair_amd.engine.trainer import FusedTrainer
    from kair_amd.utils.utils_image import synth_sr_batch
    net = build_net(dtype, drop_path).to(device).train()
    ema = build_net(dtype, drop_path).to(device).eval()
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
    from kair_amd.engine.swinir_engine import swinir_flops
    tf = swinir_flops(net, 48, 48)["train"] * bpg * steps / dt / 1e12
    peak = PEAK_F32_TFLOPS if dtype == "fp32" else PEAK_BF16_TFLOPS
    top = []
    if roles:
        _, ks = time_roles(tr)
        for v in sorted(ks.values(), key=lambda v: -v["ms_total"])[:5]:
            top.append({"kernel": v["kernel"], "launches_per_step": v["launches"], "kernel_ms": round(v["ms"], 5),
                        "step_ms_total": round(v["ms_total"], 4)})
    del tr, net, ema
    return {"value": round(bpg * steps / dt, 2), "unit": "patches/s", "ms_per_step": round(1000 * dt / steps, 3),
            "steps": steps, "warmup": warmup, "dtype": dtype, "per_gpu_batch": bpg, "precision": PRECISION[dtype],
            "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(tf / peak, 4),
                         "what": "whole training step: train FLOPs per patch (swinir_flops) x patches/s vs the dense MFMA "
                                 "peak of the engine's operand type"},
            "kernels_by_duration": top}


def psnr_parity(net_gpu, device, dtype, n_eval=8):
    """PSNR of the GPU forward vs the CPU oracle on the same (trained) weights, DropPath off (eval),
    averaged per image over n_eval held-out 48-px patches as the reference's test loop averages
    (main_train_psnr.py: avg_psnr over the test set), float and uint8 / border-4; the largest single-image
    deviation beside the means.

    The exact-fp32 engine and the fp32x3 engine (the headline) must match the oracle to 1e-3 dB; a bf16
    engine's deviation is reported the same way.  One patch alone is not an evaluation set: bf16 activation
    rounding moves a single 192x192 uint8 PSNR by up to ~1e-3 dB either way, the 8-patch mean by ~3e-4
    (tools/parity_seeds.py, DESIGN.md "parity at bf16")."""
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
    (hf, hu), (ff, fu), (rf, ru) = per_image(E), per_image(E32), per_image(Er)
    mean = lambda v: sum(v) / len(v)
    dmax = lambda a, b: max(abs(x - y) for x, y in zip(a, b))
    return {"eval": f"{n_eval} held-out 48-px LQ patches (synth seed 77), per-image PSNR averaged",
            "headline_dtype": dtype, "cpu_oracle_db": round(mean(rf), 5),
            "headline_gpu_db": round(mean(hf), 5), "headline_delta_db": round(abs(mean(hf) - mean(rf)), 7),
            "uint8_border4_cpu_db": round(mean(ru), 5), "uint8_border4_headline_gpu_db": round(mean(hu), 5),
            "uint8_headline_delta_db": round(abs(mean(hu) - mean(ru)), 7),
            "headline_max_single_image_delta_db": round(dmax(hf, rf), 7),
            "uint8_headline_max_single_image_delta_db": round(dmax(hu, ru), 7),
            "max_abs_headline_vs_oracle": float((E - Er).abs().max()),
            "fp32_gpu_db": round(mean(ff), 5), "fp32_delta_db": round(abs(mean(ff) - mean(rf)), 7),
            "uint8_border4_fp32_gpu_db": round(mean(fu), 5), "uint8_fp32_delta_db": round(abs(mean(fu) - mean(ru)), 7),
            "max_abs_fp32_vs_oracle": float((E32 - Er).abs().max())}


OTHER_STEPS, OTHER_WARMUP = 20, 5


# the precision each config's reference option file trains at (models/model_plain.py:31-36: no amp_enabled -> fp32):
# C2 is quoted in bf16 by BASELINE.json itself; C3 (train_usrnet.json) and C5 (train_rrdb_psnr.json) are fp32, so
# they are also timed on the engines of that precision class (REF_DTYPE: fp32x3 where the engine has the split-fp16
# arithmetic -- C5 -- and the exact-fp32 MFMA engine), priced against that engine's MFMA ceiling
REF_DTYPE = {"usrnet": ["fp32"], "rrdbnet": ["fp32x3", "fp32"], "dncnn": ["fp32"]}
CEILING = {"bf16": (PEAK_BF16_TFLOPS, "dense bf16 MFMA peak"), "fp32x3": (PEAK_BF16_TFLOPS / 3, "dense f16 MFMA peak / 3"),
           "fp32": (PEAK_F32_TFLOPS, "dense fp32 MFMA peak")}


def other_configs(device):
    """The other BASELINE.json configs, one short fused-trainer run each (USRNet with (k, sf, sigma) inputs)
    on this GPU (tools/bench_models.py; synthetic seeded inputs resident in HBM): patches/s and the
    fraction of the MFMA ceiling of the engine's arithmetic their training FLOPs reach -- in bf16 and, for the
    configs whose option files train in fp32, at that precision class too (REF_DTYPE).  C1 (DnCNN) is a CPU
    config in the reference; its network's GPU step is reported for completeness."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    import bench_models as bm
    labels = {"swinir_light": "C2 SwinIR-lightweight x2, 64-px LQ, batch 64",
              "usrnet": "C3 USRNet x4, 128-px LQ (512^2 HR), batch 48, n_iter 6",
              "rrdbnet": "C5 RRDBNet x4, 32-px LQ, batch 16 (the N=1 shape of global batch 16)",
              "dncnn": "C1 DnCNN sigma 25, 40x40, batch 64 (GPU step of the CPU config's network)"}
    res = {}
    for name, label in labels.items():
        for dt in ["bf16"] + REF_DTYPE.get(name, []):
            key = name if dt == "bf16" else f"{name}_{dt}"
            try:
                B, sec, loss = bm.run(name, OTHER_STEPS, OTHER_WARMUP, device, dt)
                pps = B / sec
                tf = pps * bm.TRAIN_GFLOP[name] / 1e3
                pk, what = CEILING[dt]
                res[key] = {"config": label, "dtype": dt, "value": round(pps, 2), "unit": "patches/s",
                            "ms_per_step": round(sec * 1e3, 3), "steps": OTHER_STEPS, "warmup": OTHER_WARMUP,
                            "train_gflop_per_patch": bm.TRAIN_GFLOP[name],
                            "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": round(pk, 1), "peak_what": what,
                                         "unit": "TFLOP/s", "frac": round(tf / pk, 4)},
                            "final_loss": round(loss, 6)}
                if dt in REF_DTYPE.get(name, []):
                    res[key]["precision"] = "the reference option file's precision class (fp32)"
            except Exception as e:  # noqa: BLE001
                res[key] = {"config": label, "dtype": dt, "error": repr(e)}
            torch.cuda.empty_cache()
    return res


def launch_plan(gpus, env):
    """How this invocation runs (reference: one process per GPU, main_train_psnr.py:52-54,122-130 /
    utils/utils_dist.py:13-28):
      ("run", W)    already a rank of a W-process launch (torchrun / this script's own spawn): --gpus must
                    equal W, else SystemExit -- a scaling run must never silently time fewer GPUs;
      ("spawn", N)  a plain `python bench.py --gpus N` with N > 1: start N rank processes (before any GPU
                    call in this parent) and wait for them."""
    if gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {gpus})")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}: launch one process per GPU with matching counts")
        return ("run", world)
    return ("spawn", gpus) if gpus > 1 else ("run", 1)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(n, argv):
    """Run `python bench.py argv` as n ranks (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on
    127.0.0.1); rank 0's stdout is the JSON line.  Returns the worst exit code."""
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def dry_run(world, rank):
    """--dry-run: the launch path on the CPU (gloo, no GPU call): every rank reports in to rank 0."""
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
        got = [None] * world
        dist.all_gather_object(got, rank)
    else:
        got = [rank]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": got}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); without torchrun the script spawns them")
    ap.add_argument("--steps", type=int, default=100)   # >= 100 timed steps after >= 20 warm-up
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--global-batch", type=int, default=32)
    ap.add_argument("--per-gpu-batch", type=int, default=None, help="weak scaling: fixed batch per GPU")
    ap.add_argument("--dtype", default="fp32x3", choices=["bf16", "fp32", "fp32x3"],
                    help="fp32x3 (default): the reference's fp32 precision class on the fp16 matrix cores (split pairs); "
                         "bf16: the 16-bit engine; fp32: exact fp32 MFMA")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--drop-path", type=float, default=0.1)
    ap.add_argument("--no-fp32-line", action="store_true", help="skip the other engines' throughput lines")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the short single-GPU throughput lines of BASELINE.json configs C2 / C3 / C5 (and the "
                         "C1 network on the GPU)")
    ap.add_argument("--no-roles", action="store_true", help="skip the in-step per-kernel timing pass")
    ap.add_argument("--no-psnr", action="store_true",
                    help="skip the PSNR parity evaluation (profiling runs: only full-batch dispatches)")
    ap.add_argument("--side-ctas", type=int, default=None,
                    help="A/B: workgroup budget of the side-stream launches (0: uncapped; < 0: that many times more row "
                         "splits; default: the engine's -- 192 for fp32x3, uncapped for bf16)")
    ap.add_argument("--side-priority", type=int, default=0, help="A/B: torch priority of the side stream")
    ap.add_argument("--main-priority", type=int, default=0, help="A/B: torch priority of the step's capture stream")
    ap.add_argument("--no-side-stream", action="store_true",
                    help="A/B: run the deferred per-RSTB gradient work in place on the main stream")
    ap.add_argument("--split-linear", action="store_true",
                    help="A/B: hi/lo split weights in the fused Swin-block linears (SwinIREngine split_linear)")
    ap.add_argument("--conv-wr-min-tiles", type=int, default=None,
                    help="A/B: 96-pixel tiles from which the RSTB convs run on kair_conv3x3_wr (< 0: never)")
    ap.add_argument("--dry-run", action="store_true", help="exercise the rank launch on the CPU (gloo) and exit")
    ap.add_argument("--data", default="pool", choices=["pool", "static"],
                    help="pool: every step synthesises a fresh batch on the GPU from an HBM-resident HR pool "
                         "(kair_synth_sr: crop + 8-way augment + MATLAB bicubic x1/4, DatasetSR semantics) inside "
                         "the timed loop; static: one staged batch reused")
    args = ap.parse_args()

    mode, world = launch_plan(args.gpus, os.environ)
    if mode == "spawn":
        sys.exit(spawn_ranks(world, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dry_run(world, rank)
        return
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
    if args.no_side_stream or args.side_ctas is not None or args.side_priority or args.split_linear:
        from kair_amd.engine.swinir_engine import SwinIREngine
        kw = {"side_stream": not args.no_side_stream, "side_priority": args.side_priority}
        if args.split_linear:
            kw["split_linear"] = True
        if args.side_ctas is not None:
            kw["side_ctas"] = args.side_ctas
        net._engine = SwinIREngine(net, args.dtype, **kw)
    if args.conv_wr_min_tiles is not None:
        eng = net.engine()
        if args.conv_wr_min_tiles < 0:
            eng.conv_wr = False
        eng.conv_wr_min_tiles = max(0, args.conv_wr_min_tiles)
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999, use_graph=not args.no_graph, stream_priority=args.main_priority)
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
    tr.check_range()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        loss = tr.step(*batch())
    tr.check_range()   # fp32x3 range guard: the last step's flag (every earlier one is settled inside step())
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
    # the MFMA ceiling a FLOP of this engine is priced against: bf16 the dense bf16 peak; fp32x3 issues THREE fp16
    # products per fp32 FLOP on the f16 pipe (2.5 PF dense), so its ceiling is 2.5 PF / 3; exact fp32 the fp32 peak
    peak = {"bf16": PEAK_BF16_TFLOPS, "fp32x3": PEAK_BF16_TFLOPS / 3, "fp32": PEAK_F32_TFLOPS}[args.dtype]
    peak_what = {"bf16": "dense bf16 MFMA peak (2.5 PF)",
                 "fp32x3": "dense f16 MFMA peak / 3 (2.5 PF / 3 = 833 TF: three fp16 products per fp32 FLOP)",
                 "fp32": "dense fp32 MFMA peak (157.3 TF)"}[args.dtype]
    roles, kernels, roles_err = {}, {}, None
    if not args.no_roles:
        try:
            roles, kernels = time_roles(tr)
        except Exception as e:  # noqa: BLE001
            roles_err = repr(e)
    TIMING = ("kernel duration as rocprofv3 --kernel-trace reports it (the dispatch packet's start / end timestamps, "
              "hipExtLaunchKernel event pairs of a kair_ktime window), mean per launch over an eager fwd+loss+bwd pass "
              "of the timed configuration with the step's side-stream concurrency, queued whole behind a held wave "
              "(kair_gate_hold) and released at once so it runs back to back as the graph-replayed step does "
              "(bench.time_roles)")

    def roof(d, role=None):
        r = {"bound": "hbm", "kernel": d["kernel"], "launches_per_step": d["launches"], "kernel_ms": round(d["ms"], 5),
             "step_ms_total": round(d["ms_total"], 4)}
        if role is not None:
            r["role"] = role
        else:
            r.update({"roles": d["roles"], "symbol": d["symbol"], "attributed_launches": d["attributed"]})
        # the figures cover the launches they were attributed to: all of them (then their mean is the kernel's), or
        # the attributed ones' own mean duration
        ms_b = d["ms"] if role is not None else d.get("ms_bytes")
        ms_f = d["ms"] if role is not None else d.get("ms_flops")
        if d.get("bytes") and ms_b:
            gbs = d["bytes"] / (ms_b * 1e-3) / 1e9
            r.update({"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4),
                      "bytes_per_launch": round(d["bytes"]),
                      "traffic": pmc_traffic(d["symbol"], d["kernel"]) if role is None else None})
        else:
            r.update({"achieved": None, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": None, "traffic": None})
        if d.get("flops") and ms_f:
            tf = d["flops"] / (ms_f * 1e-3) / 1e12
            r.update({"flops_per_launch": d["flops"], "achieved_tflops": round(tf, 2), "mfma_frac": round(tf / peak, 4),
                      "mfma_peak": peak_what})
            if args.dtype == "fp32x3":
                r["frac_of_fp32_peak"] = round(tf / PEAK_F32_TFLOPS, 4)
        return r
    ranked = sorted(roles.items(), key=lambda kv: -kv[1]["ms_total"])
    kranked = sorted(kernels.values(), key=lambda v: -v["ms_total"])
    # attention GEMMs (QKV / q.k^T / p.v / proj): the fused attention half, the attention backward, the proj and
    # q/k/v input-gradient row GEMMs (bf16) / the split window-attention kernels (fp32x3) -- FLOPs over their
    # in-step time against the engine's MFMA ceiling
    att_names = ("swin_attn_fwd", "attn_bwd_bf16_kernel", "rowgemm_kernel<12, 4, 2, 0", "rowgemm_kernel<36",
                 "attn_fwd_x3_kernel", "attn_bwd_x3_kernel")
    att = [v for v in kernels.values() if v.get("flops") and v["kernel"].startswith(att_names) and v["ms_flops"]]
    att_mfma = None
    if att:
        fl_att = sum(v["flops"] * v["attributed"] for v in att)
        ms_att = sum(v["ms_flops"] * v["attributed"] for v in att)
        tf = fl_att / (ms_att * 1e-3) / 1e12
        att_mfma = {"kernels": sorted(v["kernel"] for v in att), "flops_per_step": fl_att, "ms_per_step": round(ms_att, 4),
                    "achieved_tflops": round(tf, 2), "peak_tflops": round(peak, 1), "peak": peak_what,
                    "mfma_frac": round(tf / peak, 4)}
        if args.dtype == "fp32x3":
            att_mfma["frac_of_fp32_peak"] = round(tf / PEAK_F32_TFLOPS, 4)
    out = {
        "metric": "train patches/sec + PSNR, SwinIR x4 48-px LQ, at 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "patches/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
        "dtype": args.dtype,
        "precision": PRECISION[args.dtype],
        "data": ("synthetic: per step a fresh batch synthesised on the GPU (crop / augment / MATLAB bicubic) from "
                 "a 64-image 256x256 HR pool resident in HBM (SURVEY §8d recipe)" if args.data == "pool" else
                 "synthetic (one seeded bicubic-LR / HR batch resident in HBM, SURVEY §8d)"),
        "config": {"workload": "SwinIR classical x4 SR train step (fwd+L1+bwd+allreduce+Adam+EMA), 48-px LQ",
                   "global_batch": gbatch, "per_gpu_batch": bpg, "lq": 48, "hr": 192, "embed_dim": 180,
                   "depths": [6] * 6, "heads": 6, "window": 8, "drop_path_rate": args.drop_path,
                   "parallelism": f"dp{world}", "hip_graph": not args.no_graph},
        # roofline: the step's dominant kernel -- the kernel (template instantiation, all its call sites) with the
        # largest summed duration in the step, as rocprofv3 ranks the bench command's kernels
        "roofline": ({**roof(kranked[0]), "kernel_ms_timing": TIMING} if kranked else
                     {"error": roles_err or "roles skipped"}),
        "kernels_by_duration": [roof(v) for v in kranked[:10]],
        "roles_by_duration": [roof(v, k) for k, v in ranked[:12]],
        "attention_gemm_mfma": att_mfma,
        "step_roofline": {"train_flop_per_patch": fl["train"], "achieved_tflops_per_gpu": round(step_tflops, 2),
                          "peak_tflops": round(peak, 1), "peak": peak_what, "frac_of_peak": round(step_tflops / peak, 4),
                          **({"frac_of_fp32_peak": round(step_tflops / PEAK_F32_TFLOPS, 4)}
                             if args.dtype == "fp32x3" else {})},
        "range_guard": ({"events": tr.range_events, "act_exp": tr.engine.X3_AEXP, "grad_exp_offset": tr.engine.x3_gexp_off}
                        if getattr(tr, "range_guard", False) else None),
        "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
        "final_loss": round(final_loss, 6),
    }
    if world == 1 and not args.no_fp32_line:   # the other engines of the same program, same step
        for dt in ("fp32", "bf16"):
            if dt == args.dtype:
                continue
            try:
                out[f"{dt}_engine_line"] = engine_line(dt, bpg, device, args.drop_path, args.steps, args.warmup,
                                                      roles=not args.no_roles)
            except Exception as e:  # noqa: BLE001
                out[f"{dt}_engine_line"] = {"error": repr(e)}
    if not args.no_psnr:
        try:
            out["psnr"] = psnr_parity(net, device, args.dtype)
        except Exception as e:  # noqa: BLE001
            out["psnr"] = {"error": repr(e)}
    if world == 1 and not args.no_other_configs:
        out["other_configs"] = other_configs(device)
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline()
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
