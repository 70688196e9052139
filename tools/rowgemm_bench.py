"""A/B timing of the Swin-block input-gradient products: the round-2 path (hipBLASLt / kair_gemm_nt +
kair_layernorm_bwd) against the fused row GEMMs (kair_rowgemm_*), at the classical x4 block's shapes.

    python tools/rowgemm_bench.py [--batch 32 4] [--reps 20]

Each variant rotates over 3 independent operand sets (> the 256 MB Infinity Cache at B = 32) so the
launches read HBM as they do inside a step.  Prints one JSON line per (batch, product)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402

dev = torch.device("cuda", 0)
C, CP, HD, HDP, NH = 180, 192, 360, 384, 6


def lin(N, K, n_grp, k_grp):
    w = torch.randn(N, K, device=dev) * 0.05
    Np, Kp = n_grp[0] * n_grp[2], k_grp[0] * k_grp[2]
    frag = torch.empty(Kp, Np, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w, frag, H.wmap(13, N, K, n_grp, k_grp))
    wt = torch.empty(Kp, Np, device=dev, dtype=torch.bfloat16)      # kind 3: the unfused dgrad operand
    H.pack_weight(w, wt, H.wmap(3, N, K, n_grp, k_grp))
    return frag, wt


def timed(fn, sets, reps):
    for i in range(3):
        fn(sets[i % len(sets)])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(sets[i % len(sets)])
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[32, 4])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    Hh = Ww = 48
    for B in a.batch:
        M = B * Hh * Ww
        win1 = (Hh, Ww, 8, 4)
        mk = lambda *s, dt=torch.bfloat16: torch.randn(*s, device=dev).to(dt)
        sets = []
        for _ in range(3):
            x = torch.zeros(M, CP, device=dev)
            x[:, :C] = torch.randn(M, C, device=dev)
            sets.append({"Da": mk(M, CP), "dU": mk(M, HDP), "dqkv": mk(M, 3 * NH * 32), "Dm": mk(M, CP),
                         "g": mk(M, HDP), "x": x, "D": torch.randn(M, CP, device=dev),
                         "mean": torch.randn(M, device=dev), "rstd": torch.rand(M, device=dev) + 0.5,
                         "dO": mk(M, CP), "dxn": mk(M, CP), "cp": mk(M, CP), "dUo": mk(M, HDP)})
        gamma = torch.randn(C, device=dev)
        proj = lin(C, C, (1, C, CP), (NH, C // NH, 32))
        fc1 = lin(HD, C, (1, HD, HDP), (1, C, CP))
        qkv = lin(3 * C, C, (3 * NH, C // NH, 32), (1, C, CP))
        fc2 = lin(C, HD, (1, C, CP), (1, HD, HDP))
        ws_ln = torch.empty(2 * 2048 * CP, device=dev)
        nb = max(H.rowgemm_ln_blocks(M, 384), H.rowgemm_ln_blocks(M, 576))
        part = torch.empty(nb * 2 * C, device=dev)
        res = {}

        # proj input gradient: dO = Da . Wproj
        res["proj_dgrad"] = {
            "old_hipblaslt_us": timed(lambda s: torch.matmul(s["Da"], proj[1].t(), out=s["dO"]), sets, a.reps),
            "new_us": timed(lambda s: H.rowgemm_store(s["Da"], M, CP, proj[0], CP, s["dO"]), sets, a.reps),
            "bytes": M * CP * 2 * 2}

        # fc1 input gradient + LN2 backward (+ the window-order proj operand copy)
        def old_fc1(s):
            torch.matmul(s["dU"], fc1[1].t(), out=s["dxn"])
            H.layernorm_bwd(s["x"], CP, s["dxn"], CP, gamma, s["mean"], s["rstd"], s["D"], CP, True, None, None, False,
                            ws_ln, M, C, copy=H.copy_desc(s["cp"], win=win1))

        def new_fc1(s):
            H.rowgemm_lnbwd(s["dU"], M, HDP, fc1[0], s["x"], gamma, s["mean"], s["rstd"], C, s["D"], part,
                            copy=H.copy_desc(s["cp"], win=win1))
        res["fc1_dgrad_ln2"] = {"old_us": timed(old_fc1, sets, a.reps), "new_us": timed(new_fc1, sets, a.reps),
                                "bytes": M * (HDP * 2 + CP * 4 * 3 + CP * 2 + 8)}

        # q/k/v input gradient + LN1 backward (rows in window order, copy in token order)
        def old_qkv(s):
            torch.matmul(s["dqkv"], qkv[1].t(), out=s["dxn"])
            H.layernorm_bwd(s["x"], CP, s["dxn"], CP, gamma, s["mean"], s["rstd"], s["D"], CP, True, None, None, False,
                            ws_ln, M, C, win1, copy=H.copy_desc(s["cp"]))

        def new_qkv(s):
            H.rowgemm_lnbwd(s["dqkv"], M, 3 * NH * 32, qkv[0], s["x"], gamma, s["mean"], s["rstd"], C, s["D"], part,
                            win=win1, copy=H.copy_desc(s["cp"]))
        res["qkv_dgrad_ln1"] = {"old_us": timed(old_qkv, sets, a.reps), "new_us": timed(new_qkv, sets, a.reps),
                                "bytes": M * (3 * NH * 32 * 2 + CP * 4 * 3 + CP * 2 + 8)}

        # fc2 input gradient through the stored GELU' gate
        def old_fc2(s):
            H.gemm_nt(H.rows(s["Dm"]), H.rows(fc2[1]), H.epilogue(s["dUo"], gate=s["g"], gate_kind=4), M, HDP, CP, H.BF16)
        res["fc2_dgrad_gate"] = {
            "old_ring_us": timed(old_fc2, sets, a.reps),
            "new_us": timed(lambda s: H.rowgemm_gate(s["Dm"], M, CP, fc2[0], HDP, s["g"], s["dUo"]), sets, a.reps),
            "bytes": M * (CP * 2 + HDP * 2 * 2)}
        for k, v in res.items():
            new = v["new_us"]
            v["new_TBps"] = round(v["bytes"] / (new * 1e-6) / 1e12, 3)
            print(json.dumps({"batch": B, "M": M, "product": k, **{kk: (round(vv, 2) if isinstance(vv, float) else vv)
                                                                    for kk, vv in v.items()}}), flush=True)


if __name__ == "__main__":
    main()
