"""MFMA utilisation and HBM rate of the SwinIR attention GEMMs (QKV, q.k^T, p.v, proj; forward and
backward) from a rocprofv3 kernel trace of `bench.py` (classical x4, B = 32 per GPU).

    python tools/attn_mfma.py gpurun_out/prof/run_kernel_trace.csv [out.json]

Each training step is the stretch between two adam_ema launches; inside it the L1-loss kernel
splits forward from backward.  Roles are told apart by kernel instance and, where one instance
serves two roles, by position:
  forward   gemm_nt_ring<192,5,0,1,0> = QKV, attn_fwd = q.k^T + p.v, the first residual ring GEMM
            after it = proj (fc2 is the second)
  backward  after each fc2 dgrad (gemm_nt_ring<192,5,0,0,2>) the second gemm_nt_ring<96,5,0,0,0> is
            proj dgrad (the first is fc1 dgrad; with KAIR_RING_SPLIT_N=0 proj dgrad is
            gemm_nt_ring<192,5,0,0,0>),
            gemm_tn_ring<0> #3 of each block = proj wgrad,
            attn_bwd = the five attention products, gemm_nt_ring<64,5,2,0,0> = QKV dgrad,
            gemm_tn_ring<2> = QKV wgrad (+ the wgrad_finalize that follows each wgrad)
FLOPs and bytes are algorithmic at the reference dims (C = 180, 6 heads x 30, 64-token windows):
network_swinir.py:114-145 (WindowAttention.forward), 121 (qkv), 142 (proj).
"""
import csv
import json
import sys

PEAK_TFLOPS = 2500.0   # dense bf16 MFMA, MI355X_MICROARCH.md
PEAK_GBS = 8000.0
B, HW, C, N3, WT = 32, 48 * 48, 180, 540, 64
M = B * HW

ROLES = {   # role: (flops per launch, algorithmic HBM bytes per launch)
    "qkv_fwd": (2 * M * N3 * C, M * (C + N3) * 2 + N3 * C * 2),
    "attn_fwd": (2 * 2 * M * WT * C, M * N3 * 2 + M * C * 2 + M * 6 * 4),
    "proj_fwd": (2 * M * C * C, M * C * 2 + 2 * M * C * 4 + C * C * 2),
    "proj_dgrad": (2 * M * C * C, 2 * M * C * 2 + C * C * 2),
    "proj_wgrad": (2 * M * C * C, 2 * M * C * 2 + C * C * 4),
    "attn_bwd": (5 * 2 * M * WT * C, M * N3 * 2 * 2 + 2 * M * C * 2 + M * 6 * 4),
    "qkv_dgrad": (2 * M * N3 * C, M * N3 * 2 + M * C * 4 + N3 * C * 2),
    "qkv_wgrad": (2 * M * N3 * C, M * (N3 + C) * 2 + N3 * C * 4),
}


def _ring(name, em, ex):
    """gemm_nt_ring<BN, 5, 0, em, ex> with BN 96 or 192 (K <= 192 GEMMs split N into two 96-wide
    tiles unless KAIR_RING_SPLIT_N=0)."""
    return any(f"gemm_nt_ring<{bn}, 5, 0, {em}, {ex}>" in name for bn in (96, 192))


class Classifier:
    """Per-step state: proj fwd is the first residual ring GEMM after each attn_fwd (fc2 fwd is the
    second); see the module docstring for the backward."""

    def __init__(self):
        self.in_bwd, self.tn0, self.after_attn, self.plain_bwd = False, 0, False, 0

    def __call__(self, name):
        if "l1_kernel" in name:
            self.in_bwd = True
            return None
        if "gemm_nt_ring<192, 5, 0, 1, 0>" in name:
            return "qkv_fwd" if not self.in_bwd else None
        if "attn_fwd_bf16_kernel" in name:
            self.after_attn = True
            return "attn_fwd" if not self.in_bwd else None
        if _ring(name, 0, 1) and not self.in_bwd:
            first, self.after_attn = self.after_attn, False
            return "proj_fwd" if first else None
        if self.in_bwd and "gemm_nt_ring<192, 5, 0, 0, 2>" in name:   # fc2 dgrad opens a block backward
            self.plain_bwd = 0
            return None
        if self.in_bwd and "gemm_nt_ring<96, 5, 0, 0, 0>" in name:     # fc1 dgrad, then (split-N) proj dgrad
            self.plain_bwd += 1
            return "proj_dgrad" if self.plain_bwd == 2 else None
        if self.in_bwd and "gemm_nt_ring<192, 5, 0, 0, 0>" in name:    # proj dgrad (KAIR_RING_SPLIT_N=0)
            return "proj_dgrad"
        if "gemm_tn_ring<0>" in name and self.in_bwd:
            self.tn0 += 1
            return "proj_wgrad" if self.tn0 % 3 == 0 else None
        if "attn_bwd_bf16_kernel" in name:
            return "attn_bwd"
        if "gemm_nt_ring<64, 5, 2, 0, 0>" in name:
            return "qkv_dgrad"
        if "gemm_tn_ring<2>" in name:
            return "qkv_wgrad"
        return None


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps = [i for i, r in enumerate(rows) if "adam_ema" in r["Kernel_Name"]]
    dur = {k: [] for k in ROLES}
    fin = {"proj_wgrad": [], "qkv_wgrad": []}
    for a, b in zip(steps[:-1], steps[1:]):
        cls, pending = Classifier(), None
        for r in rows[a + 1:b]:
            n = r["Kernel_Name"]
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            if pending and "wgrad_finalize" in n:
                fin[pending].append(d)
                pending = None
                continue
            role = cls(n)
            if role:
                dur[role].append(d)
                pending = role if role in fin else None
    res, tf, tt = {}, 0.0, 0.0
    for k, (fl, by) in ROLES.items():
        if not dur[k]:
            continue
        us = sum(dur[k]) / len(dur[k]) / 1e3
        if k in fin and fin[k]:
            us_fin = sum(fin[k]) / len(fin[k]) / 1e3
        else:
            us_fin = 0.0
        t = us + us_fin
        ai = fl / by
        res[k] = {"launches": len(dur[k]), "avg_us": round(us, 2), "finalize_us": round(us_fin, 2),
                  "gflop": round(fl / 1e9, 3), "tflops": round(fl / t / 1e6, 1),
                  "mfma_frac": round(fl / t / 1e6 / PEAK_TFLOPS, 4),
                  "alg_GBs": round(by / t / 1e3, 1), "hbm_frac": round(by / t / 1e3 / PEAK_GBS, 4),
                  "flop_per_byte": round(ai, 1),
                  "mfma_ceiling_at_hbm_peak": round(min(1.0, ai * PEAK_GBS / 1e3 / PEAK_TFLOPS), 4)}
        tf += fl * len(dur[k])
        tt += t * len(dur[k])
    summary = {"source": path, "batch": B, "peak_tflops_bf16_dense": PEAK_TFLOPS, "peak_hbm_GBs": PEAK_GBS,
               "attention_gemms_mfma_frac": round(tf / tt / 1e6 / PEAK_TFLOPS, 4),
               "attention_gemms_tflops": round(tf / tt / 1e6, 1), "roles": res}
    print(json.dumps(summary, indent=1))
    if out:
        json.dump(summary, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
