"""Isolated 3x3 halo conv launches at the SwinIR classical x4 B = 32 shapes (M = 73,728 LQ pixels):
the RSTB conv forward over an fp32 image with split weights and split activations (two passes, three
products), the same over a bf16 image (one pass, two products), its input gradient (bf16, flipped taps,
one product), and the upsampling conv (64 -> 256 over the 96 x 96 image, [hi | lo] pair input).
Prints per-launch time and MFMA TFLOP/s (products counted).  For rocprofv3 PMC passes.

    python tools/conv_micro.py [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402

dev = torch.device("cuda", 0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20


def timeit(f):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000


def split_w(Cout, Cin, Cop, Cig, kG=1, n_perm=0):
    """Cig: the padded input channels of one group (kG groups: [hi | lo] pair images)"""
    w = torch.randn(Cout, Cin, 3, 3, device=dev) * 0.05
    W = torch.empty(Cop, 2 * ((9 * Cig * kG + 63) // 64) * 64, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w, W, H.wmap(9, Cout, Cin, (1, Cout, Cop), (kG, Cin, Cig), n_perm=n_perm))
    return W


B, Hh, Ww, C, Cp = 32, 48, 48, 180, 192
M = B * Hh * Ww
x32 = torch.randn(M, Cp, device=dev)
x16 = x32.bfloat16()
out = torch.empty(M, Cp, device=dev)
resid = torch.randn(M, Cp, device=dev)
bias = torch.zeros(Cp, device=dev)
Ws = split_w(C, C, Cp, Cp)
Wd = torch.randn(Cp, 9 * Cp, device=dev).bfloat16()
fl = 2.0 * M * Cp * 9 * Cp

rows = []
t = timeit(lambda: H.gemm_nt(H.asplit(H.im2col(x32, Hh, Ww, Cp)), H.rows(Ws, w_split=True),
                             H.epilogue(out, bias=bias, resid=resid), M, Cp, 9 * Cp, H.BF16))
rows.append(("rstb fwd fp32 2-pass (3 products)", t, 3 * fl))
t = timeit(lambda: H.gemm_nt(H.im2col(x16, Hh, Ww, Cp), H.rows(Ws, w_split=True),
                             H.epilogue(out, bias=bias, resid=resid), M, Cp, 9 * Cp, H.BF16))
rows.append(("rstb fwd bf16 (2 products)", t, 2 * fl))
t = timeit(lambda: H.gemm_nt(H.im2col(x16, Hh, Ww, Cp, flip=True), H.rows(Wd), H.epilogue(out), M, Cp, 9 * Cp, H.BF16))
rows.append(("rstb dgrad bf16 (1 product)", t, fl))
t = timeit(lambda: H.gemm_nt(H.im2col(x32, Hh, Ww, Cp, flip=True), H.rows(Wd), H.epilogue(out), M, Cp, 9 * Cp, H.BF16))
rows.append(("rstb dgrad fp32 G (1 product)", t, fl))
# the register-streamed-weight kernel (csrc/conv_wr.hip) on the same shapes
w32 = torch.randn(C, C, 3, 3, device=dev) * 0.05
Wf = torch.empty(192 * 2 * 9 * Cp, device=dev, dtype=torch.bfloat16)
H.pack_weight(w32, Wf, H.wmap(15, C, C, (1, C, Cp), (1, C, Cp)))
Wdf = torch.empty(192 * 9 * Cp, device=dev, dtype=torch.bfloat16)
H.pack_weight(w32, Wdf, H.wmap(16, C, C, (1, C, Cp), (1, C, Cp)))
ac = torch.empty(M, Cp, device=dev, dtype=torch.bfloat16)
t = timeit(lambda: H.conv3x3_wr(x32, Cp, 0, Wf, bias, resid, out, B, Hh, Ww, Cp, Cp, acopy=ac, acones=C))
rows.append(("wr: rstb fwd fp32 split (3 products)", t, 3 * fl))
t = timeit(lambda: H.conv3x3_wr(x16, Cp, 1, Wdf, None, None, out, B, Hh, Ww, Cp, Cp))
rows.append(("wr: rstb dgrad bf16 (1 product)", t, fl))
t = timeit(lambda: H.conv3x3_wr(x32, Cp, 1, Wdf, None, None, out, B, Hh, Ww, Cp, Cp, acopy=ac, split=False))
rows.append(("wr: rstb dgrad fp32 G + a_copy (1 product)", t, fl))
# upsampling conv 2 of x4: 64 -> 256 over 96 x 96, [hi | lo] pair input, PixelShuffle output
h2, w2 = 96, 96
M2 = B * h2 * w2
pair = torch.randn(M2, 128, device=dev).bfloat16()
Wu = split_w(256, 64, 256, 64, kG=2, n_perm=4)
ups = torch.empty(M2 * 4, 128, device=dev, dtype=torch.bfloat16)
t = timeit(lambda: H.gemm_nt(H.asplit(H.im2col(pair, h2, w2, 128), pair=True), H.rows(Wu, w_split=True),
                             H.epilogue(ups, mode=H.OUT_PSHUF_SPM, ldo=128, ps=(2, h2, w2), out_lo=ups[:, 64:]),
                             M2, 256, 9 * 128, H.BF16))
rows.append(("ups conv pair 64->256 @96^2 (3 products)", t, 3 * 2.0 * M2 * 256 * 9 * 64))
for name, t, f in rows:
    print("%-44s %8.1f us %7.1f TFLOP/s (%.3f of 2.5 PF)" % (name, t, f / t * 1e-6, f / t * 1e-6 / 2500))

# the x4 upsampling conv's input gradient at 96^2: 256 -> 64, PixelUnshuffle store (wr) vs the halo kernel's
# four channel-group passes
Gd = torch.randn(M2, 256, device=dev).bfloat16()
w_up = torch.randn(256, 64, 3, 3, device=dev) * 0.03
Wd16 = torch.empty(64 * 9 * 256, device=dev, dtype=torch.bfloat16)
H.pack_weight(w_up, Wd16, H.wmap(16, 256, 64, (1, 256, 256), (1, 64, 64), n_perm=4))
Wd2 = torch.empty(64, 9 * 256, device=dev, dtype=torch.bfloat16)
H.pack_weight(w_up, Wd2, H.wmap(2, 256, 64, (1, 256, 256), (1, 64, 64), n_perm=4))
dprev = torch.empty(M2 // 4, 256, device=dev, dtype=torch.bfloat16)
fl_d = 2.0 * M2 * 64 * 9 * 256
t = timeit(lambda: H.gemm_nt(H.im2col(Gd, h2, w2, 256, flip=True), H.rows(Wd2),
                             H.epilogue(dprev, mode=H.OUT_PUNSHUF_SPM, ldo=256, ps=(2, h2 // 2, w2 // 2)), M2, 64, 9 * 256,
                             H.BF16))
print("%-44s %8.1f us %7.1f TFLOP/s (%.3f of 2.5 PF)" % ("ups dgrad 256->64 @96^2 halo CG", t, fl_d / t * 1e-6, fl_d / t * 1e-6 / 2500))
t = timeit(lambda: H.conv3x3_wr(Gd, 256, 1, Wd16, None, None, dprev, B, h2, w2, 256, 64, ldo=256, split=False, ps_r=-2))
print("%-44s %8.1f us %7.1f TFLOP/s (%.3f of 2.5 PF)" % ("wr: ups dgrad 256->64 @96^2 punshuf", t, fl_d / t * 1e-6, fl_d / t * 1e-6 / 2500))
