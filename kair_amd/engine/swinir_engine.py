"""SwinIR step program for MI355X: the whole forward and backward of network_swinir.py as an
explicit sequence of libkair_hip launches over preallocated HBM buffers.

Reference call stack replaced: SwinIR.forward network_swinir.py:805-839 ->
forward_features :790-803 -> RSTB.forward :481-482 -> SwinTransformerBlock.forward :239-279 ->
WindowAttention.forward :114-145 / Mlp.forward :24-30.

Layout: tokens are rows of NHWC matrices; channels padded C -> Cp (a multiple of
32 with at least one spare column that serves as the fused bias-gradient "ones" column); heads
padded hd -> 32; MLP hidden Hd -> Hdp.  The residual stream and every tensor a LayerNorm reads
are fp32; GEMM operands are bf16 (or fp32 in parity mode); accumulation is fp32.  Window
partition + cyclic shift never materialise: LayerNorm-1 writes window-ordered rows, the proj
epilogue scatters back to token order.  PixelShuffle is a store remap of the upsampling conv.

The program is launch-only (no host syncs, no allocation after planning), so a whole training
step can be captured in a HIP graph (kair_amd/engine/trainer.py).
"""
import contextlib
import math
import os
import weakref

import torch

from .. import _hip as H
from .plans import Lease, PlanPool, autograd_mode, plan_mode

WS_TOK = 64


def _rup(x, m):
    return (x + m - 1) // m * m


def swinir_flops(net, Hh, Ww):
    """Dense-contraction FLOPs per patch (GEMM + conv, 2 per MAC), the quantity FlopCounterMode
    reports (60.25 G fwd / 180.73 G train for classical x4 @48)."""
    C = net.embed_dim
    HW = Hh * Ww
    f = 2 * HW * 9 * net.conv_first.in_channels * C                       # conv_first
    def resi(m):   # '1conv' / '3conv' residual-connection convs
        if isinstance(m, torch.nn.Sequential):
            q = m[0].out_channels
            return 2 * HW * (9 * C * q + q * q + 9 * q * C)
        return 2 * HW * 9 * C * C

    for layer in net.layers:
        for blk in layer.residual_group.blocks:
            Hd = blk.mlp.fc1.out_features
            f += 2 * HW * C * 3 * C + 2 * HW * C * C                      # qkv, proj
            f += 2 * 2 * HW * (blk.window_size ** 2) * C                 # q k^T, p v
            f += 2 * 2 * HW * C * Hd                                     # fc1, fc2
        f += resi(layer.conv)                                             # RSTB conv
    f += resi(net.conv_after_body)                                        # conv_after_body
    first_dgrad = 2 * HW * 9 * net.conv_first.in_channels * C
    if net.upsampler == "nearest+conv":
        nf = 64
        f += 2 * HW * 9 * C * nf + 2 * (4 * HW + 16 * HW + 16 * HW) * 9 * nf * nf + 2 * 16 * HW * 9 * nf * net.conv_last.out_channels
    elif net.upsampler in (None, ""):
        f += 2 * HW * 9 * C * net.conv_last.out_channels
    elif net.upsampler == "pixelshuffle":
        nf = 64
        f += 2 * HW * 9 * C * nf
        hw = HW
        for m in net.upsample:
            if isinstance(m, torch.nn.Conv2d):
                f += 2 * hw * 9 * nf * m.out_channels
                hw *= m.out_channels // nf
        f += 2 * hw * 9 * nf * net.conv_last.out_channels
    else:
        conv = net.upsample[0]
        f += 2 * HW * 9 * C * conv.out_channels
    return {"fwd": f, "train": 3 * f - first_dgrad}


class _Lin:
    """A linear layer's packed forms.  n/k groupings map reference rows/cols to padded ones."""

    def __init__(self, eng, mod, n_grp, k_grp, frag=False, split=False, frag_t=False, rows=True, frag16=False):
        """rows: pack the plain [Np][Kp] form (the unfused forward GEMM's operand); frag / frag_t: the
        fragment-order forms of the fused forward / MLP-backward kernels, which replace [Np][Kp] /
        [Kp][Np]; frag16: the frag form in 16x16x32 fragment order (pack kind 14, the fused MLP
        kernel's fc2 operand) unless split.  Forms no kernel of the engine reads are not packed
        (kair_pack_weights per step)."""
        self.w, self.b = mod.weight, mod.bias
        N, K = self.w.shape[:2]      # nn.Linear [N, K] or a 1x1 nn.Conv2d [N, K, 1, 1]
        self.N, self.K = N, K
        self.map = H.wmap(0, N, K, n_grp, k_grp)
        self.mapT = H.wmap(3, N, K, n_grp, k_grp)
        self.mapb = H.wmap(4, N, 0, n_grp, (1, 1, 1))
        self.Np = n_grp[0] * n_grp[2]
        self.Kp = k_grp[0] * k_grp[2]
        dev = self.w.device
        # fp32x3 engine: the rows forms hold fp16 pairs of w 2^KAIR_X3_WEXP interleaved per 64 columns (pack
        # kinds 17 / 19), multiplied hi.hi + hi.lo + lo.hi by kair_gemm_nt (compute KAIR_COMPUTE_X3)
        self.x3 = getattr(eng, "x3", False)
        if self.x3:   # (self.map stays the plain kind-0 map: the weight gradient's finalize layout)
            self.pmap, self.pmapT = H.wmap(17, N, K, n_grp, k_grp), H.wmap(19, N, K, n_grp, k_grp)
            self.Wp = torch.empty(self.Np, 2 * _rup(self.Kp, 64), device=dev, dtype=torch.float16) if rows else None
            self.Wt = torch.empty(self.Kp, 2 * _rup(self.Np, 64), device=dev, dtype=torch.float16) if not frag_t else None
        else:
            self.pmap, self.pmapT = self.map, self.mapT
            self.Wp = torch.empty(self.Np, self.Kp, device=dev, dtype=eng.tdt) if rows else None
            self.Wt = torch.empty(self.Kp, self.Np, device=dev, dtype=eng.tdt) if not frag_t else None
        self.bp = torch.empty(self.Np, device=dev)
        # MFMA-fragment order of Wp for the fused block kernels: pack kind 10, or kind 12 (hi/lo
        # bf16 pairs, the same ~16-bit weight precision as the split convs) when split
        self.split = bool(frag and split)
        self.mapg = H.wmap(12 if self.split else (14 if frag16 else 10), N, K, n_grp, k_grp) if frag else None
        self.Wg = (torch.empty((2 if self.split else 1) * self.Np, self.Kp, device=dev, dtype=eng.tdt)
                   if frag else None)
        # transposed fragment order (pack kind 13) for the fused MLP backward
        self.mapgt = H.wmap(13, N, K, n_grp, k_grp) if frag_t else None
        self.Wgt = torch.empty(self.Kp, self.Np, device=dev, dtype=eng.tdt) if frag_t else None

    def pack_jobs(self):
        w, b = self.w.detach(), self.b.detach()
        jobs = [(b, self.bp, self.mapb)]
        if self.Wp is not None:
            jobs.append((w, self.Wp, self.pmap))
        if self.Wt is not None:
            jobs.append((w, self.Wt, self.pmapT))
        if self.Wg is not None:
            jobs.append((w, self.Wg, self.mapg))
        if self.Wgt is not None:
            jobs.append((w, self.Wgt, self.mapgt))
        return jobs


class _Conv:
    """A 3x3 conv's packed forms: forward [Cop][9*Cip] and input-gradient [Cip][9*Cop].

    split (bf16 engines): the forward form holds a hi/lo bf16 pair per weight (pack kind 9,
    kair_operand.w_split), so the forward product sees the fp32 master weight to ~16 bits.  Plain
    bf16 weight rounding shifts every output pixel by the same sum(dW * a) and biases PSNR
    (DESIGN.md "parity at bf16"); activation rounding is unbiased and averages out."""

    def __init__(self, eng, mod, Cop, Cip, need_dgrad=True, split=None, n_perm=0, tied_in=False, fwd_cip=None,
                 narrow=False, wr=False):
        """n_perm = r*r: output channels stored sub-pixel-major for a following PixelShuffle(r)
        (kair_wmap.n_perm; the KAIR_OUT_PSHUF_SPM / PUNSHUF_SPM epilogues store 16 bytes at a time).
        tied_in: the forward form repeats the input channels in both halves of Cip (kair_wmap kG = 2),
        for an input held as a hi/lo pair in channels [0, Ci) and [Cip/2, Cip/2 + Ci)
        (kair_image_to_nhwc_hilo); the weight gradient keeps the plain map (the hi channels).
        fwd_cip: the forward form's packed input width when it differs from Cip (a [hi | lo] pair image of
        2 x Cip channels read through tied weights: the SwinIR tail under split_act).
        narrow: a 64 -> NR <= 4 conv run by the narrow-output kernels (kair_conv3x3_narrow_*): its forward
        form is pack kind 15 (16x16x32 fragment order, hi/lo halves), the backward reads the fp32 weight.
        wr: a 192 -> 192 conv also packed for kair_conv3x3_wr: forward pack kind 15, input gradient kind 16."""
        self.w, self.b = mod.weight, mod.bias
        Co, Ci = self.w.shape[:2]
        self.Co, self.Ci, self.Cop, self.Cip = Co, Ci, Cop, Cip
        if split is None:
            split = getattr(eng, "split_conv", False)
        x3 = getattr(eng, "x3", False)   # (the RRDBNet / USRNet engines share this class and have no x3 form)
        self.split = (bool(split) and eng.tdt == torch.bfloat16) or x3
        self.x3 = x3
        self.n_perm = n_perm
        self.map = H.wmap(1, Co, Ci, (1, Co, Cop), (1, Ci, Cip), n_perm=n_perm)
        fcip = fwd_cip or Cip
        self.fcip = fcip
        kf_grp = (2, Ci, fcip // 2) if tied_in else (1, Ci, Cip)
        self.mapf = H.wmap(9 if self.split else 1, Co, Ci, (1, Co, Cop), kf_grp, n_perm=n_perm)
        self.mapd = H.wmap(2, Co, Ci, (1, Co, Cop), (1, Ci, Cip), n_perm=n_perm)
        self.mapb = H.wmap(4, Co, 0, (1, Co, Cop), (1, 1, 1), n_perm=n_perm)
        dev = self.w.device
        kf = 2 * _rup(9 * fcip, 64) if self.split else 9 * fcip
        self.Wf = torch.empty(Cop, kf, device=dev, dtype=torch.float16 if self.x3 else
                              (torch.bfloat16 if self.split else eng.tdt))
        self.narrow = bool(narrow)
        if self.narrow:   # the narrow kernels' forward form (their backward reads the fp32 master weight)
            self.mapn = H.wmap(15, Co, Ci, (1, Co, 16), (1, Ci, Cip))
            self.Wn = torch.empty(16, 2 * 9 * Cip, device=dev, dtype=torch.bfloat16)
        if self.x3:   # fp16 pairs of the dgrad form (pack kind 18)
            self.mapd = H.wmap(18, Co, Ci, (1, Co, Cop), (1, Ci, Cip), n_perm=n_perm)
            self.Wd = torch.empty(Cip, 2 * _rup(9 * Cop, 64), device=dev, dtype=torch.float16) if need_dgrad else None
        else:
            self.Wd = torch.empty(Cip, 9 * Cop, device=dev, dtype=eng.tdt) if need_dgrad else None
        self.bp = torch.empty(Cop, device=dev)
        self.wr = bool(wr) and Cop == 192 and Cip == 192 and self.split
        # wr_pair: an upsampling conv (64 -> 256, sub-pixel-major rows) reading a [hi | lo] pair image
        self.wr_pair = bool(wr) and not self.wr and tied_in and Cip == 64 and fcip == 128 and Cop == 256 and self.split
        if self.wr_pair:   # + its input-gradient form (kind 16, rows = the 64 input channels)
            self.mapp = H.wmap(15, Co, Ci, (1, Co, Cop), (1, Ci, Cip), n_perm=n_perm)
            self.Wp15 = torch.empty(Cop * 2 * 9 * Cip, device=dev, dtype=torch.bfloat16)
            self.mapp16 = H.wmap(16, Co, Ci, (1, Co, Cop), (1, Ci, Cip), n_perm=n_perm)
            self.Wp16 = torch.empty(Cip * 9 * Cop, device=dev, dtype=torch.bfloat16)
        # wr_n64: conv_before_upsample (192 -> 64) on kair_conv3x3_wr's N <= 64 form
        self.wr_n64 = bool(wr) and not self.wr and not self.wr_pair and Cop == 64 and Cip == 192 and self.split and not tied_in
        if self.wr_n64:
            self.mapc = H.wmap(15, Co, Ci, (1, Co, Cop), (1, Ci, Cip))
            self.Wc15 = torch.empty(Cop * 2 * 9 * Cip, device=dev, dtype=torch.bfloat16)
            self.mapc16 = H.wmap(16, Co, Ci, (1, Co, Cop), (1, Ci, Cip))
            self.Wc16 = torch.empty(Cip * 9 * Cop, device=dev, dtype=torch.bfloat16)
        if self.wr:
            self.map15 = H.wmap(15, Co, Ci, (1, Co, Cop), (1, Ci, Cip))
            self.Wf15 = torch.empty(Cop * 2 * 9 * Cip, device=dev, dtype=torch.bfloat16)
            self.map16 = H.wmap(16, Co, Ci, (1, Co, Cop), (1, Ci, Cip))
            self.Wd16 = torch.empty(Cip * 9 * Cop, device=dev, dtype=torch.bfloat16)

    def fwd(self):
        """The forward GEMM's B operand."""
        return H.rows(self.Wf, w_split=self.split)

    def pack_jobs(self):
        w, b = self.w.detach(), self.b.detach()
        jobs = [(w, self.Wf, self.mapf), (b, self.bp, self.mapb)]
        if self.Wd is not None:
            jobs.append((w, self.Wd, self.mapd))
        if self.narrow:
            jobs.append((w, self.Wn, self.mapn))
        if self.wr:
            jobs += [(w, self.Wf15, self.map15), (w, self.Wd16, self.map16)]
        if self.wr_pair:
            jobs += [(w, self.Wp15, self.mapp), (w, self.Wp16, self.mapp16)]
        if self.wr_n64:
            jobs += [(w, self.Wc15, self.mapc), (w, self.Wc16, self.mapc16)]
        return jobs


class _Resi3:
    """resi_connection '3conv' (network_swinir.py:466-471, 730-737): 3x3 C->C/4 + LeakyReLU 0.2 ->
    1x1 C/4->C/4 + LeakyReLU 0.2 -> 3x3 C/4->C, the bottleneck width padded to Cq (multiple of 8).
    The LeakyReLU is the producing GEMM's epilogue; backward gates each input gradient in the
    dgrad epilogue with LeakyReLU' read from the saved post-activation (same sign)."""

    def __init__(self, eng, seq):
        C = seq[0].in_channels
        q = seq[0].out_channels
        self.q, self.Cq = q, _rup(q, 8)
        self.c1 = _Conv(eng, seq[0], self.Cq, eng.Cp)
        self.c2 = _Lin(eng, seq[2], (1, q, self.Cq), (1, q, self.Cq))
        self.c3 = _Conv(eng, seq[4], eng.Cp, self.Cq)
        assert C == eng.C and seq[4].out_channels == C

    def pack_jobs(self):
        return self.c1.pack_jobs() + self.c2.pack_jobs() + self.c3.pack_jobs()


def _resi(eng, m):
    if isinstance(m, torch.nn.Sequential):
        return _Resi3(eng, m)
    return _Conv(eng, m, eng.Cp, eng.Cp, wr=getattr(eng, "conv_wr", False))


class _Blk:
    def __init__(self, eng, blk):
        C, Cp, nh = eng.C, eng.Cp, eng.nh
        hd = C // nh
        self.mod = blk
        self.shift = blk.shift_size
        self.dp = blk.drop_path_rate
        self.n1, self.n2 = blk.norm1, blk.norm2
        self.table = blk.attn.relative_position_bias_table
        self.scale = blk.attn.scale
        Hd = blk.mlp.fc1.out_features
        sp = eng.split_linear
        fa, fm, fb, rg = eng.fused_attn, eng.fused_mlp, eng.fused_mlp_bwd, eng.rowgemm
        # frag_t (pack kind 13): the input-gradient operand of the row GEMMs / the fused MLP backward
        hp = eng.hp
        self.qkv = _Lin(eng, blk.attn.qkv, (3 * nh, hd, hp), (1, C, Cp), frag=fa, split=sp, rows=not fa, frag_t=rg)
        self.proj = _Lin(eng, blk.attn.proj, (1, C, Cp), (nh, hd, hp), frag=fa, split=sp, rows=not fa, frag_t=rg)
        self.fc1 = _Lin(eng, blk.mlp.fc1, (1, Hd, eng.Hdp), (1, C, Cp), frag=fm, split=sp, frag_t=fb or rg, rows=not fm)
        self.fc2 = _Lin(eng, blk.mlp.fc2, (1, C, Cp), (1, Hd, eng.Hdp), frag=fm, split=sp, frag_t=fb or rg, rows=not fm,
                        frag16=True)

    def linears(self):
        return (self.qkv, self.proj, self.fc1, self.fc2)


class SwinIREngine:
    def __init__(self, net, compute_dtype="bf16", split_conv=True, fused_blocks=True, fused_mlp=None,
                 split_linear=None, fused_mlp_bwd=False, side_stream=True, side_ctas=None, side_priority=0,
                 split_act=True, conv_wr=True, head_pad=None, grouped_wgrad=None):
        """split_conv (bf16 only): forward 3x3 convs multiply hi/lo bf16 weight pairs (_Conv), i.e.
        see the fp32 master weights to ~16 bits; split_linear does the same for the linears of the
        fused block kernels (_Lin, pack kind 12).
        split_act (bf16 with split_conv only): the forward convs also read their input activation as a hi/lo bf16
        pair (kair_operand.a_split: the input image, every RSTB / conv_after_body conv input and the
        reconstruction tail's activations), the operand roundings that move the evaluation PSNR
        (tools/drift_ablation.py, DESIGN.md "parity at bf16"); the Swin-block internals stay bf16.
        fused_blocks (bf16 only): each Swin block's attention half and MLP half run as one kernel
        each (kair_swin_attn_fwd, kair_swin_mlp_fwd) where the geometry allows it (6 heads,
        Cp = 192, hidden padded to 384); fused_mlp (default: fused_blocks) selects the MLP-half
        kernel separately."""
        self.net_ref = weakref.ref(net)
        if compute_dtype not in ("bf16", "fp32", "fp32x3"):
            raise ValueError(compute_dtype)
        # fp32x3: the fp32 reference's arithmetic on the 16-bit matrix cores -- every contraction multiplies
        # fp16 pairs of power-of-2-scaled operands (hi.hi + hi.lo + lo.hi, fp32 accumulation; ~2^-21 relative
        # per product), operands fp32 (split inside the kernels) or fp16 hi/lo planes; the unfused launch
        # sequence of the fp32 engine.  Exponents put the bulk of every operand at 2^2 .. 2^10 -- the lo half
        # (2^-11 of the value) then stays a normal fp16 number (>= 2^-14) while the largest values keep
        # >= 16x headroom below fp16's 65504: weights KAIR_X3_WEXP (packs: |w| ~ 0.02 -> ~2^6),
        # activations X3_AEXP (O(1) -> 2^4), gradients P["e_g"] (the loss normalisation, _x3_grad_exp)
        self.x3 = compute_dtype == "fp32x3"
        self._ax = 0   # x3: the exponent of the GEMM A operands / fp16 outputs of the phase being issued
        # x3 exponents of the activation class and of the gradient class (offset over the loss normalisation);
        # lowered together by x3_backoff() when the range guard sees an operand leave fp16's window
        self.X3_AEXP = 4
        self.x3_gexp_off = 4
        self.x3_backoffs = 0
        self.cd = H.BF16 if compute_dtype in ("bf16", "fp32x3") else H.F32
        self.tn_cd = H.X3 if self.x3 else self.cd   # kair_gemm_tn compute of the weight gradients
        self.tdt = torch.bfloat16 if compute_dtype == "bf16" else torch.float32
        self.split_conv = bool(split_conv) and compute_dtype == "bf16"
        # split activations only pay with split weights (a bf16 weight rounding dominates otherwise), and
        # the tied pair forms need split weight packs
        self.split_act = bool(split_act) and self.split_conv
        self.C = net.embed_dim
        heads = {l.residual_group.blocks[0].num_heads for l in net.layers}
        if len(heads) != 1:
            raise NotImplementedError("kair_amd SwinIR: per-stage head counts must match")
        self.nh = heads.pop()
        hd = self.C // self.nh
        if hd >= 32 or self.C % self.nh:
            raise NotImplementedError("kair_amd SwinIR: head_dim must be < 32")
        self.ws = net.window_size
        if self.ws != 8:
            raise NotImplementedError("kair_amd SwinIR: window_size 8 only (fused attention tile)")
        self.Cp = _rup(self.C + 1, 32)
        self.fused_attn = bool(fused_blocks) and compute_dtype == "bf16" and self.nh == 6 and self.Cp == 32 * self.nh
        Hd = net.layers[0].residual_group.blocks[0].mlp.fc1.out_features
        self.Hdp = _rup(Hd + 1, 32)
        # fused_mlp=False: the LN2 / fc1 / fc2 launches instead of the fused MLP half (A/B timing).  Every
        # engine variant is a constructor argument: no environment variable changes what the engine runs
        if fused_mlp is None:
            fused_mlp = fused_blocks
        self.fused_mlp = bool(fused_mlp) and compute_dtype == "bf16" and self.Cp == 192 and self.Hdp == 384
        # head pad of the q/k/v / O / dO layouts: 16 for head dims below 16 on the unfused bf16 path (SwinIR-lightweight,
        # 60 / 6 = 10: half the attention bytes of a 32 pad, kair_window_attn_fwd_ex), else 32; head_pad=32 forces the
        # wide layout (A/B timing, parity of both layouts)
        hp16 = compute_dtype == "bf16" and hd < 16 and not self.fused_attn and not (self.Cp == 192 and self.Hdp == 384)
        self.hp = 16 if hp16 and head_pad in (None, 16) else 32
        if head_pad not in (None, 16, 32) or (head_pad == 16 and self.hp != 16):
            raise ValueError(f"head_pad {head_pad}: 32, or 16 for bf16 head dims below 16 on the unfused path")
        # the MLP-half backward kernel: off by default -- 205 us per block at B = 32 against 172-186 us
        # for the fc2 / fc1 input-gradient GEMMs + LN2 backward it replaces (its memory
        # waves' LayerNorm rows and the tile loads run latency-exposed); fused_mlp_bwd=True enables it
        self.fused_mlp_bwd = (bool(fused_blocks) and compute_dtype == "bf16" and self.Cp == 192 and self.Hdp == 384
                              and bool(fused_mlp_bwd))
        # split linears measured: the PSNR effect of bf16 linear-weight rounding is ~1e-4 dB against
        # ~5e-4 dB of activation-rounding noise per image (tools/parity_seeds.py, DESIGN.md "parity at
        # bf16"), at +45 us per block for the attention kernel -- off unless asked for
        self.split_linear = bool(split_linear) and compute_dtype == "bf16"
        # Swin-block input gradients on the row GEMMs with fused consumers (kair_rowgemm_*, csrc/rowgemm.hip):
        # fc2 (GELU' gate), fc1 + LayerNorm-2 backward, proj, q/k/v + LayerNorm-1 backward -- bf16, Cp = 192
        # geometry (classical / real-world x4); other widths run the same products on kair_gemm_nt +
        # kair_layernorm_bwd.  No library GEMM is on the training path.
        self.rowgemm = (compute_dtype == "bf16" and self.Cp == 192 and self.Hdp == 384 and self.nh * self.hp == self.Cp)
        self.upsampler, self.scale = net.upsampler, net.upscale
        self.in_ch = net.conv_first.in_channels
        self.img_range = float(net.img_range)
        self.Cin_p = 8
        # split_act: the input image as a hi/lo pair in channels [0, in_ch) / [4, 4 + in_ch) of Cin_p
        self.xin_hilo = self.split_act and 2 * self.in_ch <= self.Cin_p
        # the '1conv' RSTB / conv_after_body convs (192 -> 192) and their input gradients on the
        # register-streamed-weight kernel (kair_conv3x3_wr, csrc/conv_wr.hip) where the per-GPU batch gives
        # it enough tiles (plan: P["conv_wr"]); the LDS-ring halo kernel otherwise
        self.conv_wr = bool(conv_wr) and self.split_act and self.Cp == 192 and self.C % 4 == 0
        self.device = net.conv_first.weight.device
        dev = self.device
        self.mean = net.mean.view(-1).to(dev, torch.float32).contiguous()
        # layer objects
        self.conv_first = _Conv(self, net.conv_first, self.Cp, self.Cin_p, need_dgrad=False, tied_in=self.xin_hilo)
        self.pe_norm = net.patch_embed.norm
        self.rstb = []
        for layer in net.layers:
            blks = [_Blk(self, b) for b in layer.residual_group.blocks]
            self.rstb.append((blks, _resi(self, layer.conv)))
        self.norm = net.norm
        self.cab = _resi(self, net.conv_after_body)
        nf = 64
        self.last_narrow_x3 = False
        if self.upsampler == "pixelshuffle":
            self.cbu = _Conv(self, net.conv_before_upsample[0], nf, self.Cp, wr=self.conv_wr)
            self.ups = []
            # split_act: a0 / the upsampled activations are stored as [hi | lo] pairs (128 channels), read by
            # the upsampling convs through weights tied over both halves (the halo kernel skips lo . lo)
            for m in net.upsample:
                if isinstance(m, torch.nn.Conv2d):   # output channels sub-pixel-major (PSHUF_SPM)
                    self.ups.append(_Conv(self, m, m.out_channels, nf, n_perm=m.out_channels // nf,
                                          tied_in=self.split_act, fwd_cip=2 * nf if self.split_act else None,
                                          wr=self.conv_wr))
            self.ups_r = [int(math.isqrt(c.Co // nf)) for c in self.ups]
            # conv_last 64 -> in_ch on the narrow-output kernels (bf16 engine; HR width a multiple of 16)
            # (per call: the HR width must be a multiple of 64, else the implicit-GEMM path runs)
            self.last_narrow = self.tdt == torch.bfloat16 and self.split_conv and self.in_ch <= 4
            self.last = _Conv(self, net.conv_last, 16, nf, narrow=self.last_narrow)
            # ... and their fp32x3 forms (csrc/tail.hip *_x3: fp16 pairs of the fp32 operands, as kair_gemm_nt_x3)
            self.last_narrow_x3 = self.x3 and self.in_ch <= 4
        elif self.upsampler == "pixelshuffledirect":
            conv = net.upsample[0]
            self.ups_r = [self.scale]
            self.up1 = _Conv(self, conv, _rup(conv.out_channels, 16), self.Cp)
        elif self.upsampler == "nearest+conv":   # x4: two nearest x2 + conv + LeakyReLU 0.2, conv_hr, conv_last
            self.cbu = _Conv(self, net.conv_before_upsample[0], nf, self.Cp)
            self.nup = [_Conv(self, net.conv_up1, nf, nf), _Conv(self, net.conv_up2, nf, nf)]
            self.hrc = _Conv(self, net.conv_hr, nf, nf)
            self.last = _Conv(self, net.conv_last, 16, nf)
        elif self.upsampler in (None, ""):        # denoising / JPEG: E = x + conv_last(res)
            self.last = _Conv(self, net.conv_last, 16, self.Cp)
        else:
            raise NotImplementedError(self.upsampler)
        self.blocks = [b for blks, _ in self.rstb for b in blks]
        self.plans = PlanPool(self._build_plan)
        self.plan_mode = "primary"
        self._packed_version = None
        self._pack_table = None
        self.seg_hook = None   # called between the gradient segments of backward() (grad_segments())
        # Swin-block weight gradients: deferred to the end of each RSTB and issued as ONE grouped
        # launch (kair_wgrad_grouped: 4 linears x depth blocks) where the bf16 TN ring takes the shapes;
        # otherwise one gemm_tn + finalize per linear, issued in place.  Narrow blocks (Cp = 64, SwinIR-lightweight) too:
        # one 192 x 192 ring tile per linear (profiles/r06_c2_head_pad16_ab.txt); grouped_wgrad=False: per linear (A/B)
        self.grouped_wgrad = (grouped_wgrad is not False and self.tdt == torch.bfloat16 and self.Hdp <= 576 and
                              3 * self.nh * self.hp <= 576 and
                              max(len(l.residual_group.blocks) for l in net.layers) <= H.WgradGroup.WG_MAX // 4)
        self._wg_pending = []
        self._lnp_pending = []    # (partials, M, C, dgamma, dbeta, accumulate) of the RSTB's LayerNorms
        self._dtab_pending = []   # (partials, nWin, nh, dtype, dtable, accumulate) of its attention blocks
        self._conv_pending = []   # the RSTB conv's weight gradient (_wgrad arguments)
        self._side = None         # side stream of the deferred per-RSTB gradient work
        # side_stream=False: the deferred per-RSTB work runs in place on the main stream (A/B timing).  fp32x3
        # defers its block weight gradients (one TN ring + finalize each) the same way: they fill the CUs the
        # data-gradient chain's 192-column ring GEMMs leave idle (576 tiles: 3 rounds on 192 CUs)
        self.x3_side = self.x3 and self.Hdp <= 576
        self.side_stream = (self.grouped_wgrad or self.x3_side) and torch.cuda.is_available() and bool(side_stream)
        self.side_priority = side_priority   # torch stream priority of the side stream (0: default)
        # workgroup budget of the side-stream launches (0: uncapped).  The weight-gradient kernels hold one
        # 512-thread workgroup per CU; spread over the chip they keep the next RSTB's data-gradient kernels
        # off it until they end (rocprof: the first fc2 input gradient of every RSTB 43 -> 495 us behind the
        # grouped launch, the attention backward 80 -> 340 us behind the conv weight gradient).  Measured
        # (profiles/r03_side_ctas_ab.txt): a cap makes the side work critical at B=32 (48 CTAs: 1080 -> 808
        # patches/s) and gains ~2% at B=4 (96 CTAs) -- so uncapped by default.
        # fp32x3: the deferred weight gradients capped at 192 workgroups (B = 32 639 -> 650 patches/s against uncapped
        # with one launch per linear, profiles/r06_side_ctas_ab.txt); with the grouped launch (one per RSTB) 96 at the
        # small per-GPU batches of a multi-GPU run (M < 36,864 rows, B < 16: B = 4 333 -> 344, B = 8 429 -> 443; B = 16
        # and 32 unchanged, profiles/r06_side_ctas_grouped_ab.txt) -- the x3_side_cap rule
        self.side_ctas_auto = side_ctas is None and self.x3
        if side_ctas is None:
            side_ctas = 192 if self.x3 else 0
        # fp32x3: an RSTB's deferred block weight gradients as ONE grouped TN-ring launch + one grouped finalize
        # (kair_wgrad_grouped with fp16-pair jobs) instead of a launch pair per linear (KAIR_X3_GROUPED=0: A/B)
        self.x3_grouped = self.x3_side and os.environ.get("KAIR_X3_GROUPED", "1") != "0"
        # fp32x3: the LayerNorm backwards fused into the qkv / fc1 input-gradient GEMMs' epilogue (kair_gemm_nt_x3_lnbwd,
        # KAIR_X3_LNFUSE=1).  Off by default: measured slower (B = 32 660 -> 614, B = 4 349 -> 340 patches/s,
        # profiles/r06_x3_lnfuse_ab.txt) -- the LayerNorm backward's own traffic (x, D read, D and its operand copy
        # written) stays and now runs in the ring's epilogue intervals, in 64-row tiles (the 128-row form spills)
        self.x3_lnfuse = (self.x3 and self.Cp == 192 and self.C % 4 == 0 and not self.rowgemm and not fused_mlp_bwd and
                          os.environ.get("KAIR_X3_LNFUSE", "0") == "1")
        self.side_ctas = int(side_ctas)
        # '1conv' weight gradients on the tap-per-tile ring (bf16 copies of G and the conv input)
        self.conv_tap = self.tdt == torch.bfloat16 and self.Cp == 192 and self.C % 4 == 0
        self.conv_wr_min_tiles = 64    # P["conv_wr"]: 96-pixel tiles needed (B = 4: 96 tiles, 1.04x faster than the halo kernel)

    def grad_segments(self):
        """Parameter groups in the order backward() completes their gradients; seg_hook() fires
        between consecutive groups.  Each group is contiguous in registration order, so the data-
        parallel trainer can all-reduce it as one bucket while the rest of backward runs."""
        net = self.net_ref()
        tail = list(net.norm.parameters()) + list(net.conv_after_body.parameters())
        if self.upsampler == "pixelshuffle":
            tail += (list(net.conv_before_upsample.parameters()) + list(net.upsample.parameters()) +
                     list(net.conv_last.parameters()))
        elif self.upsampler == "nearest+conv":
            tail += [p for m in (net.conv_before_upsample, net.conv_up1, net.conv_up2, net.conv_hr, net.conv_last)
                     for p in m.parameters()]
        elif self.upsampler in (None, ""):
            tail += list(net.conv_last.parameters())
        else:
            tail += list(net.upsample.parameters())
        segs = [tail]
        for gi in range(len(net.layers) - 1, 0, -1):
            segs.append(list(net.layers[gi].parameters()))
        segs.append(list(net.conv_first.parameters()) + list(net.patch_embed.parameters()) +
                    list(net.layers[0].parameters()))
        return segs

    def _segment_done(self):
        if self.seg_hook is not None:
            self.seg_hook()

    # ------------------------------------------------------------------------------------
    def convs(self):
        cs = [self.conv_first] + [c for _, c in self.rstb] + [self.cab]
        if self.upsampler == "pixelshuffle":
            cs += [self.cbu] + self.ups + [self.last]
        elif self.upsampler == "nearest+conv":
            cs += [self.cbu] + self.nup + [self.hrc, self.last]
        elif self.upsampler in (None, ""):
            cs += [self.last]
        else:
            cs += [self.up1]
        return cs

    def pack(self, force=False):
        net = self.net_ref()
        # repack_always: an engine whose parameters are updated outside torch (the fused trainer's Adam
        # kernel writes the flat parameter buffer; versions do not move) and that no step graph repacks
        # -- the eval-mode twin (SwinIR.eval_engine)
        force = force or getattr(self, "repack_always", False)
        ver = None if force else tuple(p._version for p in net.parameters())
        if ver is not None and ver == self._packed_version:
            return
        ptrs = tuple(p.data_ptr() for p in net.parameters())
        if self._pack_table is None or self._pack_table[0] != ptrs:   # params re-homed (e.g. flattened)
            jobs = [j for c in self.convs() for j in c.pack_jobs()]
            jobs += [j for b in self.blocks for l in b.linears() for j in l.pack_jobs()]
            self._pack_table = (ptrs, H.PackTable(jobs))
        self._pack_table[1].run()
        self._packed_version = ver

    def plan(self, B, Hh, Ww):
        return self.plans.get((B, Hh, Ww), self.plan_mode)

    def _build_plan(self, key, infer):
        """Buffers of one input shape.  infer=True: forward only -- the Swin blocks ping-pong between
        two buffer sets (nothing is kept for a backward) and no backward scratch is allocated."""
        B, Hh, Ww = key
        dev, T, f32 = self.device, self.tdt, torch.float32
        M = B * Hh * Ww
        Cp, Hdp, nh, hp = self.Cp, self.Hdp, self.nh, self.hp
        nWin = M // WS_TOK
        e = lambda *s, dt=f32: torch.empty(*s, device=dev, dtype=dt)
        hf = torch.float16
        P = {"B": B, "H": Hh, "W": Ww, "M": M, "nWin": nWin}
        # fp32x3: the exponent of the backward's data gradients (the mean loss over the output image)
        P["e_g"] = self._x3_grad_exp(B * self.in_ch * Hh * self.scale * Ww * self.scale)
        P["xin"] = e(M, self.Cin_p, dt=T)
        P["f0"] = e(M, Cp)
        P["pe_mean"], P["pe_rstd"] = e(M), e(M)
        P["s0"] = e(M, Cp)
        blocks = []
        for bi in range(len(self.blocks)):
            if infer and bi >= 2:
                blocks.append(blocks[bi % 2])
                continue
            # fp32x3: every Swin-block GEMM operand -- ln1, q/k/v, O, ln2, h -- is stored ONCE by its producer as the
            # fp16 pair [2, ...] (hi plane, lo plane) of v 2^X3_AEXP, so the consuming ring GEMMs (forward NT, weight-
            # gradient TN) and the attention kernels read pairs instead of splitting fp32 rows at every fragment load
            pr = (lambda *sh: e(2, *sh, dt=hf)) if self.x3 else (lambda *sh: e(*sh, dt=T))
            blocks.append({
                "mid": e(M, Cp), "out": e(M, Cp), "ln1": pr(M, Cp), "m1": e(M), "r1": e(M),
                "qkv": e(2, 3 * M * nh * hp, dt=hf) if self.x3 else e(3 * M * nh * hp, dt=T),
                "O": pr(M, nh * hp), "lse": e(nWin * nh * WS_TOK),
                "ln2": pr(M, Cp), "m2": e(M), "r2": e(M), "u": e(M, Hdp, dt=T), "h": pr(M, Hdp)})
        P["blocks"] = blocks
        P["rstb_out"] = [e(M, Cp) for _ in range(min(2, len(self.rstb)) if infer else len(self.rstb))]
        if infer:
            P["rstb_out"] = [P["rstb_out"][i % len(P["rstb_out"])] for i in range(len(self.rstb))]
        P["nf"], P["n_mean"], P["n_rstd"] = e(M, Cp), e(M), e(M)
        P["fb"] = e(M, Cp)
        if self.upsampler == "pixelshuffle":
            nf = 64
            # split_act: [hi | lo] pair rows (ld 2 nf); the backward reads the hi half as its bf16 operand
            tl = P["tail_ld"] = 2 * nf if self.split_act else nf
            P["a0"] = e(M, tl, dt=T)
            acts, hw = [], M
            for r in self.ups_r:
                hw *= r * r
                acts.append(e(hw, tl, dt=T))
            P["ups_act"] = acts
            P["M_hr"] = hw
            if self.last_narrow_x3:
                P["narrow_fws"] = e(H.conv3x3_narrow_x3_ws())
        elif self.upsampler == "nearest+conv":
            nf = 64
            P["a0"] = e(M, nf, dt=T)
            P["nup_act"] = [e(4 * M, nf, dt=T), e(16 * M, nf, dt=T)]
            P["nhr"] = e(16 * M, nf, dt=T)
            P["M_hr"] = 16 * M
        # '3conv' bottleneck activations (post-LeakyReLU, compute dtype) of every residual connection
        P["r3"] = {id(r): (e(M, r.Cq, dt=T), e(M, r.Cq, dt=T)) for r in [c for _, c in self.rstb] + [self.cab]
                   if isinstance(r, _Resi3)}
        P["E"] = e(B, self.in_ch, Hh * self.scale, Ww * self.scale)
        P["infer"] = infer
        if infer:
            return P
        # backward scratch
        # residual-gradient rows: zero-filled once, so their pad columns [C, Cp) are finite zeros.  The LN row
        # GEMMs write all Cp columns of their bf16 operand copies (scale * D's pad) and the gate / store
        # contractions read them: a NaN bit pattern left in a pad column would become 0 * NaN = NaN
        z32 = lambda *s: torch.zeros(*s, device=dev, dtype=f32)
        P["D"], P["G"] = z32(M, Cp), z32(M, Cp)
        P["dxn"] = e(M, Cp, dt=T)
        if self.fused_mlp_bwd:
            P["mlp_ws"] = e(H.swin_mlp_bwd_ws())
        # per block position in an RSTB: the weight-gradient operands of that block, kept until the
        # RSTB's grouped weight-gradient launch (Dm: s_mlp * dL/dout, token order; Da: s_attn * dL/dmid,
        # window order -- the compute-dtype copies LayerNorm backward writes; dU: fc1 pre-activation
        # gradient; dqkv: head-blocked q/k/v gradient)
        # (zero-filled: kair_layernorm_bwd's copies write the C real columns only, the GEMMs read Cp)
        depth = max(len(blks) for blks, _ in self.rstb)
        z = lambda *s: torch.zeros(*s, device=dev, dtype=T)
        # fp32x3: the block's gradient operands as fp16 pairs [2, ...] of v 2^e_g (zero-filled pads as above)
        zp = (lambda *sh: torch.zeros(2, *sh, device=dev, dtype=hf)) if self.x3 else z
        ep = (lambda *sh: e(2, *sh, dt=hf)) if self.x3 else (lambda *sh: e(*sh, dt=T))
        # (the fused fp32x3 LayerNorm backward leaves one partial row per 16 GEMM rows)
        lnp = max(2 * 2048 * Cp, 2 * self.C * H.gemm_nt_lnbwd_parts(M, Cp) if self.x3_lnfuse else 0)
        # Two sets (RSTB parity): the side stream still reads one RSTB's while the next RSTB writes the other.
        P["gw"] = [[{"Dm": zp(M, Cp), "Da": zp(M, Cp), "dU": ep(M, Hdp),
                     # fp32x3: dq/dk/dv as token rows [M][3 nh 32] (pairs: the ring GEMMs' operand)
                     "dqkv": ep(M, 3 * nh * hp) if self.x3 else e(3 * M * nh * hp, dt=T),
                     # LN1 / LN2 parameter partials and the attention bias-table partials of the block, reduced
                     # by one grouped launch each at the end of the RSTB
                     "ln1p": e(lnp), "ln2p": e(lnp), "attn_ws": e(H.window_attn_bwd_ws(nWin, nh))}
                    for _ in range(depth)] for _ in range(2)]
        P["G3"] = z32(M, Cp)   # third residual-gradient buffer (rotation, see backward())
        if self.rowgemm:   # LayerNorm-parameter partial rows the fused row GEMMs leave (<= the ln*p buffers' 2048)
            P["rg_nb"] = {k: H.rowgemm_ln_blocks(M, k) for k in (Hdp, 3 * nh * hp)}
            assert max(P["rg_nb"].values()) <= 2048, P["rg_nb"]
        P["dO"] = e(2, M, nh * hp, dt=hf) if self.x3 else e(M, nh * hp, dt=T)
        P["ln_ws"] = e(2 * 2048 * Cp)   # kair_layernorm_bwd: 2 * 2048 * C floats
        P["attn_ws"] = e(H.window_attn_bwd_ws(nWin, nh))
        P["loss"] = e(1)
        P["loss_ws"] = e(1024)
        P["colsum_ws"] = e(1024 * 256)
        if self.upsampler == "pixelshuffle":
            # the HR-image gradient rows: 4 fp32 slots when only the fp32x3 narrow kernels read them (conv_last at
            # an HR width % 64 == 0), else the 16 slots of the implicit-GEMM conv_last's K = 9 x 16
            P["dE_ld"] = 4 if self.last_narrow_x3 and (Ww * self.scale) % 64 == 0 else 16
            P["dE"] = e(P["M_hr"], P["dE_ld"], dt=T)
            if self.last.narrow or self.last_narrow_x3:
                P["narrow_ws"] = e(H.conv3x3_narrow_wgrad_ws(self.in_ch))
                P["narrow_dws"] = e(H.conv3x3_narrow_x3_ws() if self.x3 else H.conv3x3_narrow_dgrad_ws())
            dpre, hw = [], M
            for c in self.ups:
                dpre.append(e(hw, c.Co, dt=T))
                hw *= c.Co // 64
            P["dpre"] = dpre
            P["da0"] = e(M, 64, dt=T)
        elif self.upsampler == "nearest+conv":
            nf = 64
            P["dE"] = e(16 * M, 16, dt=T)
            P["dz_hr"], P["dz_u"] = e(16 * M, nf, dt=T), e(16 * M, nf, dt=T)
            P["G_hi"], P["G_lo"] = e(16 * M, nf), e(4 * M, nf)
            P["da0"] = e(M, nf, dt=T)
        elif self.upsampler in (None, ""):
            P["dE"] = e(M, 16, dt=T)
        else:
            P["dE"] = e(M, self.up1.Cop, dt=T)
        if P["r3"]:
            q = max(r.Cq for r in [c for _, c in self.rstb] + [self.cab] if isinstance(r, _Resi3))
            P["r3_dz"] = (e(M, q, dt=T), e(M, q, dt=T))
        P["dfb"] = e(M, Cp)
        if self.conv_tap:
            # bf16 operands of each '1conv' weight gradient: (G, conv input with 1.0 in channel C), written by
            # the halo convs (forward: input, backward dgrad: G) or, off that path, copied when the job runs
            P["conv_halo"] = H.conv_halo_geometry(Hh, Ww, Cp, M, Cp)
            # the register-streamed-weight conv: one 96-pixel tile per workgroup per CU round, so only with
            # at least a full round of tiles (B = 32: 768 tiles; B = 4: 96 -> the halo kernel's N tiles)
            P["conv_wr"] = bool(self.conv_wr and H.conv3x3_wr_tile(1, B, Hh, Ww, Cp, Cp) > 0 and
                                H.conv3x3_wr_tile(0, B, Hh, Ww, Cp, Cp) > 0 and M // 96 >= self.conv_wr_min_tiles)
            if P["conv_wr"]:
                P["conv_halo"] = True   # the wr kernel leaves the same bf16 copies
            P["conv_bf"] = {}
            for r in [c for _, c in self.rstb] + [self.cab]:
                if not isinstance(r, _Resi3):
                    P["conv_bf"][id(r)] = (torch.zeros(M, Cp, device=dev, dtype=T), torch.zeros(M, Cp, device=dev, dtype=T))
                    P["conv_bf"][id(r)][1][:, self.C] = 1.0
        # one shared wgrad workspace sized for the largest (splits * N * K)
        P["wg_ws"] = e(self._max_wgrad_ws(M, P))
        P["wg_ws2"] = (e(P["wg_ws"].numel() * max(1, -self.side_ctas)) if self.grouped_wgrad or self.side_stream
                       else None)   # the side stream's
        return P

    def _wgrad_shapes(self, M, P):
        """(M_rows, N, K) of every weight-gradient GEMM in the step."""
        Cp, Hdp, nh = self.Cp, self.Hdp, self.nh
        out = [(M, Cp, 9 * self.Cin_p)]

        def resi(r):
            if isinstance(r, _Resi3):
                return [(M, r.Cq, 9 * Cp), (M, r.Cq, r.Cq), (M, Cp, 9 * r.Cq)]
            return [(M, Cp, 9 * Cp)]

        for blks, conv in self.rstb:
            for _ in blks:
                out += [(M, Cp, Hdp), (M, Hdp, Cp), (M, Cp, nh * self.hp), (M, 3 * nh * self.hp, Cp)]
            out += resi(conv)
        out += resi(self.cab)
        if self.upsampler == "nearest+conv":
            out += [(M, 64, 9 * Cp), (4 * M, 64, 9 * 64), (16 * M, 64, 9 * 64), (16 * M, 64, 9 * 64),
                    (16 * M, 16, 9 * 64)]
        elif self.upsampler in (None, ""):
            out.append((M, 16, 9 * Cp))
        elif self.upsampler == "pixelshuffle":
            out.append((M, 64, 9 * Cp))
            hw = M
            for c in self.ups:
                out.append((hw, c.Co, 9 * 64))
                hw *= c.Co // 64
            out.append((hw, 16, 9 * 64))
        else:
            out.append((M, self.up1.Cop, 9 * Cp))
        return out

    def _max_wgrad_ws(self, M, P):
        ws = max(H.wgrad_splits(m, n, k) * n * k for m, n, k in self._wgrad_shapes(M, P))
        if self.grouped_wgrad or self.x3_grouped:
            Cp, Hdp, nh = self.Cp, self.Hdp, self.nh
            depth = max(len(blks) for blks, _ in self.rstb)
            shapes = [(Cp, Hdp), (Hdp, Cp), (Cp, nh * self.hp), (3 * nh * self.hp, Cp)] * depth
            for i in range(0, len(shapes), H.WgradGroup.WG_MAX):
                ws = max(ws, H.wgrad_grouped_ws(shapes[i:i + H.WgradGroup.WG_MAX], M, x3=self.x3))
        return ws

    # ------------------------------------------------------------------------------------
    # forward
    # ------------------------------------------------------------------------------------
    def forward(self, x, drop_scales=None):
        """x: [B, in_ch, H, W] fp32 on the device (H, W multiples of 8).  Returns P['E'] (NCHW fp32).
        drop_scales: optional [nblocks, 2, B] fp32 DropPath scales (0 or 1/keep)."""
        B, _, Hh, Ww = x.shape
        P = self.plan(B, Hh, Ww)
        self.pack()
        cd, T = self.cd, self.tdt
        M, Cp, nh = P["M"], self.Cp, self.nh
        HW = Hh * Ww
        x = x.contiguous()
        self.cur = P
        self._ax = self.X3_AEXP   # fp32x3: forward operands are activations
        P["x"] = x
        P["drop"] = drop_scales
        if self.xin_hilo:
            H.image_to_nhwc_hilo(x, P["xin"], self.Cin_p, self.mean, self.img_range, B, self.in_ch, Hh, Ww)
        else:
            H.image_to_nhwc(x, P["xin"], self.Cin_p, self.mean, self.img_range, B, self.in_ch, Hh, Ww)
        c = self.conv_first
        self._nt(H.im2col(P["xin"], Hh, Ww, self.Cin_p), c.fwd(), H.epilogue(P["f0"], bias=c.bp), M, Cp,
                  9 * self.Cin_p, cd)
        n = self.pe_norm
        H.layernorm_fwd(P["f0"], Cp, P["s0"], Cp, n.weight, n.bias, P["pe_mean"], P["pe_rstd"], M, self.C, n.eps)
        cur = P["s0"]
        bi = 0
        for gi, (blks, conv) in enumerate(self.rstb):
            g_in = cur
            for blk in blks:
                cur = self._block_fwd(blk, P, P["blocks"][bi], cur, bi)
                bi += 1
            out = P["rstb_out"][gi]
            self._resi_fwd(conv, P, cur, out, g_in)
            cur = out
        n = self.norm
        H.layernorm_fwd(cur, Cp, P["nf"], Cp, n.weight, n.bias, P["n_mean"], P["n_rstd"], M, self.C, n.eps)
        self._resi_fwd(self.cab, P, P["nf"], P["fb"], P["f0"])
        return self._forward_tail(P)

    def _resi_fwd(self, r, P, src, out, resid):
        """out = resi_conv(src) + resid (fp32 token rows, Cp columns)."""
        cd, Cp, M, Hh, Ww = self.cd, self.Cp, P["M"], P["H"], P["W"]
        if not isinstance(r, _Resi3):
            # training: the halo conv also leaves the bf16 weight-gradient operand (1.0 in channel C)
            ac = (P["conv_bf"][id(r)][1], self.C) if P.get("conv_halo") else None
            if P.get("conv_wr") and r.wr:
                assert src.dtype == torch.float32 and resid.dtype == torch.float32
                H.conv3x3_wr(src, Cp, 0, r.Wf15, r.bp, resid, out, P["B"], Hh, Ww, Cp, Cp, acopy=ac[0], acones=ac[1],
                             split=True)
                return
            self._nt(self._ain(H.im2col(src, Hh, Ww, Cp)), r.fwd(), H.epilogue(out, bias=r.bp, resid=resid, acopy=ac), M,
                      Cp, 9 * Cp, cd)
            return
        t1, t2 = P["r3"][id(r)]
        lk = dict(act=H.ACT_LEAKY, slope=0.2)
        self._nt(H.im2col(src, Hh, Ww, Cp), r.c1.fwd(), H.epilogue(t1, bias=r.c1.bp, **lk), M, r.Cq, 9 * Cp, cd)
        self._nt(H.rows(t1), H.rows(r.c2.Wp), H.epilogue(t2, bias=r.c2.bp, **lk), M, r.Cq, r.Cq, cd)
        self._nt(H.im2col(t2, Hh, Ww, r.Cq), r.c3.fwd(), H.epilogue(out, bias=r.c3.bp, resid=resid), M, Cp, 9 * r.Cq, cd)

    def _resi_bwd(self, r, P, G, src, D, grads):
        """resi_conv backward for out = resi_conv(src) + resid: G = dL/d out (fp32 rows) -> D = dL/d src
        (the conv path only; the caller adds the skip).  '1conv' returns its weight-gradient job for
        the deferred per-RSTB work; '3conv' issues its weight gradients here."""
        cd, Cp, M, Hh, Ww = self.cd, self.Cp, P["M"], P["H"], P["W"]
        g = lambda p: grads[p]
        if not isinstance(r, _Resi3):
            ac = (P["conv_bf"][id(r)][0], -1) if P.get("conv_halo") else None
            if P.get("conv_wr") and r.wr:
                H.conv3x3_wr(G, Cp, 1, r.Wd16, None, None, D, P["B"], Hh, Ww, Cp, Cp, acopy=ac[0], split=False)
            else:
                self._nt(H.im2col(G, Hh, Ww, Cp, flip=True), H.rows(r.Wd), H.epilogue(D, acopy=ac), M, Cp, 9 * Cp, cd)
            if self.conv_tap:   # bf16 operands: the halo convs' copies (else taken when the job runs)
                return ("tap", G, src, r, g(r.w), g(r.b))
            return (H.rows(G), H.im2col(src, Hh, Ww, Cp, ones_col=self.C), M, Cp, 9 * Cp, r.map, g(r.w), g(r.b), self.C)
        t1, t2 = P["r3"][id(r)]
        q = r.Cq
        lk = dict(gate_kind=2, slope=0.2)
        # 3x3 Cq -> C: dL/d t2, gated by LeakyReLU'(t2 pre-activation)
        dz2 = P["r3_dz"][0].view(-1)[:M * q].view(M, q)
        dz1 = P["r3_dz"][1].view(-1)[:M * q].view(M, q)
        self._nt(H.im2col(G, Hh, Ww, Cp, flip=True), H.rows(r.c3.Wd), H.epilogue(dz2, gate=t2, **lk), M, q, 9 * Cp, cd)
        self._wgrad(P, H.rows(G), H.im2col(t2, Hh, Ww, q), M, Cp, 9 * q, r.c3.map, g(r.c3.w))
        self._bias_colsum(P, H.rows(G), M, Cp, r.c3.mapb, g(r.c3.b))
        # 1x1 Cq -> Cq
        self._nt(H.rows(dz2), H.rows(r.c2.Wt), H.epilogue(dz1, gate=t1, **lk), M, q, q, cd)
        self._wgrad(P, H.rows(dz2), H.rows(t1), M, q, q, r.c2.map, g(r.c2.w))
        self._bias_colsum(P, H.rows(dz2), M, q, r.c2.mapb, g(r.c2.b))
        # 3x3 C -> Cq
        self._nt(H.im2col(dz1, Hh, Ww, q, flip=True), H.rows(r.c1.Wd), H.epilogue(D), M, Cp, 9 * q, cd)
        self._wgrad(P, H.rows(dz1), H.im2col(src, Hh, Ww, Cp), M, q, 9 * Cp, r.c1.map, g(r.c1.w))
        self._bias_colsum(P, H.rows(dz1), M, q, r.c1.mapb, g(r.c1.b))
        return None

    @staticmethod
    def _op(t, **kw):
        """A row operand of tensor t: an fp16 pair [2, M, N] (fp32x3: hi plane + its lo plane) or plain rows."""
        if t.dtype == torch.float16 and t.dim() == 3 and t.shape[0] == 2:
            return H.with_lo(H.rows(t[0], **kw), t[1])
        return H.rows(t, **kw)

    def _ain(self, op, lo=None):
        """A forward conv's input operand: a hi/lo pair under split_act (fp32 source: lo formed in the
        kernel; bf16 source: its lo plane `lo`), else as is."""
        return H.asplit(op, lo) if self.split_act else op

    def _nt_lnbwd(self, A, B, M, K, x, gamma, mean, rstd, D, part, win=(0, 0, 0, 0), copy=None):
        """fp32x3: the input-gradient GEMM A B^T of the Linear after a LayerNorm (N = Cp = 192) fused with that
        LayerNorm's backward into D (kair_gemm_nt_x3_lnbwd), exponents as in _nt."""
        A.x3_exp, B.x3_exp = self._ax, H.X3_WEXP
        H.gemm_nt_lnbwd(A, B, M, self.Cp, K, x, self.Cp, gamma, mean, rstd, self.C, D, self.Cp, part, win=win, copy=copy)

    def _nt(self, A, B, E, M, N, K, cd):
        """kair_gemm_nt; under fp32x3 the split-fp16 arithmetic (compute KAIR_COMPUTE_X3): A is fp32 (split in the
        kernel) or an fp16 pair (its lo plane attached with H.with_lo) carrying the phase exponent (forward 0,
        backward the gradient exponent), B a split-packed fp16 weight (2^KAIR_X3_WEXP), an fp16 output the
        pair of v 2^(phase exponent)."""
        if self.x3:
            if A.dtype == H.F16 and not A.lo_ptr:
                raise RuntimeError("fp32x3: an fp16 GEMM operand needs its lo plane")
            A.x3_exp, B.x3_exp = self._ax, H.X3_WEXP
            if A.ones_col >= 0:
                raise RuntimeError("fp32x3: no injected ones column on a GEMM A operand")
            if E.out_dtype == H.F16:
                E.x3_out_exp = self._ax
            H.gemm_nt(A, B, E, M, N, K, H.X3)
            return
        H.gemm_nt(A, B, E, M, N, K, cd)

    X3_AEXP = 4   # fp32x3 activation exponent (default; per engine: self.X3_AEXP, lowered by x3_backoff)
    X3_BACKOFF_STEP = 6      # exponent drop per range-guard event (x 1/64)
    X3_BACKOFF_MAX = 4       # events before the guard gives up and raises

    def _x3_grad_exp(self, numel, weight=1.0):
        """The fp32x3 gradient exponent: the mean-loss gradient is O(weight / numel) per output element (weight: the
        loss weight over img_range), so data gradients times 2^(log2(numel / weight) + 4) sit near 2^4 at the loss,
        2^12 below fp16's overflow."""
        return int(round(math.log2(max(numel, 1) / max(abs(weight), 1e-30)))) + self.x3_gexp_off

    def x3_backoff(self, step=None, act=True, grad=True):
        """Range guard reaction (kair_range_check saw an inf / NaN the split operands can cause): lower the activation
        exponent (act: a forward overflow, the loss went non-finite) and / or the gradient exponent (grad: a backward
        overflow) by `step` (default X3_BACKOFF_STEP), so that operand class gains that much headroom below fp16's
        65504 (the lo halves of its smallest values go subnormal first: an absolute error <= 2^-25 of the scaled
        unit).  The caller re-runs the step (re-captured graph).  Raises after X3_BACKOFF_MAX events: the data is not
        finite in fp32 either, or a weight left its pack window."""
        if not self.x3:
            raise RuntimeError("x3_backoff: not an fp32x3 engine")
        if self.x3_backoffs >= self.X3_BACKOFF_MAX:
            raise RuntimeError(f"fp32x3 range guard: the step is still non-finite after {self.x3_backoffs} exponent "
                               f"back-offs (activation 2^{self.X3_AEXP}, gradient offset 2^{self.x3_gexp_off}): the data "
                               f"is not finite, or a weight left its pack window |w| < 2^{16 - H.X3_WEXP}")
        step = self.X3_BACKOFF_STEP if step is None else int(step)
        if act:
            self.X3_AEXP -= step
        if grad:
            self.x3_gexp_off -= step
        self.x3_backoffs += 1
        return self.X3_AEXP, self.x3_gexp_off

    def _forward_tail(self, P):
        """Reconstruction tail: P['fb'] (conv_after_body + residual) -> P['E']."""
        cd, Cp, M, B, Hh, Ww = self.cd, self.Cp, P["M"], P["B"], P["H"], P["W"]
        sa = self.split_act
        if self.upsampler == "pixelshuffle":
            tl = P["tail_ld"]
            lo = (lambda t: t[:, 64:]) if sa else (lambda t: None)   # the lo half of a pair buffer
            c = self.cbu
            if (c.wr_n64 and self.conv_wr and H.conv3x3_wr_tile(1, B, Hh, Ww, Cp, 64) > 0 and
                    M // 96 >= self.conv_wr_min_tiles):
                H.conv3x3_wr(P["fb"], Cp, 0, c.Wc15, c.bp, None, P["a0"], B, Hh, Ww, Cp, 64, ldo=tl, split=True,
                             out_lo=lo(P["a0"]), act=H.ACT_LEAKY, slope=0.01)
            else:
                self._nt(self._ain(H.im2col(P["fb"], Hh, Ww, Cp)), c.fwd(),
                          H.epilogue(P["a0"], ldo=tl, bias=c.bp, act=H.ACT_LEAKY, slope=0.01, out_lo=lo(P["a0"])), M, 64,
                          9 * Cp, cd)
            src, h, w = P["a0"], Hh, Ww
            for c, r, dst in zip(self.ups, self.ups_r, P["ups_act"]):
                if (c.wr_pair and self.conv_wr and H.conv3x3_wr_tile(1, B, h, w, 64, c.Co) > 0 and
                        B * h * w // 96 >= self.conv_wr_min_tiles):   # kair_conv3x3_wr, pair form
                    H.conv3x3_wr(src, tl, 0, c.Wp15, c.bp, None, dst, B, h, w, 64, c.Co, ldo=tl, split=True,
                                 out_lo=lo(dst), ps_r=r)
                    src, h, w = dst, h * r, w * r
                    continue
                A = H.asplit(H.im2col(src, h, w, c.fcip), pair=True) if sa else H.im2col(src, h, w, 64)
                self._nt(A, c.fwd(), H.epilogue(dst, mode=H.OUT_PSHUF_SPM, ldo=tl, bias=c.bp, ps=(r, h, w), out_lo=lo(dst)),
                          B * h * w, c.Co, 9 * c.fcip, cd)
                src, h, w = dst, h * r, w * r
            c = self.last
            if self.last_narrow_x3 and w % 64 == 0:
                H.conv3x3_narrow_fwd_x3(src, tl, self.X3_AEXP, c.w.detach(), c.bp, self.in_ch, P["narrow_fws"], self.mean,
                                        self.img_range, None, P["E"], B, h, w)
                return P["E"]
            if c.narrow and w % 64 == 0:   # 64 -> in_ch: the narrow-output kernel (weights in VGPRs)
                H.conv3x3_narrow_fwd(src, tl, 64 if sa else 0, c.Wn, c.bp, self.in_ch, self.mean, self.img_range, None,
                                     P["E"], B, h, w)
                return P["E"]
            self._nt(self._ain(H.im2col(src, h, w, 64, ld=tl), lo(src)), c.fwd(),
                      H.epilogue(P["E"], mode=H.OUT_NCHW, ldo=0, bias=c.bp, img=(self.mean, self.img_range, self.in_ch, h, w)),
                      B * h * w, c.Cop, 9 * 64, cd)
        elif self.upsampler == "nearest+conv":
            c = self.cbu
            self._nt(H.im2col(P["fb"], Hh, Ww, Cp), c.fwd(),
                      H.epilogue(P["a0"], bias=c.bp, act=H.ACT_LEAKY, slope=0.01), M, 64, 9 * Cp, cd)
            src, h, w = P["a0"], Hh, Ww
            for c, dst in zip(self.nup, P["nup_act"]):   # lrelu(conv(nearest x2)): im2col reads through the upsample
                h, w = 2 * h, 2 * w
                self._nt(H.im2col(src, h, w, 64, up=2), c.fwd(), H.epilogue(dst, bias=c.bp, act=H.ACT_LEAKY, slope=0.2),
                          B * h * w, 64, 9 * 64, cd)
                src = dst
            c = self.hrc
            self._nt(H.im2col(src, h, w, 64), c.fwd(), H.epilogue(P["nhr"], bias=c.bp, act=H.ACT_LEAKY, slope=0.2),
                      B * h * w, 64, 9 * 64, cd)
            c = self.last
            self._nt(H.im2col(P["nhr"], h, w, 64), c.fwd(),
                      H.epilogue(P["E"], mode=H.OUT_NCHW, ldo=0, bias=c.bp, img=(self.mean, self.img_range, self.in_ch, h, w)),
                      B * h * w, c.Cop, 9 * 64, cd)
        elif self.upsampler in (None, ""):
            # x/range + mean with x = (x_in - mean) * range + conv_last(res)  ==  x_in + conv_last(res) / range
            c = self.last
            self._nt(self._ain(H.im2col(P["fb"], Hh, Ww, Cp)), c.fwd(),
                      H.epilogue(P["E"], mode=H.OUT_NCHW, ldo=0, bias=c.bp, resid=P["x"],
                                 img=(None, self.img_range, self.in_ch, Hh, Ww)), M, c.Cop, 9 * Cp, cd)
        else:
            c = self.up1
            self._nt(self._ain(H.im2col(P["fb"], Hh, Ww, Cp)), c.fwd(),
                      H.epilogue(P["E"], mode=H.OUT_PSHUF_NCHW, ldo=0, bias=c.bp, ps=(self.scale, Hh, Ww),
                                 img=(self.mean, self.img_range, self.in_ch, Hh, Ww)), M, c.Cop, 9 * Cp, cd)
        return P["E"]

    def _block_fwd(self, blk, P, S, x, bi):
        cd = self.cd
        M, Cp, nh, hp, Hh, Ww = P["M"], self.Cp, self.nh, self.hp, P["H"], P["W"]
        HW = Hh * Ww
        win = (Hh, Ww, 8, blk.shift)
        drop = P["drop"]
        s_attn = drop[bi, 0] if drop is not None else None
        s_mlp = drop[bi, 1] if drop is not None else None
        # LN1 / LN2 / fc1 / attention write 1.0 into their first pad column: the ones column the
        # weight-gradient GEMMs use for the bias gradient (the packed weights are 0 there)
        if self.fused_attn:   # LN1 -> qkv -> window attention -> proj + residual in one launch
            H.swin_attn_fwd(x, Cp, blk.n1.weight, blk.n1.bias, blk.n1.eps, self.C, S["ln1"], Cp, S["m1"], S["r1"],
                            blk.qkv.Wg, blk.qkv.bp, S["qkv"], blk.table, blk.scale, S["O"], nh * 32, self.C // nh,
                            S["lse"], blk.proj.Wg, blk.proj.bp, s_attn, HW, S["mid"], Cp, P["nWin"], nh, Hh, Ww,
                            blk.shift, w_split=blk.qkv.split)
        else:
            if self.x3:   # ln1 as the fp16 pair of its qkv / wgrad consumers
                H.layernorm_fwd_x3(x, Cp, S["ln1"], Cp, blk.n1.weight, blk.n1.bias, S["m1"], S["r1"], M, self.C, blk.n1.eps,
                                   win, one_col=self.C, x3_exp=self.X3_AEXP)
            else:
                H.layernorm_fwd(x, Cp, S["ln1"], Cp, blk.n1.weight, blk.n1.bias, S["m1"], S["r1"], M, self.C, blk.n1.eps,
                                win, one_col=self.C)
            l = blk.qkv
            if self.x3:   # q/k/v as hi/lo planes into the split attention kernels, O out as a pair too
                self._nt(self._op(S["ln1"]), H.rows(l.Wp), H.epilogue(S["qkv"][0], mode=H.OUT_QKVBLK, ldo=0, bias=l.bp,
                                                                       qkv=(nh, 32, WS_TOK), out_lo=S["qkv"][1]),
                         M, l.Np, Cp, cd)
                H.window_attn_fwd_x3(S["qkv"], blk.table, S["O"], nh * 32, S["lse"], P["nWin"], nh, self.C // nh, blk.scale,
                                     Hh, Ww, blk.shift, ones_col=self.C // nh, e_in=self.X3_AEXP, e_out=self.X3_AEXP)
                A_o = self._op(S["O"])
            else:
                self._nt(H.rows(S["ln1"]), H.rows(l.Wp), H.epilogue(S["qkv"], mode=H.OUT_QKVBLK, ldo=0, bias=l.bp,
                                                                     qkv=(nh, hp, WS_TOK)), M, l.Np, Cp, cd)
                H.window_attn_fwd(S["qkv"], blk.table, S["O"], nh * hp, S["lse"], P["nWin"], nh, self.C // nh, blk.scale,
                                  Hh, Ww, blk.shift, ones_col=self.C // nh, head_pad=hp)
                A_o = H.rows(S["O"])
            l = blk.proj
            self._nt(A_o, H.rows(l.Wp), H.epilogue(S["mid"], win=win, bias=l.bp, resid=x, rowscale=s_attn,
                                                  rows_per_scale=HW), M, Cp, nh * hp, cd)
        if self.fused_mlp:   # LN2 -> fc1 + GELU -> fc2 + residual in one launch
            f1, f2 = blk.fc1, blk.fc2
            H.swin_mlp_fwd(S["mid"], Cp, blk.n2.weight, blk.n2.bias, blk.n2.eps, self.C, S["ln2"], Cp, S["m2"], S["r2"],
                           f1.Wg, f1.bp, S["u"], S["h"], self.Hdp, f1.N, f2.Wg, f2.bp, s_mlp, HW, S["out"], Cp, M, Cp,
                           self.Hdp, w_split=f1.split)
            return S["out"]
        if self.x3:
            H.layernorm_fwd_x3(S["mid"], Cp, S["ln2"], Cp, blk.n2.weight, blk.n2.bias, S["m2"], S["r2"], M, self.C,
                               blk.n2.eps, one_col=self.C, x3_exp=self.X3_AEXP)
        else:
            H.layernorm_fwd(S["mid"], Cp, S["ln2"], Cp, blk.n2.weight, blk.n2.bias, S["m2"], S["r2"], M, self.C, blk.n2.eps,
                            one_col=self.C)
        l = blk.fc1
        hb = S["h"]
        E1 = (H.epilogue(hb[0], out_lo=hb[1], bias=l.bp, act=H.ACT_GELU, pre=S["u"], ones_col=l.N, pre_grad=True)
              if self.x3 else H.epilogue(hb, bias=l.bp, act=H.ACT_GELU, pre=S["u"], ones_col=l.N, pre_grad=True))
        self._nt(self._op(S["ln2"]), H.rows(l.Wp), E1, M, l.Np, Cp, cd)
        l = blk.fc2
        self._nt(self._op(S["h"]), H.rows(l.Wp), H.epilogue(S["out"], bias=l.bp, resid=S["mid"], rowscale=s_mlp,
                                                              rows_per_scale=HW), M, Cp, self.Hdp, cd)
        return S["out"]

    # ------------------------------------------------------------------------------------
    # backward
    # ------------------------------------------------------------------------------------
    def _wgrad(self, P, A, Bop, M, N, K, layer_map, wgrad, bgrad=None, ones_col=-1, ws=None, max_ctas=0):
        S = H.wgrad_splits(M, N, K)
        if self.x3:   # (gradient, activation) operands
            A.x3_exp, Bop.x3_exp = P["e_g"], self.X3_AEXP
        if max_ctas > 0:   # fewer row splits: at most max_ctas (tile, split) workgroups
            S = max(1, min(S, max_ctas // H.wgrad_tiles(N, K)))
        elif max_ctas < 0:   # more, shorter ones (-max_ctas times the splits, >= 32 rows each)
            S = min(S * -max_ctas, -(-M // 32))
        ws = P["wg_ws"] if ws is None else ws
        H.gemm_tn(A, Bop, ws, S, M, N, K, self.tn_cd)
        H.wgrad_finalize(ws, S, layer_map, wgrad, bgrad, ones_col)

    def _run_conv_job(self, P, job, ws=None, max_ctas=0):
        """A '1conv' residual conv's weight gradient (the job _resi_bwd returned).  Tap form: G and the
        conv input go to bf16 copies (the input with 1.0 in channel C for the bias), then one ring launch
        with a tap per K tile reads each operand row ~once (gemm.hip BM_TAP) instead of the fp32 im2col
        kernel's re-read per K tile."""
        if job[0] != "tap":
            self._wgrad(P, *job, ws=ws, max_ctas=max_ctas)
            return
        _, G, src, r, gw, gb = job
        Cp, C, M = self.Cp, self.C, P["M"]
        gbf, xbf = P["conv_bf"][id(r)]
        if not P["conv_halo"]:
            H.row_copy(G, Cp, M, C, H.copy_desc(gbf))
            H.row_copy(src, Cp, M, C, H.copy_desc(xbf))
        oc = 4 * Cp + C   # the center tap's channel C: 1.0 for every pixel
        self._wgrad(P, H.rows(gbf), H.im2col(xbf, P["H"], P["W"], Cp, ones_col=oc, ones_in_data=True), M, Cp, 9 * Cp,
                    r.map, gw, gb, oc, ws=ws, max_ctas=max_ctas)

    def _bias_colsum(self, P, G, M, Np, layer_map, bgrad):
        H.colsum(G, M, Np, layer_map, bgrad, P["colsum_ws"])

    def backward_from_loss(self, H_img, grads, loss_weight=1.0, charb_eps=None):
        """L1 loss (mean) against H_img, then the full backward.  grads: {param: fp32 tensor to write}.
        Returns the device loss tensor [1]."""
        P = self.cur
        B, Hh, Ww = P["B"], P["H"], P["W"]
        # E = v / img_range + ...: dL/dv = dL/dE / img_range, folded into the loss kernel's gradient scale
        # (which also scales the reported loss, undone below)
        wr = loss_weight / self.img_range
        P["e_g"] = self._x3_grad_exp(B * self.in_ch * Hh * self.scale * Ww * self.scale, wr)
        if self.upsampler == "pixelshuffledirect":
            H.l1_loss(P["E"], H_img, P["loss"], P["dE"], self.up1.Cop, wr, B, self.in_ch, Hh * self.scale,
                      Ww * self.scale, P["loss_ws"], ps_r=self.scale, charb_eps=charb_eps)
        else:
            H.l1_loss(P["E"], H_img, P["loss"], P["dE"], P.get("dE_ld", 16), wr, B, self.in_ch, Hh * self.scale,
                      Ww * self.scale, P["loss_ws"], charb_eps=charb_eps)
        if self.img_range != 1.0:
            P["loss"].mul_(self.img_range)
        self.backward(grads, P)
        return P["loss"]

    def backward_from_grad(self, gE, grads, e_off=0):
        """Backward given dL/dE (NCHW fp32), for the generic autograd path.  e_off: fp32x3 gradient-exponent shift
        (the range guard's retry, SwinIRFunction.backward)."""
        P = self.cur
        B, Hh, Ww = P["B"], P["H"], P["W"]
        # dE = gE through the same layout the loss kernel writes: reuse l1 machinery is not possible,
        # so scatter with the image->nhwc kernel (channel stride / pre-shuffle layout).
        inv = 1.0 / self.img_range   # E = v / img_range + ...
        if self.x3:   # an arbitrary upstream gradient: its exponent from its own range (one host sync)
            mx = float(gE.abs().max()) * inv
            P["e_g"] = (8 - int(math.ceil(math.log2(mx))) if mx > 0 and math.isfinite(mx) else 0) + e_off   # max -> <= 2^8
        if self.upsampler != "pixelshuffledirect":
            H.image_to_nhwc(gE.contiguous(), P["dE"], P.get("dE_ld", 16), None, inv, B, self.in_ch, Hh * self.scale,
                            Ww * self.scale)
        else:
            tmp = torch.nn.functional.pixel_unshuffle(gE.contiguous(), self.scale)   # [B, C*r*r, H, W]
            H.image_to_nhwc(tmp.contiguous(), P["dE"], self.up1.Cop, None, inv, B, tmp.shape[1], Hh, Ww)
        self.backward(grads, P)

    def backward(self, grads, P):
        cd = self.cd
        self._ax = P["e_g"]   # fp32x3: backward GEMM A operands / fp16 outputs are data gradients
        B, Hh, Ww, M = P["B"], P["H"], P["W"], P["M"]
        Cp = self.Cp
        g = lambda p: grads[p]
        # ---- reconstruction tail -------------------------------------------------------
        if self.upsampler == "pixelshuffle":
            h, w = Hh, Ww
            for r in self.ups_r:
                h, w = h * r, w * r
            c = self.last
            src = P["ups_act"][-1]
            tl = P["tail_ld"]   # the activations' row stride (a [hi | lo] pair under split_act: the hi half is read)
            # conv_last: dgrad into the pre-shuffle layout of the last upsampling conv
            r_last = self.ups_r[-1]
            if self.last_narrow_x3 and w % 64 == 0:
                H.conv3x3_narrow_dgrad_x3(P["dE"], P["dE_ld"], P["e_g"], c.w.detach(), self.in_ch, P["narrow_dws"], P["dpre"][-1],
                                          self.ups[-1].Co, r_last, B, h, w)
                H.conv3x3_narrow_wgrad_x3(P["dE"], P["dE_ld"], P["e_g"], src, tl, self.X3_AEXP, self.in_ch, P["narrow_ws"], g(c.w),
                                          g(c.b), B, h, w)
            elif c.narrow and w % 64 == 0:   # the narrow-output kernels (rolling row window, fp32 master weight)
                H.conv3x3_narrow_dgrad(P["dE"], 16, c.w.detach(), self.in_ch, P["narrow_dws"], P["dpre"][-1], self.ups[-1].Co,
                                       r_last, B, h, w)
                H.conv3x3_narrow_wgrad(P["dE"], 16, src, tl, self.in_ch, P["narrow_ws"], g(c.w), g(c.b), B, h, w)
            else:
                self._nt(H.im2col(P["dE"], h, w, 16, flip=True), H.rows(c.Wd),
                          H.epilogue(P["dpre"][-1], mode=H.OUT_PUNSHUF_SPM, ldo=self.ups[-1].Co,
                                     ps=(r_last, h // r_last, w // r_last)),
                          B * h * w, 64, 9 * 16, cd)
                self._wgrad(P, H.rows(P["dE"]), H.im2col(src, h, w, 64, ld=tl), B * h * w, 16, 9 * 64, c.map, g(c.w))
                self._bias_colsum(P, H.rows(P["dE"]), B * h * w, 16, c.mapb, g(c.b))
            # upsampling convs, last to first
            for i in range(len(self.ups) - 1, -1, -1):
                c, r = self.ups[i], self.ups_r[i]
                h, w = h // r, w // r
                dpre = P["dpre"][i]
                src = P["ups_act"][i - 1] if i > 0 else P["a0"]
                wr_d = (c.wr_pair and self.conv_wr and H.conv3x3_wr_tile(0, B, h, w, c.Co, 64) > 0 and
                        B * h * w // 96 >= self.conv_wr_min_tiles)
                if wr_d and i > 0:   # kair_conv3x3_wr: PixelUnshuffle store into the previous conv's pre-shuffle rows
                    rp = self.ups_r[i - 1]
                    H.conv3x3_wr(dpre, c.Co, 1, c.Wp16, None, None, P["dpre"][i - 1], B, h, w, c.Co, 64,
                                 ldo=self.ups[i - 1].Co, split=False, ps_r=-rp)
                elif wr_d:           # ... or the LeakyReLU'(a0) gate of conv_before_upsample's output
                    H.conv3x3_wr(dpre, c.Co, 1, c.Wp16, None, None, P["da0"], B, h, w, c.Co, 64, split=False,
                                 gate=P["a0"], ldg=tl, slope=0.01)
                elif i > 0:
                    rp = self.ups_r[i - 1]
                    self._nt(H.im2col(dpre, h, w, c.Co, flip=True), H.rows(c.Wd),
                              H.epilogue(P["dpre"][i - 1], mode=H.OUT_PUNSHUF_SPM, ldo=self.ups[i - 1].Co,
                                         ps=(rp, h // rp, w // rp)),
                              B * h * w, 64, 9 * c.Co, cd)
                else:
                    self._nt(H.im2col(dpre, h, w, c.Co, flip=True), H.rows(c.Wd),
                              H.epilogue(P["da0"], gate=P["a0"], ldg=tl, gate_kind=2, slope=0.01), M, 64, 9 * c.Co, cd)
                self._wgrad(P, H.rows(dpre), H.im2col(src, h, w, 64, ld=tl), B * h * w, c.Co, 9 * 64, c.map, g(c.w))
                self._bias_colsum(P, H.rows(dpre), B * h * w, c.Co, c.mapb, g(c.b))
            c = self.cbu
            if (c.wr_n64 and self.conv_wr and H.conv3x3_wr_tile(0, B, Hh, Ww, 64, Cp) > 0 and
                    M // 96 >= self.conv_wr_min_tiles):
                H.conv3x3_wr(P["da0"], 64, 1, c.Wc16, None, None, P["dfb"], B, Hh, Ww, 64, Cp, split=False)
            else:
                self._nt(H.im2col(P["da0"], Hh, Ww, 64, flip=True), H.rows(c.Wd), H.epilogue(P["dfb"]), M, Cp, 9 * 64, cd)
            self._wgrad(P, H.rows(P["da0"]), H.im2col(P["fb"], Hh, Ww, Cp, ones_col=self.C), M, 64, 9 * Cp, c.map,
                        g(c.w), g(c.b), self.C)
        elif self.upsampler == "nearest+conv":
            self._nearest_tail_bwd(P, grads)
        else:   # pixelshuffledirect (one conv + PixelShuffle) or the denoising conv_last (E = x + conv_last / range)
            c = self.up1 if self.upsampler == "pixelshuffledirect" else self.last
            self._nt(H.im2col(P["dE"], Hh, Ww, c.Cop, flip=True), H.rows(c.Wd), H.epilogue(P["dfb"]), M, Cp, 9 * c.Cop, cd)
            self._wgrad(P, H.rows(P["dE"]), H.im2col(P["fb"], Hh, Ww, Cp, ones_col=self.C), M, c.Cop, 9 * Cp, c.map,
                        g(c.w), g(c.b), self.C)
        # ---- conv_after_body (fb = cab(nf) + f0) ------------------------------------------
        G, D = P["G"], P["D"]
        job = self._resi_bwd(self.cab, P, P["dfb"], P["nf"], D, grads)
        if job is not None:
            self._run_conv_job(P, job)
        # ---- final norm: nf = LN(u_G) -----------------------------------------------------
        n = self.norm
        last_in = P["rstb_out"][-1]
        H.layernorm_bwd(last_in, Cp, D, Cp, n.weight, P["n_mean"], P["n_rstd"], G, Cp, False, g(n.weight), g(n.bias), False,
                        P["ln_ws"], M, self.C)
        self._segment_done()   # reconstruction tail + conv_after_body + norm gradients are final
        # G = dL/d u_G
        bi = len(self.blocks)
        # Each RSTB's deferred gradient work (the grouped block weight gradients, LayerNorm-parameter and
        # bias-table reductions, the RSTB conv's weight gradient) runs on a side stream beside the NEXT
        # RSTB's data-gradient chain, and is joined at the end of that chain, where RSTB gi's gradient
        # segment is reported (seg_hook: DDP bucket).  So that the chain never overwrites what the
        # side stream still reads: the per-block operand sets alternate by RSTB parity (gw[gi % 2]) and
        # the residual-stream gradient rotates through three buffers (the conv weight gradient reads the
        # G that entered the RSTB; the chain two RSTBs later is the first to write that buffer again).
        bufs = [G, D, P["G3"]]
        side_open = side_pending = False
        for gi in range(len(self.rstb) - 1, -1, -1):
            blks, conv = self.rstb[gi]
            G, D, par = bufs[0], bufs[1], gi % 2
            t_d = P["blocks"][bi - 1]["out"]
            # u_{g+1} = conv(t_d) + u_g : conv dgrad -> D = dL/dt_d
            job = self._resi_bwd(conv, P, G, t_d, D, grads)
            if side_pending:   # RSTB gi + 1's deferred work, forked behind this conv (which it would starve)
                side_open = self._flush_deferred(P)
                side_pending = False
            if job is not None:
                self._conv_pending.append(job)
            # GEMM-operand copy of D for the last block's MLP branch: s_mlp * D in compute dtype
            drop = P["drop"]
            H.row_copy(D, Cp, M, Cp, H.copy_desc(P["gw"][par][len(blks) - 1]["Dm"],
                                                 rowscale=drop[bi - 1, 1] if drop is not None else None,
                                                 rows_per_scale=Hh * Ww, x3_exp=P["e_g"]))
            for j in range(len(blks) - 1, -1, -1):
                bi -= 1
                x_in = P["blocks"][bi - 1]["out"] if j > 0 else (P["rstb_out"][gi - 1] if gi > 0 else P["s0"])
                self._block_bwd(blks[j], P, P["blocks"][bi], x_in, D, bi, grads, j, par)
            H.axpy(D, G, 1.0)   # dL/du_g = skip + blocks path (into D: G stays intact for the conv's wgrad)
            bufs = [D, bufs[2], G]
            if side_open:   # RSTB gi + 1's deferred work ran beside this chain: join, report its segment
                torch.cuda.current_stream().wait_stream(self._side)
                self._segment_done()
                side_open = False
            if self.side_stream:
                side_pending = True     # forked at the next RSTB (or below, after the last one)
            else:
                self._flush_deferred(P)
                if gi > 0:
                    self._segment_done()   # RSTB gi's gradients are final (RSTB 0 joins the head segment)
        if side_pending:
            self._flush_deferred(P)
        if side_pending or side_open:
            torch.cuda.current_stream().wait_stream(self._side)
        G = bufs[0]
        # ---- patch_embed norm: s0 = LN(f0); f0 also feeds fb (long skip) --------------------
        n = self.pe_norm
        H.layernorm_bwd(P["f0"], Cp, G, Cp, n.weight, P["pe_mean"], P["pe_rstd"], P["dfb"], Cp, True, g(n.weight),
                        g(n.bias), False, P["ln_ws"], M, self.C)
        c = self.conv_first
        self._wgrad(P, H.rows(P["dfb"]), H.im2col(P["xin"], Hh, Ww, self.Cin_p, ones_col=self.in_ch), M, Cp,
                    9 * self.Cin_p, c.map, g(c.w), g(c.b), self.in_ch)

    def _nearest_tail_bwd(self, P, grads):
        """'nearest+conv' reconstruction backward (network_swinir.py:824-830): conv_last, conv_hr and the
        two conv(nearest x2) stages, each input gradient gated by LeakyReLU' in the dgrad epilogue (conv_hr,
        conv_up2) or after the 2x2 sum-pool that is nearest x2's adjoint (conv_up2 -> up1 -> cbu);
        ends with P['dfb'] = dL/d fb."""
        cd, B, Hh, Ww, M, Cp = self.cd, P["B"], P["H"], P["W"], P["M"], self.Cp
        g = lambda p: grads[p]
        h, w = 4 * Hh, 4 * Ww
        ML = B * h * w
        c = self.last
        self._nt(H.im2col(P["dE"], h, w, 16, flip=True), H.rows(c.Wd),
                  H.epilogue(P["dz_hr"], gate=P["nhr"], gate_kind=2, slope=0.2), ML, 64, 9 * 16, cd)
        self._wgrad(P, H.rows(P["dE"]), H.im2col(P["nhr"], h, w, 64), ML, 16, 9 * 64, c.map, g(c.w))
        self._bias_colsum(P, H.rows(P["dE"]), ML, 16, c.mapb, g(c.b))
        c = self.hrc
        self._nt(H.im2col(P["dz_hr"], h, w, 64, flip=True), H.rows(c.Wd),
                  H.epilogue(P["dz_u"], gate=P["nup_act"][1], gate_kind=2, slope=0.2), ML, 64, 9 * 64, cd)
        self._wgrad(P, H.rows(P["dz_hr"]), H.im2col(P["nup_act"][1], h, w, 64), ML, 64, 9 * 64, c.map, g(c.w))
        self._bias_colsum(P, H.rows(P["dz_hr"]), ML, 64, c.mapb, g(c.b))
        dz = P["dz_u"]
        for i in (1, 0):   # conv_up2 then conv_up1: dz = dL/d(pre-activation) on the (h, w) grid
            c = self.nup[i]
            Mi = B * h * w
            src = P["nup_act"][0] if i == 1 else P["a0"]
            G_hi = P["G_hi"][:Mi]
            self._nt(H.im2col(dz, h, w, 64, flip=True), H.rows(c.Wd), H.epilogue(G_hi), Mi, 64, 9 * 64, cd)
            self._wgrad(P, H.rows(dz), H.im2col(src, h, w, 64, up=2), Mi, 64, 9 * 64, c.map, g(c.w))
            self._bias_colsum(P, H.rows(dz), Mi, 64, c.mapb, g(c.b))
            h, w = h // 2, w // 2
            Mo = B * h * w
            G_lo = P["G_lo"][:Mo]
            H.sumpool2x(G_hi, 64, G_lo, 64, B, h, w, 64)
            nxt = P["dz_hr"][:Mo] if i == 1 else P["da0"]      # dz_hr is free again after conv_hr's wgrad
            H.act_grad_cast(G_lo, 64, src, 64, nxt, 64, Mo, 64, 2, 0.2 if i == 1 else 0.01)
            dz = nxt
        c = self.cbu
        self._nt(H.im2col(P["da0"], Hh, Ww, 64, flip=True), H.rows(c.Wd), H.epilogue(P["dfb"]), M, Cp, 9 * 64, cd)
        self._wgrad(P, H.rows(P["da0"]), H.im2col(P["fb"], Hh, Ww, Cp, ones_col=self.C), M, 64, 9 * Cp, c.map,
                    g(c.w), g(c.b), self.C)

    def _wg(self, P, A, Bop, N, K, lin, grads, ones_col):
        """One block linear's weight gradient: queued for the RSTB's grouped launch, or issued now."""
        g_w, g_b = grads[lin.w], grads[lin.b]
        if self.grouped_wgrad or (self.x3_side and (self.side_stream or self.x3_grouped)):
            self._wg_pending.append((A, Bop, N, K, lin.map, g_w, g_b, ones_col))
        else:
            self._wgrad(P, A, Bop, P["M"], N, K, lin.map, g_w, g_b, ones_col)

    def _flush_deferred(self, P):
        """Issue the RSTB's deferred gradient work: on the side stream when the block weight gradients
        are grouped (returns True: the caller joins it), else in place on the current stream."""
        side = None
        if self.side_stream:
            if self._side is None:
                self._side = torch.cuda.Stream(device=self.device, priority=self.side_priority)
            side = self._side
            side.wait_stream(torch.cuda.current_stream())
        ws = P["wg_ws2"] if side is not None else P["wg_ws"]
        cap = (self.side_ctas if not self.side_ctas_auto else (96 if P["M"] < 36864 else 192)) if side is not None else 0
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            if self._wg_pending:
                jobs, self._wg_pending = self._wg_pending, []
                if self.x3:   # fp16-pair operands at the step's exponents (gradient, activation)
                    for A, Bop, *_ in jobs:
                        A.x3_exp, Bop.x3_exp = P["e_g"], self.X3_AEXP
                if self.x3 and not (self.x3_grouped and all(
                        A.dtype == H.F16 and Bop.dtype == H.F16 and A.win_ws == 0 and Bop.win_ws == 0
                        for A, Bop, *_ in jobs)):   # one split-fp16 TN ring + finalize per linear, in queue order
                    for A, Bop, N, K, m, g_w, g_b, oc in jobs:
                        self._wgrad(P, A, Bop, P["M"], N, K, m, g_w, g_b, oc, ws=ws, max_ctas=cap)
                else:
                    for i in range(0, len(jobs), H.WgradGroup.WG_MAX):
                        H.WgradGroup(jobs[i:i + H.WgradGroup.WG_MAX], P["M"]).run(ws, max_ctas=cap)
            # grouped launches take at most 32 jobs each (LNP_MAX / DTAB_MAX): deep RSTBs run in chunks
            if self._lnp_pending:
                jobs, self._lnp_pending = self._lnp_pending, []
                for i in range(0, len(jobs), H.GROUP_MAX):
                    H.ln_param_reduce_grouped(jobs[i:i + H.GROUP_MAX])
            if self._dtab_pending:
                jobs, self._dtab_pending = self._dtab_pending, []
                for i in range(0, len(jobs), H.GROUP_MAX):
                    H.attn_dtable_grouped(jobs[i:i + H.GROUP_MAX])
            jobs, self._conv_pending = self._conv_pending, []
            for job in jobs:
                self._run_conv_job(P, job, ws=ws, max_ctas=cap)
        return side is not None

    def _block_bwd(self, blk, P, S, x_in, D, bi, grads, j, par):
        """D: dL/d out (fp32, token rows) -> updated in place to dL/d x_in.  j: the block's position in
        its RSTB; P["gw"][j] holds this block's weight-gradient operands until the RSTB's grouped
        launch.  On entry gw[j]["Dm"] = s_mlp * D (compute dtype, token order); LN2 backward writes
        gw[j]["Da"] = s_attn * D_mid (window order, proj operand); LN1 backward, when the previous block
        is in the same RSTB, writes that block's gw[j - 1]["Dm"]."""
        cd, g = self.cd, (lambda p: grads[p])
        M, Cp, nh, Hh, Ww = P["M"], self.Cp, self.nh, P["H"], P["W"]
        HW = Hh * Ww
        win = (Hh, Ww, 8, blk.shift)
        drop = P["drop"]
        s_attn = drop[bi, 0] if drop is not None else None
        hd = self.C // nh
        W = P["gw"][par][j]
        Dm, Da, dU, dqkv = W["Dm"], W["Da"], W["dU"], W["dqkv"]
        # MLP: out = mid + s_mlp * fc2(gelu(fc1(LN2(mid))))
        fc2, fc1 = blk.fc2, blk.fc1
        n = blk.n2
        self._wg(P, self._op(Dm), self._op(S["h"], ones_col=fc2.K, ones_in_data=True), Cp, self.Hdp, fc2, grads, fc2.K)
        if self.fused_mlp_bwd:
            # fc2 / fc1 input gradients + LN2 backward in one launch
            H.swin_mlp_bwd(Dm, S["u"], fc2.Wgt, fc1.Wgt, dU, S["mid"], n.weight, S["m2"], S["r2"], self.C, D, Da,
                           s_attn, HW, Hh, Ww, blk.shift, g(n.weight), g(n.bias), P["mlp_ws"], M, Cp, self.Hdp)
        elif self.rowgemm:
            # S["u"] holds GELU'(fc1 pre-activation), stored by the forward: the fc2 input gradient is gated
            H.rowgemm_gate(Dm, M, Cp, fc2.Wgt, self.Hdp, S["u"], dU)
            # fc1 input gradient -> LN2 backward into D, the window-order proj operand Da = s_attn * dL/dmid
            H.rowgemm_lnbwd(dU, M, self.Hdp, fc1.Wgt, S["mid"], n.weight, S["m2"], S["r2"], self.C, D, W["ln2p"],
                            copy=H.copy_desc(Da, rowscale=s_attn, rows_per_scale=HW, win=win))
            self._lnp_pending.append((W["ln2p"], M, self.C, g(n.weight), g(n.bias), False, P["rg_nb"][self.Hdp]))
        else:
            # S["u"] holds GELU'(fc1 pre-activation), stored by the forward (pre_grad): a plain multiply here
            Eu = (H.epilogue(dU[0], out_lo=dU[1], gate=S["u"], gate_kind=4) if self.x3 else
                  H.epilogue(dU, gate=S["u"], gate_kind=4))
            self._nt(self._op(Dm), H.rows(fc2.Wt), Eu, M, self.Hdp, Cp, cd)
            cpy = H.copy_desc(Da, rowscale=s_attn, rows_per_scale=HW, win=win, x3_exp=P["e_g"])
            if self.x3_lnfuse:   # fc1 input gradient + LN2 backward in one launch
                self._nt_lnbwd(self._op(dU), H.rows(fc1.Wt), M, self.Hdp, S["mid"], n.weight, S["m2"], S["r2"], D,
                               W["ln2p"], copy=cpy)
                self._lnp_pending.append((W["ln2p"], M, self.C, g(n.weight), g(n.bias), False,
                                          H.gemm_nt_lnbwd_parts(M, Cp)))
            else:
                self._nt(self._op(dU), H.rows(fc1.Wt), H.epilogue(P["dxn"]), M, Cp, self.Hdp, cd)
                H.layernorm_bwd(S["mid"], Cp, P["dxn"], Cp, n.weight, S["m2"], S["r2"], D, Cp, True, None, None, False,
                                W["ln2p"], M, self.C, copy=cpy)
                self._lnp_pending.append((W["ln2p"], M, self.C, g(n.weight), g(n.bias), False))
        self._wg(P, self._op(dU), self._op(S["ln2"], ones_col=self.C, ones_in_data=True), self.Hdp, Cp, fc1, grads, self.C)
        # attention: mid = x + s_attn * proj(attn(LN1(x)))   (window order inside)
        proj, qkv = blk.proj, blk.qkv
        if self.x3:
            self._block_bwd_attn_x3(blk, P, S, x_in, D, bi, grads, j, par)
            return
        hp = self.hp
        self._wg(P, H.rows(Da), H.rows(S["O"], ones_col=hd, ones_in_data=True), Cp, nh * hp, proj, grads, hd)
        if self.rowgemm:
            H.rowgemm_store(Da, M, Cp, proj.Wgt, Cp, P["dO"])
        else:
            self._nt(H.rows(Da), H.rows(proj.Wt), H.epilogue(P["dO"]), M, nh * hp, Cp, cd)
        rows = self.rowgemm   # dq/dk/dv as token rows [M][3 nh 32]: the row GEMM's A operand
        H.window_attn_bwd(S["qkv"], S["O"], nh * hp, P["dO"], nh * hp, blk.table, S["lse"], dqkv, None, False,
                          W["attn_ws"], P["nWin"], nh, hd, blk.scale, Hh, Ww, blk.shift, dqkv_rows=rows, head_pad=hp)
        self._dtab_pending.append((W["attn_ws"], P["nWin"], nh, self.cd, g(blk.table), False))
        A_qkv = H.rows(dqkv.view(M, qkv.Np)) if rows else H.qkvblk(dqkv, nh, hdp=hp)
        self._wg(P, A_qkv, H.rows(S["ln1"], ones_col=self.C, ones_in_data=True), qkv.Np, Cp, qkv, grads, self.C)
        n = blk.n1
        cp = None
        if j > 0:   # the previous block's MLP operand: s_mlp(prev) * dL/d x_in
            cp = H.copy_desc(P["gw"][par][j - 1]["Dm"], rowscale=drop[bi - 1, 1] if drop is not None else None,
                             rows_per_scale=HW)
        if rows:
            # q/k/v input gradient (rows in window order) -> LN1 backward into D (+ the previous block's operand)
            H.rowgemm_lnbwd(dqkv.view(M, qkv.Np), M, qkv.Np, qkv.Wgt, x_in, n.weight, S["m1"], S["r1"], self.C, D,
                            W["ln1p"], win=win, copy=cp)
            self._lnp_pending.append((W["ln1p"], M, self.C, g(n.weight), g(n.bias), False, P["rg_nb"][qkv.Np]))
        else:
            self._nt(H.qkvblk(dqkv, nh, hdp=hp), H.rows(qkv.Wt), H.epilogue(P["dxn"]), M, Cp, qkv.Np, cd)
            H.layernorm_bwd(x_in, Cp, P["dxn"], Cp, n.weight, S["m1"], S["r1"], D, Cp, True, None, None, False,
                            W["ln1p"], M, self.C, win, copy=cp)
            self._lnp_pending.append((W["ln1p"], M, self.C, g(n.weight), g(n.bias), False))


    def _block_bwd_attn_x3(self, blk, P, S, x_in, D, bi, grads, j, par):
        """The attention half of _block_bwd under fp32x3: q/k/v and dO as hi/lo fp16 planes, O and dq/dk/dv fp32, the
        split attention backward, split GEMMs (kair_gemm_nt / kair_gemm_tn compute X3)."""
        cd, g = self.cd, (lambda p: grads[p])
        M, Cp, nh, Hh, Ww = P["M"], self.Cp, self.nh, P["H"], P["W"]
        HW = Hh * Ww
        win = (Hh, Ww, 8, blk.shift)
        drop = P["drop"]
        hd = self.C // nh
        W = P["gw"][par][j]
        Da, dqkv = W["Da"], W["dqkv"]
        proj, qkv = blk.proj, blk.qkv
        self._wg(P, self._op(Da), self._op(S["O"], ones_col=hd, ones_in_data=True), Cp, nh * 32, proj, grads, hd)
        self._nt(self._op(Da), H.rows(proj.Wt), H.epilogue(P["dO"][0], out_lo=P["dO"][1]), M, nh * 32, Cp, cd)
        H.window_attn_bwd_x3(S["qkv"], S["O"], nh * 32, P["dO"], nh * 32, blk.table, S["lse"], dqkv, None, False,
                             W["attn_ws"], P["nWin"], nh, hd, blk.scale, Hh, Ww, blk.shift, e_act=self.X3_AEXP,
                             e_grad=P["e_g"])
        self._dtab_pending.append((W["attn_ws"], P["nWin"], nh, H.X3, g(blk.table), False))
        self._wg(P, self._op(dqkv), self._op(S["ln1"], ones_col=self.C, ones_in_data=True), qkv.Np, Cp, qkv, grads, self.C)
        n = blk.n1
        cp = None
        if j > 0:   # the previous block's MLP operand: s_mlp(prev) * dL/d x_in
            cp = H.copy_desc(P["gw"][par][j - 1]["Dm"], rowscale=drop[bi - 1, 1] if drop is not None else None,
                             rows_per_scale=HW, x3_exp=P["e_g"])
        if self.x3_lnfuse:   # q/k/v input gradient + LN1 backward in one launch
            self._nt_lnbwd(self._op(dqkv), H.rows(qkv.Wt), M, qkv.Np, x_in, n.weight, S["m1"], S["r1"], D, W["ln1p"],
                           win=win, copy=cp)
            self._lnp_pending.append((W["ln1p"], M, self.C, g(n.weight), g(n.bias), False, H.gemm_nt_lnbwd_parts(M, Cp)))
            return
        self._nt(self._op(dqkv), H.rows(qkv.Wt), H.epilogue(P["dxn"]), M, Cp, qkv.Np, cd)
        H.layernorm_bwd(x_in, Cp, P["dxn"], Cp, n.weight, S["m1"], S["r1"], D, Cp, True, None, None, False,
                        W["ln1p"], M, self.C, win, copy=cp)
        self._lnp_pending.append((W["ln1p"], M, self.C, g(n.weight), g(n.bias), False))


class SwinIRFunction(torch.autograd.Function):
    """The whole SwinIR forward/backward as one autograd node (params are inputs so that any
    optimizer / DDP reducer sees ordinary .grad tensors).

    The node leases its plan (kair_amd/engine/plans.py) from forward to backward, so two forwards
    before one backward each keep their own saved activations; no-grad forwards use a small
    inference plan."""

    @classmethod
    def run(cls, engine, x, params):
        """Entry point: the plan mode is decided here, where the caller's grad mode is visible
        (inside Function.forward autograd has switched it off)."""
        return cls.apply(engine, autograd_mode(params), x, *params)

    @staticmethod
    def forward(ctx, engine, mode, x, *params):
        net = engine.net_ref()
        B, C, H0, W0 = x.shape
        ws = engine.ws
        ph, pw = (ws - H0 % ws) % ws, (ws - W0 % ws) % ws
        if ph or pw:   # check_image_size (network_swinir.py:783-788)
            x = torch.nn.functional.pad(x, (0, pw, 0, ph), "reflect")
        drop = None
        if mode == "lease" and net.training and any(b.dp > 0 for b in engine.blocks):
            drop = drop_path_scales(engine, x.shape[0], x.device)
        with plan_mode(engine, mode):
            E = engine.forward(x.float(), drop)
            # fp32x3 range guard (eager path, one host sync): an activation that left the fp16 window shows as a
            # non-finite output -> lower the exponents and run the forward again (the trainer's graph step has the
            # same guard on device, FusedTrainer._check_range)
            while engine.x3 and not bool(torch.isfinite(E).all()):
                if not bool(torch.isfinite(x).all()):
                    raise RuntimeError("kair_amd SwinIR: non-finite input")
                engine.x3_backoff(act=True, grad=False)
                E = engine.forward(x.float(), drop)
        ctx.engine = engine
        ctx.params = params
        ctx.lease = Lease(engine.cur) if mode == "lease" else None
        out = E[:, :, :H0 * engine.scale, :W0 * engine.scale]
        return out.clone() if (ph or pw) else E.clone()

    @staticmethod
    def backward(ctx, gE):
        eng = ctx.engine
        if ctx.lease is None or ctx.lease.plan is None:
            raise RuntimeError("kair_amd SwinIR: backward through a forward whose activations were released "
                               "(a second backward needs retain_graph-style reuse, which is not supported)")
        flat = torch.empty(sum(p.numel() for p in ctx.params), device=gE.device)
        grads, off = {}, 0
        for p in ctx.params:
            grads[p] = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        P = ctx.lease.plan
        eng.cur = P
        full = gE
        if gE.shape[-2:] != P["E"].shape[-2:]:
            full = torch.zeros_like(P["E"])
            full[:, :, :gE.shape[2], :gE.shape[3]] = gE
        eng.backward_from_grad(full.float(), grads)
        if eng.x3 and bool(torch.isfinite(full).all()):
            # range guard: a data gradient that left the fp16 window makes the parameter gradients non-finite ->
            # rerun the backward (the saved activations are unchanged) with the gradient exponent lowered
            e_off = 0
            while not bool(torch.isfinite(flat).all()):
                if e_off <= -eng.X3_BACKOFF_STEP * eng.X3_BACKOFF_MAX:
                    raise RuntimeError("fp32x3 range guard: the backward stays non-finite after exponent back-offs")
                e_off -= eng.X3_BACKOFF_STEP
                eng.backward_from_grad(full.float(), grads, e_off=e_off)
        ctx.lease.release()
        return (None, None, None) + tuple(grads[p] for p in ctx.params)


def drop_path_scales(engine, B, device, generator=None):
    """Per-block, per-branch stochastic-depth scales (timm DropPath semantics: keep-mask / keep)."""
    keep = getattr(engine, "_keep", None)
    if keep is None or keep.device != torch.device(device):   # built once, outside any graph capture
        rates = torch.tensor([b.dp for b in engine.blocks], dtype=torch.float32)
        keep = engine._keep = (1.0 - rates).view(-1, 1, 1).to(device)
    u = torch.rand(len(engine.blocks), 2, B, device=device, generator=generator)
    return (u < keep).float() / keep
