"""ctypes binding of libkair_hip.so (include/kair_hip.h).

This is the ONLY way the product reaches its kernels.  There is no CPU or PyTorch fallback: if the
library is missing or a call fails, a RuntimeError is raised (tests/test_boundary.py checks both).
Tensors are passed as raw device pointers; the current torch stream is passed explicitly.
"""
import ctypes
import os

import torch

# KAIR_LIB=debug: the debug-ablation build (python -m kair_amd.build --debug-ablations), for the
# perf-investigation tools only; the release library is the default and the only one tests / bench use
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                        {"debug": "libkair_hip_dbg.so", "base": "libkair_hip_base.so"}.get(os.environ.get("KAIR_LIB"),
                                                                                          "libkair_hip.so"))
# KAIR_LIB=base: an A/B baseline library (same ABI, earlier sources) placed there by hand; never shipped

F32, BF16, F16 = 0, 1, 3
X3 = 2   # KAIR_COMPUTE_X3: split-fp16 arithmetic (hi.hi + hi.lo + lo.hi of power-of-2-scaled fp16 pairs)
X3_WEXP = 12   # KAIR_X3_WEXP: the exponent of the fp16 weight packs
LD_ROWS, LD_IM2COL3, LD_QKVBLK, LD_S2D = 0, 1, 2, 3
USR_SRC_NCHW, USR_SRC_PSF, USR_SRC_ZUP, USR_SRC_NHWC = 0, 1, 2, 3
USR_COL_FB, USR_COL_FBFY, USR_COL_DATA_FWD, USR_COL_DATA_BWD = 0, 1, 2, 3
USR_CHAN_CHUNKS = 64
USR_PAD_REPLICATE, USR_PAD_ZERO, USR_PAD_FOLD, USR_CROP_NCHW = 0, 1, 2, 3
OUT_ROWS, OUT_QKVBLK, OUT_PSHUF, OUT_PUNSHUF, OUT_NCHW, OUT_PSHUF_NCHW = 0, 1, 2, 3, 4, 5
OUT_PSHUF_SPM, OUT_PUNSHUF_SPM = 6, 7
ACT_NONE, ACT_GELU, ACT_LEAKY, ACT_RELU = 0, 1, 2, 3

c_long, c_int, c_float, c_vp = ctypes.c_long, ctypes.c_int, ctypes.c_float, ctypes.c_void_p


class Operand(ctypes.Structure):
    _fields_ = [("ptr", c_vp), ("dtype", c_int), ("mode", c_int), ("ld", c_long),
                ("win_H", c_int), ("win_W", c_int), ("win_ws", c_int), ("win_shift", c_int),
                ("im_H", c_int), ("im_W", c_int), ("im_C", c_int), ("im_flip", c_int),
                ("qkv_nh", c_int), ("qkv_hdp", c_int), ("qkv_tok", c_int),
                ("rowscale", c_vp), ("rows_per_scale", c_int), ("ones_col", c_int), ("ones_in_data", c_int),
                ("im_up", c_int), ("w_split", c_int), ("a_split", c_int), ("lo_ptr", c_vp), ("x3_exp", c_int)]


class CopyDesc(ctypes.Structure):
    _fields_ = [("out", c_vp), ("dtype", c_int), ("ld", c_long), ("rowscale", c_vp), ("rows_per_scale", c_int),
                ("win_H", c_int), ("win_W", c_int), ("win_ws", c_int), ("win_shift", c_int), ("out_lo", c_vp),
                ("x3_exp", c_int)]


def copy_desc(out, ld=None, rowscale=None, rows_per_scale=1, win=None, x3_exp=0):
    """Row-scaled cast copy target (GEMM A operand); win puts the rows in Swin window order.  out an fp16 pair
    [2, ...] (hi plane, lo plane): the x3 pair of v 2^x3_exp."""
    d = CopyDesc()
    d._keep = (out, rowscale)
    if out.dtype == torch.float16:
        d.out, d.out_lo, d.dtype, d.x3_exp = ptr(out[0]), ptr(out[1]), F16, int(x3_exp)
    else:
        d.out, d.dtype = ptr(out), dtype_code(out)
    d.ld = ld if ld is not None else out.shape[-1]
    d.rowscale, d.rows_per_scale = ptr(rowscale), rows_per_scale
    if win:
        d.win_H, d.win_W, d.win_ws, d.win_shift = win
    return d


class Epilogue(ctypes.Structure):
    _fields_ = [("out", c_vp), ("out_dtype", c_int), ("out_mode", c_int), ("ldo", c_long),
                ("win_H", c_int), ("win_W", c_int), ("win_ws", c_int), ("win_shift", c_int),
                ("bias", c_vp), ("act", c_int), ("slope", c_float),
                ("out_pre", c_vp), ("pre_dtype", c_int), ("ldp", c_long),
                ("resid", c_vp), ("ldr", c_long),
                ("rowscale", c_vp), ("rows_per_scale", c_int),
                ("gate", c_vp), ("gate_dtype", c_int), ("ldg", c_long), ("gate_kind", c_int),
                ("ps_r", c_int), ("ps_H", c_int), ("ps_W", c_int),
                ("qkv_nh", c_int), ("qkv_hdp", c_int), ("qkv_tok", c_int),
                ("img_mean", c_vp), ("img_range", c_float), ("img_C", c_int), ("img_H", c_int), ("img_W", c_int),
                ("out_ones_col_p1", c_int), ("resid2", c_vp), ("ldr2", c_long), ("pre_kind", c_int),
                ("a_copy", c_vp), ("ld_acopy", c_long), ("acopy_ones_col_p1", c_int), ("out_lo", c_vp),
                ("x3_out_exp", c_int)]


class WMap(ctypes.Structure):
    _fields_ = [("kind", c_int), ("N", c_int), ("K", c_int), ("nG", c_int), ("nGr", c_int), ("nGp", c_int),
                ("kG", c_int), ("kGr", c_int), ("kGp", c_int), ("n_perm", c_int)]


class WgradJob(ctypes.Structure):
    _fields_ = [("A", Operand), ("B", Operand), ("N", c_int), ("K", c_int), ("map", WMap), ("grad", c_vp),
                ("bias_grad", c_vp), ("ones_col", c_int)]


class LnParamJob(ctypes.Structure):
    _fields_ = [("part", c_vp), ("nb", c_long), ("C", c_int), ("dgamma", c_vp), ("dbeta", c_vp), ("accumulate", c_int)]


class DtabJob(ctypes.Structure):
    _fields_ = [("ws", c_vp), ("nWin", c_long), ("nh", c_int), ("dtype", c_int), ("dtable", c_vp), ("accumulate", c_int)]


class PackJob(ctypes.Structure):
    _fields_ = [("src", c_vp), ("dst", c_vp), ("dst_dtype", c_int), ("reserved", c_int), ("map", WMap),
                ("total", c_long)]


_SIGS = {
    "kair_gemm_nt": [ctypes.POINTER(Operand), ctypes.POINTER(Operand), ctypes.POINTER(Epilogue), c_long, c_int, c_int,
                     c_int, c_vp],
    "kair_wgrad_splits": [c_long, c_int, c_int],
    "kair_conv3x3_halo_geometry": [c_int, c_int, c_int, c_long, c_int],
    "kair_gemm_tn": [ctypes.POINTER(Operand), ctypes.POINTER(Operand), c_vp, c_int, c_long, c_int, c_int, c_int, c_vp],
    "kair_wgrad_grouped_ws": [ctypes.POINTER(WgradJob), c_int, c_long],
    "kair_wgrad_grouped": [ctypes.POINTER(WgradJob), c_int, c_long, c_vp, c_vp],
    "kair_wgrad_grouped_ex": [ctypes.POINTER(WgradJob), c_int, c_long, c_vp, c_int, c_vp],
    "kair_layernorm_bwd_blocks": [c_long],
    "kair_ln_param_reduce_grouped": [ctypes.POINTER(LnParamJob), c_int, c_vp],
    "kair_window_attn_bwd_groups": [c_long, c_int, c_int],
    "kair_attn_dtable_grouped": [ctypes.POINTER(DtabJob), c_int, c_vp],
    "kair_pack_weight": [c_vp, c_vp, c_int, ctypes.POINTER(WMap), c_vp],
    "kair_pack_table_bytes": [c_int],
    "kair_pack_table_build": [ctypes.POINTER(PackJob), c_int, c_vp],
    "kair_pack_weights": [c_vp, c_int, c_long, c_vp],
    "kair_wgrad_finalize": [c_vp, c_int, ctypes.POINTER(WMap), c_vp, c_vp, c_int, c_int, c_vp],
    "kair_colsum": [ctypes.POINTER(Operand), c_long, c_int, ctypes.POINTER(WMap), c_vp, c_vp, c_int, c_vp],
    "kair_layernorm_fwd": [c_vp, c_long, c_vp, c_int, c_long, c_vp, c_vp, c_vp, c_vp, c_long, c_int, c_float, c_int,
                           c_int, c_int, c_int, c_int, c_vp],
    "kair_layernorm_fwd_x3": [c_vp, c_long, c_vp, c_vp, c_long, c_vp, c_vp, c_vp, c_vp, c_long, c_int, c_float, c_int,
                              c_int, c_int, c_int, c_int, c_int, c_vp],
    "kair_layernorm_bwd": [c_vp, c_long, c_vp, c_int, c_long, c_vp, c_vp, c_vp, c_vp, c_long, c_int, c_vp, c_vp, c_int,
                           c_vp, c_long, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(CopyDesc), c_vp],
    "kair_row_copy": [c_vp, c_long, c_long, c_int, ctypes.POINTER(CopyDesc), c_vp],
    "kair_gemm_nt_x3_lnbwd": [ctypes.POINTER(Operand), ctypes.POINTER(Operand), c_long, c_int, c_int, c_int, c_int, c_int,
                              c_int, c_vp, c_long, c_vp, c_vp, c_vp, c_int, c_vp, c_long, c_vp, ctypes.POINTER(CopyDesc),
                              c_vp],
    "kair_gemm_nt_x3_lnbwd_parts": [c_long, c_int],
    "kair_window_attn_fwd": [c_vp, c_int, c_vp, c_vp, c_long, c_vp, c_long, c_int, c_int, c_float, c_int, c_int, c_int,
                             c_int, c_vp, c_int, c_vp],
    "kair_window_attn_bwd_ws": [c_long, c_int],
    "kair_window_attn_bwd": [c_vp, c_vp, c_long, c_vp, c_long, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_long, c_int,
                             c_int, c_float, c_int, c_int, c_int, c_vp, c_int, c_vp],
    "kair_window_attn_bwd_ex": [c_vp, c_vp, c_long, c_vp, c_long, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp, c_long,
                                c_int, c_int, c_float, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp],
    "kair_window_attn_fwd_ex": [c_vp, c_int, c_vp, c_vp, c_long, c_vp, c_long, c_int, c_int, c_float, c_int, c_int, c_int,
                                c_int, c_vp, c_int, c_int, c_vp],
    "kair_image_to_nhwc": [c_vp, c_vp, c_int, c_int, c_vp, c_float, c_int, c_int, c_int, c_int, c_vp],
    "kair_image_to_nhwc_hilo": [c_vp, c_vp, c_int, c_vp, c_float, c_int, c_int, c_int, c_int, c_vp],
    "kair_conv3x3_narrow_fwd": [c_vp, c_long, c_int, c_vp, c_vp, c_int, c_vp, c_float, c_vp, c_vp, c_int, c_int, c_int,
                                c_vp],
    "kair_conv3x3_wr_tile": [c_int, c_int, c_int, c_int, c_int, c_int],
    "kair_conv3x3_wr": [c_vp, c_int, c_long, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_long, c_vp, c_int, c_long, c_vp,
                        c_long, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "kair_conv3x3_wr_ex": [c_vp, c_int, c_long, c_int, c_int, c_vp, c_int, c_vp, c_vp, c_long, c_vp, c_int, c_long, c_vp,
                           c_int, c_int, c_float, c_vp, c_long, c_vp, c_long, c_int, c_int, c_int, c_int, c_int, c_int,
                           c_vp],
    "kair_conv3x3_narrow_dgrad_ws": [],
    "kair_conv3x3_narrow_dgrad": [c_vp, c_long, c_vp, c_int, c_vp, c_vp, c_int, c_long, c_int, c_int, c_int, c_int, c_vp],
    "kair_conv3x3_narrow_wgrad_ws": [c_int],
    "kair_conv3x3_narrow_wgrad": [c_vp, c_long, c_vp, c_long, c_int, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "kair_conv3x3_narrow_x3_ws": [],
    "kair_conv3x3_narrow_fwd_x3": [c_vp, c_long, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_float, c_vp, c_vp, c_int, c_int,
                                   c_int, c_vp],
    "kair_conv3x3_narrow_dgrad_x3": [c_vp, c_long, c_int, c_vp, c_int, c_vp, c_vp, c_long, c_int, c_int, c_int, c_int,
                                     c_vp],
    "kair_conv3x3_narrow_wgrad_x3": [c_vp, c_long, c_int, c_vp, c_long, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_int,
                                     c_int, c_int, c_vp],
    "kair_l1_loss": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_float, c_int, c_int, c_int, c_int, c_vp, c_vp],
    "kair_charbonnier_loss": [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_int, c_float, c_float, c_int, c_int, c_int, c_int,
                              c_vp, c_vp],
    "kair_axpy": [c_vp, c_vp, c_float, c_long, c_vp],
    "kair_axpby": [c_vp, c_vp, c_float, c_float, c_long, c_vp],
    "kair_bn_ws": [c_int],
    "kair_bn_fwd": [c_vp, c_long, c_vp, c_int, c_long, c_long, c_int, c_vp, c_vp, c_vp, c_vp, c_float, c_float, c_int,
                    c_vp, c_vp, c_int, c_float, c_vp, c_vp],
    "kair_bn_bwd": [c_vp, c_long, c_vp, c_int, c_long, c_vp, c_long, c_vp, c_int, c_long, c_long, c_int, c_vp, c_vp, c_vp,
                    c_int, c_float, c_vp, c_vp, c_int, c_vp, c_vp],
    "kair_axpby_rows": [c_vp, c_long, c_vp, c_long, c_long, c_int, c_float, c_float, c_vp],
    "kair_act_grad_cast": [c_vp, c_long, c_vp, c_int, c_long, c_vp, c_int, c_long, c_long, c_int, c_int, c_float, c_float,
                           c_vp],
    "kair_sumpool2x": [c_vp, c_long, c_vp, c_long, c_int, c_int, c_int, c_int, c_int, c_vp],
    "kair_adam_ema": [c_vp, c_vp, c_vp, c_vp, c_vp, c_long, c_vp, c_float, c_float, c_float, c_float, c_float, c_vp],
    "kair_adam_ema_ex": [c_vp, c_vp, c_vp, c_vp, c_vp, c_long, c_vp, c_float, c_float, c_float, c_float, c_float, c_vp,
                         c_vp],
    "kair_range_check": [c_vp, c_vp, c_long, c_vp, c_float, c_vp, c_vp],
    "kair_gate_hold": [c_int, c_vp],
    "kair_gate_release": [],
    "kair_gate_status": [],
    "kair_ktime_begin": [c_int],
    "kair_ktime_count": [],
    "kair_ktime_end": [],
    "kair_ktime_read": [c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_char_p)],
    "kair_usr_fft_rows": [c_vp, c_int, c_int, c_long, c_int, c_int, c_int, c_vp, c_int, c_int, c_int, c_vp],
    "kair_usr_fft_cols": [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_int,
                          c_vp],
    "kair_usr_ifft_rows": [c_vp, c_vp, c_int, c_int, c_int, c_long, c_float, c_int, c_int, c_int, c_vp],
    "kair_usr_seg_sum": [c_vp, c_int, c_int, c_float, c_vp, c_int, c_int, c_vp],
    "kair_usr_chan_sum": [c_vp, c_long, c_int, c_long, c_int, c_vp, c_vp, c_int, c_int, c_vp],
    "kair_usr_upsample_nearest": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_vp],
    "kair_usr_pack_input": [c_vp, c_vp, c_int, c_vp, c_int, c_int, c_int, c_int, c_long, c_vp],
    "kair_usr_pad": [c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "kair_hypanet_fwd": [c_vp, c_float] + [c_vp] * 6 + [c_int, c_int, c_int, c_vp, c_vp],
    "kair_hypanet_bwd": [c_vp, c_float] + [c_vp] * 6 + [c_int, c_int, c_int, c_vp] + [c_vp] * 6 + [c_int, c_vp],
    "kair_synth_sr": [c_vp, c_int, c_int, c_int, c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp,
                      c_vp],
    "kair_synth_dn": [c_vp, c_int, c_int, c_int, c_vp, c_int, c_int, c_float, ctypes.c_ulonglong, ctypes.c_ulonglong,
                      c_vp, c_vp, c_vp],
    "kair_swin_attn_fwd": [c_vp, c_long, c_vp, c_vp, c_float, c_int, c_vp, c_long, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                           c_float, c_vp, c_long, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_long, c_long, c_int,
                           c_int, c_int, c_int, c_int, c_vp],
    "kair_swin_mlp_fwd": [c_vp, c_long, c_vp, c_vp, c_float, c_int, c_vp, c_long, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                          c_long, c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_long, c_long, c_int, c_int, c_int, c_vp],
    "kair_debug_attn_stamps": [c_vp, c_int],
    "kair_debug_fused_stamps": [c_vp, c_int],
    "kair_debug_x3_stamps": [c_vp, c_int],
    "kair_swin_mlp_bwd_ws": [],
    "kair_swin_mlp_bwd": [c_vp, c_long, c_vp, c_long, c_vp, c_vp, c_vp, c_long, c_vp, c_long, c_vp, c_vp, c_vp, c_int,
                          c_vp, c_long, c_vp, c_long, c_vp, c_int, c_int, c_int, c_int, c_vp, c_vp, c_int, c_vp, c_long,
                          c_int, c_int, c_vp],
    "kair_rowgemm_store": [c_vp, c_long, c_long, c_int, c_vp, c_int, c_vp, c_long, c_vp],
    "kair_rowgemm_gate": [c_vp, c_long, c_long, c_int, c_vp, c_int, c_vp, c_long, c_vp, c_long, c_vp],
    "kair_rowgemm_ln_blocks": [c_long, c_int],
    "kair_rowgemm_lnbwd": [c_vp, c_long, c_long, c_int, c_vp, c_vp, c_long, c_vp, c_vp, c_vp, c_int, c_vp, c_long,
                           c_int, c_int, c_int, c_int, ctypes.POINTER(CopyDesc), c_vp, c_vp],
    "kair_window_attn_fwd_x3": [c_vp, c_vp, c_vp, c_vp, c_vp, c_long, c_vp, c_long, c_int, c_int, c_float, c_int, c_int,
                                c_int, c_int, c_int, c_int, c_vp],
    "kair_window_attn_bwd_x3": [c_vp, c_vp, c_vp, c_vp, c_long, c_vp, c_vp, c_long, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                                c_vp, c_long, c_int, c_int, c_float, c_int, c_int, c_int, c_int, c_int, c_vp],
    "kair_last_error": [],
    "kair_device_arch": [ctypes.c_char_p, c_int],
}
_RESTYPE = {"kair_gemm_nt_x3_lnbwd_parts": c_long, "kair_layernorm_bwd_blocks": c_long, "kair_rowgemm_ln_blocks": c_long, "kair_window_attn_bwd_groups": c_long, "kair_wgrad_grouped_ws": c_long, "kair_swin_mlp_bwd_ws": c_long, "kair_bn_ws": c_long, "kair_last_error": ctypes.c_char_p, "kair_window_attn_bwd_ws": c_long, "kair_pack_table_bytes": c_long,
            "kair_pack_table_build": c_long, "kair_conv3x3_narrow_wgrad_ws": c_long,
            "kair_conv3x3_narrow_dgrad_ws": c_long, "kair_conv3x3_narrow_x3_ws": c_long}

_lib = None


def lib():
    """Load libkair_hip.so once.  Raises RuntimeError (never falls back) when it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"kair_amd: HIP kernel library not built ({LIB_PATH}); run `python -m kair_amd.build`")
        L = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            if (name.startswith("kair_debug_") or os.environ.get("KAIR_LIB") == "base") and not hasattr(L, name):
                continue   # perf-investigation entry points, and an A/B baseline build's older symbol set
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, c_int)
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(rc, what=""):
    if rc != 0:
        msg = lib().kair_last_error().decode(errors="replace")
        raise RuntimeError(f"kair_hip {what} failed ({rc}): {msg}")


def ptr(t):
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream


def dtype_code(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float16:
        return F16
    raise TypeError(f"unsupported dtype {t.dtype}")


def require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("kair_amd runs on the HIP device only (got a CPU tensor); there is no CPU fallback")


# ------------------------------------------------------------------------------------------
# descriptor builders
# ------------------------------------------------------------------------------------------
def rows(t, ld=None, win=None, rowscale=None, rows_per_scale=1, ones_col=-1, ones_in_data=False, w_split=False):
    """Row-major operand; win = (H, W, ws, shift) applies the Swin window->token row map.
    w_split: packed hi/lo bf16 weight rows (pack kind 9; gemm_nt B operand only)."""
    o = Operand()
    o._keep = (t, rowscale)  # keep the tensors alive until the launch has been issued
    o.ptr = ptr(t)
    o.dtype = dtype_code(t)
    o.mode = LD_ROWS
    o.ld = ld if ld is not None else t.shape[-1]
    if win:
        o.win_H, o.win_W, o.win_ws, o.win_shift = win
    o.rowscale = ptr(rowscale)
    o.rows_per_scale = rows_per_scale
    o.ones_col = ones_col
    o.ones_in_data = int(ones_in_data)
    o.w_split = int(w_split)
    return o


def asplit(op, lo=None, pair=False):
    """Mark a kair_gemm_nt A operand as a hi/lo activation pair: fp32 A forms lo in the kernel, a bf16 A
    (the hi plane) reads lo from `lo` (its producer's epilogue out_lo).  pair=True: the bf16 image's
    channels already are the [hi | lo] halves (weights packed tied over them; a_split 2)."""
    op.a_split = 2 if pair else 1
    if lo is not None:
        op.lo_ptr = ptr(lo)
        op._keep = (op._keep, lo)
    return op


def im2col(t, H, W, C, flip=False, ones_col=-1, ld=None, up=1, ones_in_data=False):
    """3x3 / pad 1 im2col view of an NHWC map: H x W is the CONV grid, ld the pixel stride
    (default C), up=2 reads the source (H/2 x W/2) through a nearest x2 upsample.  ones_in_data: the
    map already holds 1.0 in channel ones_col % C of every pixel (read through the center tap,
    ones_col = 4 * C + c, by the tap-per-tile weight-gradient ring)."""
    o = Operand()
    o._keep = t
    o.ptr = ptr(t)
    o.dtype = dtype_code(t)
    o.mode = LD_IM2COL3
    o.ld = ld if ld is not None else C
    o.im_H, o.im_W, o.im_C, o.im_flip = H, W, C, int(flip)
    o.im_up = up
    o.ones_col = ones_col
    o.ones_in_data = int(ones_in_data)
    o.rows_per_scale = 1
    return o


def s2d(t, H, W, C, ld=None):
    """2x2 / stride-2 space-to-depth view of an NHWC map: H x W is the OUTPUT grid (the source is
    2H x 2W), column k = (i*2 + j) * C + c reads pixel (2y+i, 2x+j), channel c."""
    o = Operand()
    o._keep = t
    o.ptr = ptr(t)
    o.dtype = dtype_code(t)
    o.mode = LD_S2D
    o.ld = ld if ld is not None else C
    o.im_H, o.im_W, o.im_C = H, W, C
    o.ones_col = -1
    o.rows_per_scale = 1
    return o


def qkvblk(t, nh, hdp=32, tok=64, rowscale=None, rows_per_scale=1):
    o = Operand()
    o._keep = (t, rowscale)
    o.ptr = ptr(t)
    o.dtype = dtype_code(t)
    o.mode = LD_QKVBLK
    o.qkv_nh, o.qkv_hdp, o.qkv_tok = nh, hdp, tok
    o.rowscale = ptr(rowscale)
    o.rows_per_scale = rows_per_scale
    o.ones_col = -1
    return o


def epilogue(out, mode=OUT_ROWS, ldo=None, win=None, bias=None, act=ACT_NONE, slope=0.0, pre=None, ldp=None,
             resid=None, ldr=None, rowscale=None, rows_per_scale=1, gate=None, ldg=None, gate_kind=0,
             ps=None, qkv=None, img=None, ones_col=-1, resid2=None, ldr2=None, pre_grad=False, acopy=None, out_lo=None):
    """pre_grad: `pre` receives act'(x) instead of x (GELU; read back with gate_kind=4).  acopy = (bf16
    tensor, ones_col): the 3x3 halo conv also writes its A image there (ones_col >= 0: that channel 1.0).
    out_lo: bf16 lo plane bf16(v - bf16(v)) beside a bf16 ROWS / PSHUF_SPM out (same layout)."""
    e = Epilogue()
    e.pre_kind = int(bool(pre_grad))
    e._keep = (out, bias, pre, resid, rowscale, gate, img, resid2, acopy, out_lo)
    e.out_lo = ptr(out_lo)
    if acopy is not None:
        e.a_copy, e.ld_acopy, e.acopy_ones_col_p1 = ptr(acopy[0]), acopy[0].shape[-1], acopy[1] + 1
    if resid2 is not None:
        e.resid2, e.ldr2 = ptr(resid2), (ldr2 if ldr2 is not None else resid2.shape[-1])
    e.out = ptr(out)
    e.out_dtype = dtype_code(out)
    e.out_mode = mode
    e.out_ones_col_p1 = ones_col + 1
    e.ldo = ldo if ldo is not None else out.shape[-1]
    if win:
        e.win_H, e.win_W, e.win_ws, e.win_shift = win
    e.bias = ptr(bias)
    e.act, e.slope = act, slope
    if pre is not None:
        e.out_pre, e.pre_dtype, e.ldp = ptr(pre), dtype_code(pre), (ldp if ldp is not None else pre.shape[-1])
    if resid is not None:
        e.resid, e.ldr = ptr(resid), (ldr if ldr is not None else resid.shape[-1])
    e.rowscale, e.rows_per_scale = ptr(rowscale), rows_per_scale
    if gate is not None:
        e.gate, e.gate_dtype, e.ldg, e.gate_kind = ptr(gate), dtype_code(gate), (ldg if ldg is not None else gate.shape[-1]), gate_kind
    if ps:
        e.ps_r, e.ps_H, e.ps_W = ps
    if qkv:
        e.qkv_nh, e.qkv_hdp, e.qkv_tok = qkv
    if img:
        mean, rng, C, H, W = img
        e.img_mean, e.img_range, e.img_C, e.img_H, e.img_W = ptr(mean), rng, C, H, W
    return e


def wmap(kind, N, K, n_groups=(1, None, None), k_groups=(1, None, None), n_perm=0):
    """n_groups = (G, real, padded) for the out dim; k_groups likewise for the in dim; n_perm = r*r
    stores the out dim sub-pixel-major (PixelShuffle SPM layouts)."""
    m = WMap()
    m.kind, m.N, m.K = kind, N, K
    m.n_perm = n_perm
    nG, nr, npd = n_groups
    kG, kr, kpd = k_groups
    m.nG, m.nGr, m.nGp = nG, nr or N // nG, npd or nr or N // nG
    m.kG, m.kGr, m.kGp = kG, kr or (K // kG if K else 1), kpd or kr or (K // kG if K else 1)
    return m


# ------------------------------------------------------------------------------------------
# thin call wrappers (raise on error)
# ------------------------------------------------------------------------------------------
def gemm_nt(A, B, E, M, N, K, compute):
    check(lib().kair_gemm_nt(ctypes.byref(A), ctypes.byref(B), ctypes.byref(E), M, N, K, compute, stream_ptr()), "gemm_nt")


def conv_halo_geometry(H, W, C, M, N):
    """True when a bf16 3x3 conv of this geometry runs on the halo path (can write epilogue acopy)."""
    return bool(lib().kair_conv3x3_halo_geometry(H, W, C, M, N))


def wgrad_splits(M, N, K):
    return lib().kair_wgrad_splits(M, N, K)


def wgrad_tiles(N, K):
    """(N, K) tiles of one kair_gemm_tn split (the launch has tiles x splits workgroups): the 192 x 192
    ring tile where it applies, a 192-wide N tile for N in (128, 192], else 128 x 128 (gemm.hip)."""
    if N <= 576 and K <= 576 and N % 8 == 0 and K % 8 == 0 and N > 64 and K > 64:
        return -(-N // 192) * -(-K // 192)
    if N <= 576 and N % 8 == 0 and N > 64 and K == 9 * 192:   # conv weight gradient, one tap per tile
        return -(-N // 192) * 9
    if N <= 64 and K <= 64:
        return 1
    if 128 < N <= 192 and K > 128:
        return -(-K // 128)
    return -(-N // 128) * -(-K // 128)


def gemm_tn(A, B, ws, splits, M, N, K, compute):
    check(lib().kair_gemm_tn(ctypes.byref(A), ctypes.byref(B), ptr(ws), splits, M, N, K, compute, stream_ptr()), "gemm_tn")


def wgrad_grouped_ws(shapes, M, x3=False):
    """Workspace floats of a kair_wgrad_grouped launch over linears of packed (N, K) shapes (x3: fp16-pair jobs,
    the fp32x3 TN ring's 192 x 192 tiles)."""
    arr = (WgradJob * len(shapes))()
    for i, (N, K) in enumerate(shapes):
        arr[i].N, arr[i].K = N, K
        arr[i].A.dtype = F16 if x3 else BF16
    return lib().kair_wgrad_grouped_ws(arr, len(shapes), M)


class WgradGroup:
    """The weight gradients of several linear layers (kair_wgrad_grouped): one TN launch + one
    finalize launch.  jobs: (A operand, B operand, N, K, wmap, grad, bias_grad or None, ones_col)."""

    WG_MAX = 24

    def __init__(self, jobs, M):
        if not 0 < len(jobs) <= self.WG_MAX:
            raise ValueError(f"kair_wgrad_grouped: 1..{self.WG_MAX} jobs (got {len(jobs)})")
        arr = (WgradJob * len(jobs))()
        for i, (A, B, N, K, m, grad, bias, oc) in enumerate(jobs):
            arr[i].A, arr[i].B, arr[i].N, arr[i].K, arr[i].map = A, B, N, K, m
            arr[i].grad, arr[i].bias_grad, arr[i].ones_col = ptr(grad), ptr(bias), oc
        self._keep = jobs
        self.arr, self.n, self.M = arr, len(jobs), M
        self.ws_floats = lib().kair_wgrad_grouped_ws(arr, self.n, M)

    def run(self, ws, max_ctas=0):
        """max_ctas > 0: at most that many workgroups (kair_wgrad_grouped_ex: fewer row splits); < 0:
        -max_ctas times the default splits (the workspace scales with it)."""
        if ws.numel() < self.ws_floats * max(1, -max_ctas):
            raise ValueError("kair_wgrad_grouped: workspace too small")
        check(lib().kair_wgrad_grouped_ex(self.arr, self.n, self.M, ptr(ws), int(max_ctas), stream_ptr()),
              "wgrad_grouped")


def pack_weight(src, dst, m):
    check(lib().kair_pack_weight(ptr(src), ptr(dst), dtype_code(dst), ctypes.byref(m), stream_ptr()), "pack_weight")


class PackTable:
    """Every (src, dst, map) re-pack of a network, launched as ONE kernel (kair_pack_weights)."""

    def __init__(self, jobs):
        n = len(jobs)
        arr = (PackJob * n)()
        for i, (src, dst, m) in enumerate(jobs):
            arr[i].src, arr[i].dst, arr[i].dst_dtype, arr[i].map = ptr(src), ptr(dst), dtype_code(dst), m
        self._keep = [(s, d) for s, d, _ in jobs]
        self.n = n
        self.table = torch.empty(lib().kair_pack_table_bytes(n), dtype=torch.uint8, device=jobs[0][1].device)
        nb = lib().kair_pack_table_build(arr, n, ptr(self.table))
        if nb <= 0:
            check(int(nb) or -1, "pack_table_build")
        self.nblocks = nb

    def run(self):
        check(lib().kair_pack_weights(ptr(self.table), self.n, self.nblocks, stream_ptr()), "pack_weights")


def wgrad_finalize(partial, splits, m, grad, bias_grad=None, ones_col=-1, accumulate=False):
    check(lib().kair_wgrad_finalize(ptr(partial), splits, ctypes.byref(m), ptr(grad), ptr(bias_grad), ones_col,
                                    int(accumulate), stream_ptr()), "wgrad_finalize")


def colsum(G, M, Np, m, bias_grad, ws, accumulate=False):
    check(lib().kair_colsum(ctypes.byref(G), M, Np, ctypes.byref(m), ptr(bias_grad), ptr(ws), int(accumulate),
                            stream_ptr()), "colsum")


def layernorm_fwd(x, ldx, y, ldy, gamma, beta, mean, rstd, M, C, eps=1e-5, win=(0, 0, 0, 0), one_col=-1):
    check(lib().kair_layernorm_fwd(ptr(x), ldx, ptr(y), dtype_code(y), ldy, ptr(gamma), ptr(beta), ptr(mean), ptr(rstd),
                                   M, C, eps, *win, one_col, stream_ptr()), "layernorm_fwd")


def layernorm_fwd_x3(x, ldx, y, ldy, gamma, beta, mean, rstd, M, C, eps=1e-5, win=(0, 0, 0, 0), one_col=-1, x3_exp=0):
    """LayerNorm forward into an fp16 pair y [2, M, ldy] (hi, lo planes) of y 2^x3_exp (the fp32x3 GEMM operand)."""
    check(lib().kair_layernorm_fwd_x3(ptr(x), ldx, ptr(y[0]), ptr(y[1]), ldy, ptr(gamma), ptr(beta), ptr(mean), ptr(rstd),
                                      M, C, eps, *win, one_col, int(x3_exp), stream_ptr()), "layernorm_fwd_x3")


def layernorm_bwd(x, ldx, dy, ldy, gamma, mean, rstd, dx, ld_dx, dx_acc, dgamma, dbeta, dparam_acc, ws, M, C,
                  win=(0, 0, 0, 0), copy=None):
    check(lib().kair_layernorm_bwd(ptr(x), ldx, ptr(dy), dtype_code(dy), ldy, ptr(gamma), ptr(mean), ptr(rstd), ptr(dx),
                                   ld_dx, int(dx_acc), ptr(dgamma), ptr(dbeta), int(dparam_acc), ptr(ws), M, C, *win,
                                   ctypes.byref(copy) if copy is not None else None, stream_ptr()), "layernorm_bwd")


def gemm_nt_lnbwd(A, B, M, N, K, x, ldx, gamma, mean, rstd, C, D, ldd, part, win=(0, 0, 0, 0), copy=None):
    """fp32x3: dxn = A B^T fused with the LayerNorm backward (kair_gemm_nt_x3_lnbwd): D[t] += LN'(dxn), the optional
    fp16-pair copy of D, dgamma / dbeta partial rows in part (gemm_nt_lnbwd_parts(M, N) rows of 2 C)."""
    check(lib().kair_gemm_nt_x3_lnbwd(ctypes.byref(A), ctypes.byref(B), M, N, K, *win, ptr(x), ldx, ptr(gamma), ptr(mean),
                                      ptr(rstd), C, ptr(D), ldd, ptr(part),
                                      ctypes.byref(copy) if copy is not None else None, stream_ptr()), "gemm_nt_x3_lnbwd")


def gemm_nt_lnbwd_parts(M, N):
    return lib().kair_gemm_nt_x3_lnbwd_parts(M, N)


def row_copy(src, ld_src, M, C, copy):
    check(lib().kair_row_copy(ptr(src), ld_src, M, C, ctypes.byref(copy), stream_ptr()), "row_copy")


def window_attn_fwd(qkv, table, O, ldo, lse, nWin, nh, hd, scale, H, W, shift, ones_col=-1, mask=None, head_pad=32):
    """head_pad: 32, or 16 (bf16, head_dim <= 16): the per-head width of the qkv / O layouts."""
    mnw = mask.shape[0] if mask is not None else 0
    check(lib().kair_window_attn_fwd_ex(ptr(qkv), dtype_code(qkv), ptr(table), ptr(O), ldo, ptr(lse), nWin, nh, hd, scale,
                                        H, W, shift, ones_col, ptr(mask), mnw, head_pad, stream_ptr()), "window_attn_fwd")


GROUP_MAX = 32   # jobs per kair_ln_param_reduce_grouped / kair_attn_dtable_grouped launch (LNP_MAX, DTAB_MAX)


def layernorm_bwd_blocks(M):
    return lib().kair_layernorm_bwd_blocks(M)


def ln_param_reduce_grouped(jobs):
    """jobs: (partials left by layernorm_bwd(dgamma=None, dbeta=None), M, C, dgamma, dbeta, accumulate[, nb]);
    nb (the partial-row count) defaults to layernorm_bwd's for M (rowgemm_lnbwd: rowgemm_ln_blocks)."""
    arr = (LnParamJob * len(jobs))()
    for i, job in enumerate(jobs):
        part, M, C, dg, db, acc = job[:6]
        nb = job[6] if len(job) > 6 else layernorm_bwd_blocks(M)
        arr[i].part, arr[i].nb, arr[i].C = ptr(part), nb, C
        arr[i].dgamma, arr[i].dbeta, arr[i].accumulate = ptr(dg), ptr(db), int(acc)
    check(lib().kair_ln_param_reduce_grouped(arr, len(jobs), stream_ptr()), "ln_param_reduce_grouped")


def attn_dtable_grouped(jobs):
    """jobs: (ws left by window_attn_bwd(dtable=None), nWin, nh, dtype code, dtable, accumulate)."""
    arr = (DtabJob * len(jobs))()
    for i, (ws, nWin, nh, dt, dtable, acc) in enumerate(jobs):
        arr[i].ws, arr[i].nWin, arr[i].nh, arr[i].dtype = ptr(ws), nWin, nh, dt
        arr[i].dtable, arr[i].accumulate = ptr(dtable), int(acc)
    check(lib().kair_attn_dtable_grouped(arr, len(jobs), stream_ptr()), "attn_dtable_grouped")


def window_attn_bwd_ws(nWin, nh):
    return lib().kair_window_attn_bwd_ws(nWin, nh)


def window_attn_bwd(qkv, O, ldo, dO, lddo, table, lse, dqkv, dtable, dtable_acc, ws, nWin, nh, hd, scale, H, W, shift,
                    mask=None, dqkv_rows=False, head_pad=32):
    """dqkv_rows: dqkv as token rows [nWin*64, 3*nh*head_pad] (bf16) instead of head-blocked."""
    mnw = mask.shape[0] if mask is not None else 0
    check(lib().kair_window_attn_bwd_ex(ptr(qkv), ptr(O), ldo, ptr(dO), lddo, dtype_code(qkv), ptr(table), ptr(lse),
                                        ptr(dqkv), int(dqkv_rows), ptr(dtable), int(dtable_acc), ptr(ws), nWin, nh, hd,
                                        scale, H, W, shift, ptr(mask), mnw, head_pad, stream_ptr()), "window_attn_bwd")


def _planes(t):
    """(hi, lo) pointers of an x3 tensor: an fp16 pair [2, ...] or an fp32 tensor in natural units (lo NULL)."""
    return (ptr(t), None) if t.dtype == torch.float32 else (ptr(t[0]), ptr(t[1]))


def window_attn_fwd_x3(qkv, table, O, ldo, lse, nWin, nh, hd, scale, H, W, shift, ones_col=-1, e_in=0, e_out=0):
    """Split-fp16 window attention forward: qkv is [2, ...] fp16 (hi plane, lo plane) of x 2^e_in; O the same
    with e_out, or an fp32 tensor (natural units)."""
    o, ol = _planes(O)
    check(lib().kair_window_attn_fwd_x3(ptr(qkv[0]), ptr(qkv[1]), ptr(table), o, ol, ldo, ptr(lse), nWin,
                                        nh, hd, scale, H, W, shift, ones_col, e_in, e_out, stream_ptr()),
          "window_attn_fwd_x3")


def window_attn_bwd_x3(qkv, O, ldo, dO, lddo, table, lse, dqkv, dtable, dtable_acc, ws, nWin, nh, hd, scale, H, W, shift,
                       e_act=0, e_grad=0):
    """Split-fp16 window attention backward: qkv, dO are [2, ...] fp16 planes; O and dqkv (token rows [M][3 nh 32])
    fp16 pairs or fp32 (natural units); q/k/v and O pairs carry e_act, dO and a dqkv pair e_grad."""
    o, ol = _planes(O)
    dq, dql = _planes(dqkv)
    check(lib().kair_window_attn_bwd_x3(ptr(qkv[0]), ptr(qkv[1]), o, ol, ldo, ptr(dO[0]), ptr(dO[1]), lddo,
                                        ptr(table), ptr(lse), dq, dql, ptr(dtable), int(dtable_acc),
                                        ptr(ws), nWin, nh, hd, scale, H, W, shift, e_act, e_grad, stream_ptr()),
          "window_attn_bwd_x3")


def with_lo(op, lo):
    """Attach the lo plane of a 16-bit operand pair (split-fp16 GEMMs of kair_gemm_nt / kair_gemm_tn compute X3;
    the bf16 engine's a_split)."""
    op.lo_ptr = ptr(lo)
    op._keep = (op._keep, lo)
    return op


def conv3x3_narrow_fwd(x, ldx, lo_off, w, bias, NR, mean, img_range, resid, out, B, H, W):
    """conv_last forward: 64-channel bf16 rows (hi, + lo at lo_off) -> NCHW image (csrc/tail.hip)."""
    check(lib().kair_conv3x3_narrow_fwd(ptr(x), ldx, lo_off, ptr(w), ptr(bias), NR, ptr(mean), img_range, ptr(resid),
                                        ptr(out), B, H, W, stream_ptr()), "conv3x3_narrow_fwd")


def conv3x3_wr_tile(split, B, H, W, C, N):
    """Tile (pixels) of kair_conv3x3_wr for this shape, 0 when unsupported."""
    return lib().kair_conv3x3_wr_tile(int(bool(split)), B, H, W, C, N)


def conv3x3_wr(x, ldx, flip, w, bias, resid, out, B, H, W, C, N, ldr=None, ldo=None, acopy=None, ldac=None, acones=-1,
               n_blocks=None, split=None, out_lo=None, ps_r=0, act=ACT_NONE, slope=0.0, gate=None, ldg=None):
    """3x3 conv with register-streamed weights (csrc/conv_wr.hip, kair_conv3x3_wr_ex).  split (default: x
    fp32): two halos -- split activations of an fp32 image, or a bf16 [hi | lo] pair image of C channels
    per half -- with w = pack kind 15; else one bf16 product with w = pack kind 16 (flip = 1: input
    gradient).  ps_r > 0: PixelShuffle sub-pixel-major store (+ out_lo: the lo plane of a bf16 pair); ps_r < 0:
    PixelUnshuffle(-ps_r) store; gate: LeakyReLU'(gate) (slope) on the rows."""
    if split is None:
        split = x.dtype == torch.float32
    if n_blocks is None:
        n_blocks = 16 if N > 192 else 12 if N > 64 else 4
    check(lib().kair_conv3x3_wr_ex(ptr(x), dtype_code(x), ldx, int(bool(split)), int(flip), ptr(w), n_blocks, ptr(bias),
                                   ptr(resid), ldr if ldr is not None else (resid.shape[-1] if resid is not None else 0),
                                   ptr(out), dtype_code(out), ldo if ldo is not None else out.shape[-1], ptr(out_lo), ps_r,
                                   act, slope, ptr(gate), ldg if ldg is not None else (gate.shape[-1] if gate is not None else 0),
                                   ptr(acopy), ldac if ldac is not None else (acopy.shape[-1] if acopy is not None else 0),
                                   acones, B, H, W, C, N, stream_ptr()), "conv3x3_wr")


def conv3x3_narrow_dgrad_ws():
    return lib().kair_conv3x3_narrow_dgrad_ws()


def conv3x3_narrow_dgrad(dE, lde, w, NR, ws, out, ldo, ps_r, B, H, W):
    check(lib().kair_conv3x3_narrow_dgrad(ptr(dE), lde, ptr(w), NR, ptr(ws), ptr(out), dtype_code(out), ldo, ps_r, B, H, W,
                                          stream_ptr()), "conv3x3_narrow_dgrad")


def conv3x3_narrow_wgrad_ws(NR):
    return lib().kair_conv3x3_narrow_wgrad_ws(NR)


def conv3x3_narrow_wgrad(dE, lde, x, ldx, NR, ws, grad_w, grad_b, B, H, W, accumulate=False):
    check(lib().kair_conv3x3_narrow_wgrad(ptr(dE), lde, ptr(x), ldx, NR, ptr(ws), ptr(grad_w), ptr(grad_b),
                                          int(accumulate), B, H, W, stream_ptr()), "conv3x3_narrow_wgrad")


def conv3x3_narrow_x3_ws():
    return lib().kair_conv3x3_narrow_x3_ws()


def conv3x3_narrow_fwd_x3(x, ldx, ex, w, bias, NR, ws, mean, img_range, resid, out, B, H, W):
    """conv_last forward at the fp32 engine's arithmetic: 64-channel fp32 rows -> NCHW image (csrc/tail.hip)."""
    check(lib().kair_conv3x3_narrow_fwd_x3(ptr(x), ldx, ex, ptr(w), ptr(bias), NR, ptr(ws), ptr(mean), img_range, ptr(resid),
                                           ptr(out), B, H, W, stream_ptr()), "conv3x3_narrow_fwd_x3")


def conv3x3_narrow_dgrad_x3(dE, lde, eg, w, NR, ws, out, ldo, ps_r, B, H, W):
    check(lib().kair_conv3x3_narrow_dgrad_x3(ptr(dE), lde, eg, ptr(w), NR, ptr(ws), ptr(out), ldo, ps_r, B, H, W,
                                             stream_ptr()), "conv3x3_narrow_dgrad_x3")


def conv3x3_narrow_wgrad_x3(dE, lde, eg, x, ldx, ex, NR, ws, grad_w, grad_b, B, H, W, accumulate=False):
    check(lib().kair_conv3x3_narrow_wgrad_x3(ptr(dE), lde, eg, ptr(x), ldx, ex, NR, ptr(ws), ptr(grad_w), ptr(grad_b),
                                             int(accumulate), B, H, W, stream_ptr()), "conv3x3_narrow_wgrad_x3")


def image_to_nhwc_hilo(img, out, ldc, mean, img_range, B, C, H, W):
    """bf16 hi/lo pair of the normalised image: hi in channels [0, C), lo in [ldc/2, ldc/2 + C)."""
    check(lib().kair_image_to_nhwc_hilo(ptr(img), ptr(out), ldc, ptr(mean), img_range, B, C, H, W, stream_ptr()),
          "image_to_nhwc_hilo")


def image_to_nhwc(img, out, ldc, mean, img_range, B, C, H, W):
    check(lib().kair_image_to_nhwc(ptr(img), ptr(out), dtype_code(out), ldc, ptr(mean), img_range, B, C, H, W,
                                   stream_ptr()), "image_to_nhwc")


def l1_loss(E, H, loss_out, dE, ldc, weight, B, C, Hh, Ww, ws, ps_r=1, charb_eps=None):
    """L1 (mean) loss + its gradient; charb_eps set: the Charbonnier loss sqrt(d^2 + eps) instead."""
    if charb_eps is not None:
        check(lib().kair_charbonnier_loss(ptr(E), ptr(H), ptr(loss_out), ptr(dE), dtype_code(dE), ldc, ps_r, weight,
                                          float(charb_eps), B, C, Hh, Ww, ptr(ws), stream_ptr()), "charbonnier_loss")
        return
    check(lib().kair_l1_loss(ptr(E), ptr(H), ptr(loss_out), ptr(dE), dtype_code(dE), ldc, ps_r, weight, B, C, Hh, Ww,
                             ptr(ws), stream_ptr()), "l1_loss")


def axpy(y, x, a, n=None):
    check(lib().kair_axpy(ptr(y), ptr(x), a, n if n is not None else y.numel(), stream_ptr()), "axpy")


def adam_ema(p, g, m, v, ema, n, lr_t, beta1, beta2, eps, wd, decay, skip=None):
    """skip: an int32 device flag (kair_range_check): nonzero drops the step (kair_adam_ema_ex)."""
    if skip is not None:
        check(lib().kair_adam_ema_ex(ptr(p), ptr(g), ptr(m), ptr(v), ptr(ema), n, ptr(lr_t), beta1, beta2, eps, wd, decay,
                                     ptr(skip), stream_ptr()), "adam_ema_ex")
        return
    check(lib().kair_adam_ema(ptr(p), ptr(g), ptr(m), ptr(v), ptr(ema), n, ptr(lr_t), beta1, beta2, eps, wd, decay,
                              stream_ptr()), "adam_ema")


def ktime_begin(n=4096):
    """Open a kernel timing window of n slots (kair_ktime_begin): every later libkair launch into a non-capturing
    stream is timed by its dispatch packet's start / end, as rocprofv3 --kernel-trace times it."""
    check(lib().kair_ktime_begin(n), "ktime_begin")


def ktime_count():
    return lib().kair_ktime_count()


def ktime_end():
    return lib().kair_ktime_end()


def gate_hold(timeout_ms=5000):
    """Hold the current stream behind one waiting wave until gate_release() (or timeout_ms): an eager pass queued
    behind it then runs back to back (kair_gate_hold)."""
    check(lib().kair_gate_hold(timeout_ms, stream_ptr()), "gate_hold")


def gate_release():
    check(lib().kair_gate_release(), "gate_release")


def gate_status():
    """0 pending, 1 released by the host, 2 the wave's time limit passed first."""
    return lib().kair_gate_status()


def ktime_read(i):
    """(duration ms, kernel symbol) of slot i of the last window; waits for that launch."""
    ms, name = ctypes.c_float(), ctypes.c_char_p()
    check(lib().kair_ktime_read(i, ctypes.byref(ms), ctypes.byref(name)), "ktime_read")
    return ms.value, (name.value or b"").decode(errors="replace")


def range_check(g, p, loss, p_limit, flag):
    """fp32x3 range guard: flag[0] = 1 (non-finite gradient) | 2 (non-finite loss) | 4 (|p| >= p_limit)."""
    check(lib().kair_range_check(ptr(g), ptr(p), g.numel(), ptr(loss), float(p_limit), ptr(flag), stream_ptr()),
          "range_check")


def axpby(y, x, a, b, n=None):
    """y = a * x + b * y (fp32)."""
    check(lib().kair_axpby(ptr(y), ptr(x), a, b, n if n is not None else y.numel(), stream_ptr()), "axpby")


def act_grad_cast(G, ldg, X, ldx, out, ldo, M, C, kind, slope=0.0, scale=1.0):
    """out = scale * G * act'(X) (act' read from the post-activation X; kind 0 none, 1 relu, 2 leaky)."""
    check(lib().kair_act_grad_cast(ptr(G), ldg, ptr(X), dtype_code(X) if X is not None else F32, ldx, ptr(out),
                                   dtype_code(out), ldo, M, C, kind, slope, scale, stream_ptr()), "act_grad_cast")


def sumpool2x(src, lds, dst, ldd, B, H, W, C, accumulate=False):
    """dst (+)= 2x2 sum-pool of src (the adjoint of nearest x2 upsampling)."""
    check(lib().kair_sumpool2x(ptr(src), lds, ptr(dst), ldd, B, H, W, C, int(accumulate), stream_ptr()), "sumpool2x")


def axpby_rows(y, ldy, x, ldx, M, C, a, b):
    """y[:, :C] = a * x[:, :C] + b * y[:, :C] over strided fp32 rows."""
    check(lib().kair_axpby_rows(ptr(y), ldy, ptr(x), ldx, M, C, a, b, stream_ptr()), "axpby_rows")


# ------------------------------------------------------------------------------------------
# USRNet (network_usrnet_v1.py): complex planes are fp32 tensors holding float2 [planes][W][H]
# ------------------------------------------------------------------------------------------
def usr_fft_rows(src, mode, C, ld, kh, kw, sf, T, planes, Hh, Ww):
    check(lib().kair_usr_fft_rows(ptr(src), mode, C, ld, kh, kw, sf, ptr(T), planes, Hh, Ww, stream_ptr()), "usr_fft_rows")


def usr_fft_cols(mode, T, Tout, FB, FBFy, FR, invW, alpha, alpha_stride, part, planes, C, Hh, Ww, sf):
    check(lib().kair_usr_fft_cols(mode, ptr(T), ptr(Tout), ptr(FB), ptr(FBFy), ptr(FR), ptr(invW), ptr(alpha),
                                  alpha_stride, ptr(part), planes, C, Hh, Ww, sf, stream_ptr()), "usr_fft_cols")


def usr_ifft_rows(T, dst, nhwc, C, ld, scale, planes, Hh, Ww):
    check(lib().kair_usr_ifft_rows(ptr(T), ptr(dst), int(nhwc), dtype_code(dst), C, ld, scale, planes, Hh, Ww,
                                   stream_ptr()), "usr_ifft_rows")


def usr_seg_sum(ws, seglen, nseg, scale, out, ostride, accumulate=False):
    check(lib().kair_usr_seg_sum(ptr(ws), seglen, nseg, scale, ptr(out), ostride, int(accumulate), stream_ptr()),
          "usr_seg_sum")


def usr_chan_sum(x, ld, c, HW, B, ws, out, ostride, accumulate=False):
    check(lib().kair_usr_chan_sum(ptr(x), ld, c, HW, B, ptr(ws), ptr(out), ostride, int(accumulate), stream_ptr()),
          "usr_chan_sum")


def usr_upsample_nearest(L, out, planes, h, w, sf):
    check(lib().kair_usr_upsample_nearest(ptr(L), ptr(out), planes, h, w, sf, stream_ptr()), "usr_upsample_nearest")


def usr_pad(src, dst, mode, ldc, nb, H, W, Hp, Wp):
    """ResUNet replicate pad / crop and adjoints (kair_usr_pad); dst dtype = src dtype."""
    if src.dtype != dst.dtype:
        raise ValueError("usr_pad: src and dst dtypes differ")
    check(lib().kair_usr_pad(ptr(src), ptr(dst), dtype_code(dst), mode, ldc, nb, H, W, Hp, Wp, stream_ptr()), "usr_pad")


def usr_pack_input(x, beta, beta_stride, out, ld, B, C, HW):
    check(lib().kair_usr_pack_input(ptr(x), ptr(beta), beta_stride, ptr(out), dtype_code(out), ld, B, C, HW,
                                    stream_ptr()), "usr_pack_input")


def hypanet_fwd(sigma, sf, W1, b1, W2, b2, W3, b3, hc, no, B, ab):
    check(lib().kair_hypanet_fwd(ptr(sigma), sf, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(W3), ptr(b3), hc, no, B, ptr(ab),
                                 stream_ptr()), "hypanet_fwd")


def hypanet_bwd(sigma, sf, W1, b1, W2, b2, W3, b3, hc, no, B, gab, gW1, gb1, gW2, gb2, gW3, gb3, accumulate=False):
    check(lib().kair_hypanet_bwd(ptr(sigma), sf, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(W3), ptr(b3), hc, no, B, ptr(gab),
                                 ptr(gW1), ptr(gb1), ptr(gW2), ptr(gb2), ptr(gW3), ptr(gb3), int(accumulate),
                                 stream_ptr()), "hypanet_bwd")


def bn_ws(C):
    return lib().kair_bn_ws(C)


def bn_fwd(z, ldz, out, ldo, M, C, gamma, beta, running_mean, running_var, momentum, eps, training, mean, rstd, act,
           slope, ws):
    check(lib().kair_bn_fwd(ptr(z), ldz, ptr(out), dtype_code(out), ldo, M, C, ptr(gamma), ptr(beta), ptr(running_mean),
                            ptr(running_var), momentum, eps, int(training), ptr(mean), ptr(rstd), act, slope, ptr(ws),
                            stream_ptr()), "bn_fwd")


def bn_bwd(z, ldz, a, lda, da, ldda, dz, lddz, M, C, gamma, mean, rstd, act, slope, dgamma, dbeta, accumulate, ws):
    check(lib().kair_bn_bwd(ptr(z), ldz, ptr(a), dtype_code(a) if a is not None else F32, lda, ptr(da), ldda, ptr(dz),
                            dtype_code(dz), lddz, M, C, ptr(gamma), ptr(mean), ptr(rstd), act, slope, ptr(dgamma), ptr(dbeta),
                            int(accumulate), ptr(ws), stream_ptr()), "bn_bwd")


# ------------------------------------------------------------------------------------------
# training-patch synthesis (kair_amd/data/gpu_synth.py)
# ------------------------------------------------------------------------------------------
def synth_sr(pool, params, B, PS, sf, taps_h, taps_w, outH, outL):
    require_device(pool, params, outH, outL)
    N, C, Hs, Ws = pool.shape
    (ih, wh), (iw, ww) = taps_h, taps_w
    check(lib().kair_synth_sr(ptr(pool), C, Hs, Ws, ptr(params), B, PS, sf, ptr(wh), ptr(ih), ptr(ww), ptr(iw),
                              wh.shape[1], ptr(outH), ptr(outL), stream_ptr()), "synth_sr")


def synth_dn(pool, params, B, PS, sigma, seed, step, outH, outL):
    require_device(pool, params, outH, outL)
    N, C, Hs, Ws = pool.shape
    check(lib().kair_synth_dn(ptr(pool), C, Hs, Ws, ptr(params), B, PS, sigma, seed, step, ptr(outH), ptr(outL),
                              stream_ptr()), "synth_dn")


def swin_attn_fwd(x, ldx, gamma, beta, eps, C, ln, ldln, mean, rstd, wqkv, bqkv, qkv, table, scale, O, ldo, o_ones_col,
                  lse, wproj, bproj, rowscale, rows_per_scale, out, ldout, nWin, nh, H, W, shift, w_split=False):
    """Fused LN1 -> qkv -> window attention -> proj + residual (kair_swin_attn_fwd)."""
    check(lib().kair_swin_attn_fwd(ptr(x), ldx, ptr(gamma), ptr(beta), eps, C, ptr(ln), ldln, ptr(mean), ptr(rstd),
                                   ptr(wqkv), ptr(bqkv), ptr(qkv), ptr(table), scale, ptr(O), ldo, o_ones_col, ptr(lse),
                                   ptr(wproj), ptr(bproj), ptr(rowscale), rows_per_scale, ptr(out), ldout, nWin, nh, H, W,
                                   shift, int(w_split), stream_ptr()), "swin_attn_fwd")


def swin_mlp_fwd(x, ldx, gamma, beta, eps, C, ln, ldln, mean, rstd, w1, b1, u, h, ldh, hd, w2, b2, rowscale,
                 rows_per_scale, out, ldout, M, Cp, Hp, w_split=False):
    """Fused LN2 -> fc1 + GELU -> fc2 + residual (kair_swin_mlp_fwd)."""
    check(lib().kair_swin_mlp_fwd(ptr(x), ldx, ptr(gamma), ptr(beta), eps, C, ptr(ln), ldln, ptr(mean), ptr(rstd),
                                  ptr(w1), ptr(b1), ptr(u), ptr(h), ldh, hd, ptr(w2), ptr(b2), ptr(rowscale),
                                  rows_per_scale, ptr(out), ldout, M, Cp, Hp, int(w_split), stream_ptr()), "swin_mlp_fwd")


def debug_attn_stamps(n=8192 * 8):
    """Phase stamps of the last bf16 attention backward run with KAIR_ATTN_STAMP=1 (perf only)."""
    buf = (ctypes.c_ulonglong * n)()
    check(lib().kair_debug_attn_stamps(ctypes.cast(buf, c_vp), n), "debug_attn_stamps")
    return list(buf)


def debug_x3_stamps(n=4 * 8 * 64 * 5):
    """Phase stamps of the last x3 NT ring launch run with KAIR_RING_DBG bit 8 (debug builds, perf only):
    [CTA 0..3][wave][iteration 0..63][loop top, chunk waited, barrier + DMA issued, MFMAs done, epilogue done]."""
    import numpy as np
    buf = np.zeros(n, dtype=np.uint64)
    check(lib().kair_debug_x3_stamps(ctypes.c_void_p(buf.ctypes.data), n), "debug_x3_stamps")
    return buf


def debug_fused_stamps(n=4096 * 8):
    """Phase stamps of the last fused attention half run with KAIR_ATTN_DBG bit 8 (debug builds, perf only)."""
    buf = (ctypes.c_ulonglong * n)()
    check(lib().kair_debug_fused_stamps(ctypes.cast(buf, c_vp), n), "debug_fused_stamps")
    return list(buf)


def swin_mlp_bwd_ws():
    return lib().kair_swin_mlp_bwd_ws()


def swin_mlp_bwd(dc, gd, w2t, w1t, du, x, gamma, mean, rstd, C, D, dco, rowscale, rows_per_scale, H, W, shift,
                 dgamma, dbeta, ws, M, Cp, Hp, dparam_acc=False):
    """Fused MLP-half backward (kair_swin_mlp_bwd)."""
    check(lib().kair_swin_mlp_bwd(ptr(dc), dc.shape[-1], ptr(gd), gd.shape[-1], ptr(w2t), ptr(w1t), ptr(du), du.shape[-1],
                                  ptr(x), x.shape[-1], ptr(gamma), ptr(mean), ptr(rstd), C, ptr(D), D.shape[-1], ptr(dco),
                                  dco.shape[-1], ptr(rowscale), rows_per_scale, H, W, shift, ptr(dgamma), ptr(dbeta),
                                  int(dparam_acc), ptr(ws), M, Cp, Hp, stream_ptr()), "swin_mlp_bwd")


# ------------------------------------------------------------------------------------------
# Swin-block input gradients as row GEMMs with fused consumers (rowgemm.hip, bf16)
# ------------------------------------------------------------------------------------------
def _rg_check(A, W, K):
    require_device(A, W)
    if A.dtype != torch.bfloat16 or W.dtype != torch.bfloat16:
        raise TypeError("kair rowgemm: bf16 operands only")
    if A.stride(-1) != 1 or A.shape[-1] < K:
        raise ValueError("kair rowgemm: A must be row-major with at least K columns")


def rowgemm_store(A, M, K, W, N, out):
    """out[m, :N] = bf16(A[m, :K] . W^T), W in pack kind 13 (kair_rowgemm_store)."""
    _rg_check(A, W, K)
    check(lib().kair_rowgemm_store(ptr(A), A.stride(0) if A.dim() > 1 else K, M, K, ptr(W), N, ptr(out),
                                   out.stride(0) if out.dim() > 1 else N, stream_ptr()), "rowgemm_store")


def rowgemm_gate(A, M, K, W, N, gate, out):
    """out[m, :N] = bf16((A[m, :K] . W^T) * gate[m, :N]) (kair_rowgemm_gate)."""
    _rg_check(A, W, K)
    check(lib().kair_rowgemm_gate(ptr(A), A.stride(0), M, K, ptr(W), N, ptr(gate), gate.stride(0), ptr(out),
                                  out.stride(0), stream_ptr()), "rowgemm_gate")


def rowgemm_ln_blocks(M, K):
    n = lib().kair_rowgemm_ln_blocks(M, K)
    if n < 0:
        check(-1, "rowgemm_ln_blocks")
    return n


def rowgemm_lnbwd(A, M, K, W, x, gamma, mean, rstd, C, D, part, win=(0, 0, 0, 0), copy=None):
    """D[t] += LayerNorm-backward(A . W^T) with the copy / dgamma-dbeta partials (kair_rowgemm_lnbwd)."""
    _rg_check(A, W, K)
    check(lib().kair_rowgemm_lnbwd(ptr(A), A.stride(0), M, K, ptr(W), ptr(x), x.stride(0), ptr(gamma), ptr(mean),
                                   ptr(rstd), C, ptr(D), D.stride(0), *win,
                                   ctypes.byref(copy) if copy is not None else None, ptr(part), stream_ptr()),
          "rowgemm_lnbwd")
