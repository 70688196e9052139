"""PyTorch custom ops over libkair_hip: the `kair::` operator library.

The reference's native-op convention (models/op/fused_act.py:10-88: a JIT-built pybind11 module
+ torch.autograd.Function + nn.Module, TORCH_CHECK errors, the current stream) is replaced by
torch.library ops whose implementations call the C-ABI (include/kair_hip.h) through ctypes on
torch's current HIP stream, with autograd registered per op (register_autograd) so DDP and any
optimizer see ordinary .grad tensors, and fake (meta) kernels for shape propagation.

Only the CUDA dispatch key (HIP on PyTorch-ROCm) has a kernel.  A CPU tensor raises
NotImplementedError from the dispatcher: there is no CPU fallback.

  kair::linear(x, w, b, act, compute) -> (y, pre)          nn.Linear (+ exact GELU), network_swinir.py:19-30,105-107
  kair::linear_bwd(gy, x, w, pre, act, compute) -> (gx, gw, gb)
  kair::window_attn(qkv, table, mask, nh, scale, compute) -> (o, lse, o_pad)
                                                           WindowAttention core, network_swinir.py:114-143
  kair::window_attn_bwd(go, qkv, table, mask, lse, o_pad, nh, scale, compute) -> (gqkv, gtable)
  kair::layernorm(x, w, b, eps) -> (y, mean, rstd)         nn.LayerNorm, network_swinir.py:199,205
  kair::layernorm_bwd(gy, x, w, mean, rstd) -> (gx, gw, gb)
  kair::conv3x3(x, w, b, compute) -> y                     nn.Conv2d(3, 1, 1), network_swinir.py:465,669,729
  kair::conv3x3_bwd(gy, x, w, compute) -> (gx, gw, gb)

compute: 0 = exact fp32 MFMA (parity), 1 = bf16 MFMA with fp32 accumulation.  These ops are the
module-level surface (WindowAttention / SwinTransformerBlock / RSTB / forward_features callable on
their own); SwinIR.forward runs the whole network as one fused step program (engine) instead.
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _hip as H

F32, BF16 = 0, 1


def _rup(x, m):
    return (x + m - 1) // m * m


def _cd(compute):
    return H.BF16 if compute == BF16 else H.F32


def _tdt(compute):
    return torch.bfloat16 if compute == BF16 else torch.float32


def _padded(t, rows, cols, dtype):
    """t [rows, c] -> zero-padded contiguous [rows, cols] copy of dtype."""
    out = torch.zeros(rows, cols, device=t.device, dtype=dtype)
    out[:, :t.shape[1]] = t
    return out


def _wgrad(A, Bop, M, Np, Kp, wmap, grad, compute):
    """grad (reference layout) = finalize(sum_m A[m, n] B[m, k]) over the padded [Np][Kp] plane."""
    S = H.wgrad_splits(M, Np, Kp)
    ws = torch.empty(S * Np * Kp, device=grad.device)
    H.gemm_tn(A, Bop, ws, S, M, Np, Kp, _cd(compute))
    H.wgrad_finalize(ws, S, wmap, grad)


def _colsum(G, M, Np, N, grad):
    ws = torch.empty(1024 * Np, device=grad.device)
    H.colsum(H.rows(G), M, Np, H.wmap(4, N, 0, (1, N, Np), (1, 1, 1)), grad, ws)


# ------------------------------------------------------------------------------------------
# linear
# ------------------------------------------------------------------------------------------
@torch.library.custom_op("kair::linear", mutates_args=(), device_types="cuda")
def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor], act: int, compute: int) -> Tuple[Tensor, Tensor]:
    M, K = x.shape
    N = weight.shape[0]
    Kp, T = _rup(K, 8), _tdt(compute)
    A = _padded(x.float(), M, Kp, T)
    Bw = _padded(weight.detach().float(), N, Kp, T)
    y = torch.empty(M, N, device=x.device)
    pre = torch.empty(M, N, device=x.device) if act else torch.empty(0, device=x.device)
    b = bias.detach().float().contiguous() if bias is not None else None
    H.gemm_nt(H.rows(A), H.rows(Bw), H.epilogue(y, bias=b, act=H.ACT_GELU if act else H.ACT_NONE,
                                                pre=pre if act else None), M, N, Kp, _cd(compute))
    return y, pre


@linear.register_fake
def _(x, weight, bias, act, compute):
    M, N = x.shape[0], weight.shape[0]
    return x.new_empty(M, N), x.new_empty(M, N) if act else x.new_empty(0)


@torch.library.custom_op("kair::linear_bwd", mutates_args=(), device_types="cuda")
def linear_bwd(gy: Tensor, x: Tensor, weight: Tensor, pre: Tensor, act: int, compute: int,
               has_bias: bool) -> Tuple[Tensor, Tensor, Tensor]:
    M, K = x.shape
    N = weight.shape[0]
    Kp, Np, T = _rup(K, 8), _rup(N, 8), _tdt(compute)
    gz = torch.zeros(M, Np, device=x.device)
    if act:   # GELU' of the pre-activation (kair_act_grad_cast kind 3)
        H.act_grad_cast(gy.contiguous().float(), N, pre, N, gz, Np, M, N, 3)
    else:
        gz[:, :N] = gy
    gzc = gz.to(T) if T != torch.float32 else gz
    Wt = torch.zeros(Kp, Np, device=x.device, dtype=T)
    Wt[:K, :N] = weight.detach().t()
    gx = torch.empty(M, Kp, device=x.device)
    H.gemm_nt(H.rows(gzc), H.rows(Wt), H.epilogue(gx), M, Kp, Np, _cd(compute))
    gw = torch.empty(N, K, device=x.device)
    Ax = _padded(x.float(), M, Kp, T)
    _wgrad(H.rows(gzc), H.rows(Ax), M, Np, Kp, H.wmap(0, N, K, (1, N, Np), (1, K, Kp)), gw, compute)
    gb = torch.empty(N, device=x.device)
    if has_bias:
        _colsum(gz, M, Np, N, gb)
    return gx[:, :K].contiguous(), gw, gb


@linear_bwd.register_fake
def _(gy, x, weight, pre, act, compute, has_bias):
    return x.new_empty(x.shape), weight.new_empty(weight.shape), weight.new_empty(weight.shape[0])


def _linear_setup(ctx, inputs, output):
    x, weight, bias, act, compute = inputs
    ctx.save_for_backward(x, weight, output[1])
    ctx.act, ctx.compute, ctx.has_bias = act, compute, bias is not None


def _linear_backward(ctx, gy, gpre):
    x, weight, pre = ctx.saved_tensors
    gx, gw, gb = torch.ops.kair.linear_bwd(gy, x, weight, pre, ctx.act, ctx.compute, ctx.has_bias)
    return gx, gw, (gb if ctx.has_bias else None), None, None


torch.library.register_autograd("kair::linear", _linear_backward, setup_context=_linear_setup)


# ------------------------------------------------------------------------------------------
# window attention core: softmax(q*scale k^T + rel-pos bias (+ mask)) v per (window, head)
# ------------------------------------------------------------------------------------------
def _qkv_blocked(qkv, nh, T):
    """[B_, 64, 3C] -> head-blocked, head-padded [3][B_][nh][64][32] (the kernels' layout)."""
    B_, N, C3 = qkv.shape
    hd = C3 // (3 * nh)
    v = qkv.reshape(B_, N, 3, nh, hd).permute(2, 0, 3, 1, 4)
    out = torch.zeros(3, B_, nh, N, 32, device=qkv.device, dtype=T)
    out[..., :hd] = v
    return out


def _check_attn(qkv, nh, mask):
    B_, N, C3 = qkv.shape
    if N != 64 or C3 % (3 * nh) or C3 // (3 * nh) > 32:
        raise RuntimeError(f"kair::window_attn: 8x8 windows and head_dim <= 32 only (got N={N}, 3C={C3}, nh={nh})")
    if mask is not None and (mask.dim() != 3 or mask.shape[1:] != (64, 64) or B_ % mask.shape[0]):
        raise RuntimeError("kair::window_attn: mask must be [nW, 64, 64] with nW dividing the window count")


@torch.library.custom_op("kair::window_attn", mutates_args=(), device_types="cuda")
def window_attn(qkv: Tensor, table: Tensor, mask: Optional[Tensor], nh: int, scale: float,
                compute: int) -> Tuple[Tensor, Tensor, Tensor]:
    _check_attn(qkv, nh, mask)
    B_, N, C3 = qkv.shape
    C, hd, T = C3 // 3, C3 // (3 * nh), _tdt(compute)
    blk = _qkv_blocked(qkv.float(), nh, T)
    o_pad = torch.empty(B_ * N, nh * 32, device=qkv.device, dtype=T)
    lse = torch.empty(B_, nh, N, device=qkv.device)
    m = mask.float().contiguous() if mask is not None else None
    H.window_attn_fwd(blk, table.detach().float().contiguous(), o_pad, nh * 32, lse, B_, nh, hd, scale, 8, 8, 0,
                      mask=m)
    o = o_pad.view(B_, N, nh, 32)[..., :hd].reshape(B_, N, C).float()
    return o, lse, o_pad


@window_attn.register_fake
def _(qkv, table, mask, nh, scale, compute):
    B_, N, C3 = qkv.shape
    return (qkv.new_empty(B_, N, C3 // 3), qkv.new_empty(B_, nh, N),
            qkv.new_empty(B_ * N, nh * 32, dtype=_tdt(compute)))


@torch.library.custom_op("kair::window_attn_bwd", mutates_args=(), device_types="cuda")
def window_attn_bwd(go: Tensor, qkv: Tensor, table: Tensor, mask: Optional[Tensor], lse: Tensor, o_pad: Tensor, nh: int,
                    scale: float, compute: int) -> Tuple[Tensor, Tensor]:
    B_, N, C3 = qkv.shape
    C, hd, T = C3 // 3, C3 // (3 * nh), _tdt(compute)
    blk = _qkv_blocked(qkv.float(), nh, T)
    dO = torch.zeros(B_, N, nh, 32, device=qkv.device, dtype=T)
    dO[..., :hd] = go.reshape(B_, N, nh, hd)
    dblk = torch.empty_like(blk)
    dtable = torch.empty_like(table, dtype=torch.float32)
    ws = torch.empty(H.window_attn_bwd_ws(B_, nh), device=qkv.device)
    m = mask.float().contiguous() if mask is not None else None
    H.window_attn_bwd(blk, o_pad, nh * 32, dO.view(B_ * N, nh * 32), nh * 32, table.detach().float().contiguous(), lse,
                      dblk, dtable, False, ws, B_, nh, hd, scale, 8, 8, 0, mask=m)
    gqkv = dblk[..., :hd].permute(1, 3, 0, 2, 4).reshape(B_, N, C3).float()
    return gqkv, dtable


@window_attn_bwd.register_fake
def _(go, qkv, table, mask, lse, o_pad, nh, scale, compute):
    return qkv.new_empty(qkv.shape), table.new_empty(table.shape)


def _attn_setup(ctx, inputs, output):
    qkv, table, mask, nh, scale, compute = inputs
    ctx.save_for_backward(qkv, table, mask, output[1], output[2])
    ctx.nh, ctx.scale, ctx.compute = nh, scale, compute


def _attn_backward(ctx, go, glse, gopad):
    qkv, table, mask, lse, o_pad = ctx.saved_tensors
    gqkv, gtable = torch.ops.kair.window_attn_bwd(go, qkv, table, mask, lse, o_pad, ctx.nh, ctx.scale, ctx.compute)
    return gqkv, gtable, None, None, None, None


torch.library.register_autograd("kair::window_attn", _attn_backward, setup_context=_attn_setup)


# ------------------------------------------------------------------------------------------
# LayerNorm
# ------------------------------------------------------------------------------------------
def _ln_ok(x):
    if x.dim() != 2 or x.shape[1] > 256 or x.shape[1] % 4:
        raise RuntimeError("kair::layernorm: [M, C] rows with C <= 256, C % 4 == 0")


@torch.library.custom_op("kair::layernorm", mutates_args=(), device_types="cuda")
def layernorm(x: Tensor, weight: Tensor, bias: Tensor, eps: float) -> Tuple[Tensor, Tensor, Tensor]:
    _ln_ok(x)
    M, C = x.shape
    xc = x.float().contiguous()
    y = torch.empty(M, C, device=x.device)
    mean, rstd = torch.empty(M, device=x.device), torch.empty(M, device=x.device)
    H.layernorm_fwd(xc, C, y, C, weight.detach().float().contiguous(), bias.detach().float().contiguous(), mean, rstd, M,
                    C, eps)
    return y, mean, rstd


@layernorm.register_fake
def _(x, weight, bias, eps):
    return x.new_empty(x.shape), x.new_empty(x.shape[0]), x.new_empty(x.shape[0])


@torch.library.custom_op("kair::layernorm_bwd", mutates_args=(), device_types="cuda")
def layernorm_bwd(gy: Tensor, x: Tensor, weight: Tensor, mean: Tensor, rstd: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    M, C = x.shape
    gx = torch.empty(M, C, device=x.device)
    gw, gb = torch.empty(C, device=x.device), torch.empty(C, device=x.device)
    ws = torch.empty(2 * 2048 * C, device=x.device)
    H.layernorm_bwd(x.float().contiguous(), C, gy.float().contiguous(), C, weight.detach().float().contiguous(), mean,
                    rstd, gx, C, False, gw, gb, False, ws, M, C)
    return gx, gw, gb


@layernorm_bwd.register_fake
def _(gy, x, weight, mean, rstd):
    return x.new_empty(x.shape), weight.new_empty(weight.shape), weight.new_empty(weight.shape)


def _ln_setup(ctx, inputs, output):
    x, weight, bias, eps = inputs
    ctx.save_for_backward(x, weight, output[1], output[2])


def _ln_backward(ctx, gy, gmean, grstd):
    x, weight, mean, rstd = ctx.saved_tensors
    gx, gw, gb = torch.ops.kair.layernorm_bwd(gy, x, weight, mean, rstd)
    return gx, gw, gb, None


torch.library.register_autograd("kair::layernorm", _ln_backward, setup_context=_ln_setup)


# ------------------------------------------------------------------------------------------
# 3x3 / stride 1 / pad 1 convolution (implicit GEMM over NHWC rows)
# ------------------------------------------------------------------------------------------
def _nhwc(x, Cp, T):
    B, C, Hh, Ww = x.shape
    out = torch.zeros(B, Hh, Ww, Cp, device=x.device, dtype=T)
    out[..., :C] = x.permute(0, 2, 3, 1)
    return out.view(B * Hh * Ww, Cp)


def _conv_packed(w, Cop, Cip, T, flip=False):
    """forward [Cop][9*Cip] (k = tap*Cip + ci), or the dgrad form [Cip][9*Cop] with flipped taps."""
    Co, Ci = w.shape[:2]
    dst = torch.empty((Cip, 9 * Cop) if flip else (Cop, 9 * Cip), device=w.device, dtype=T)
    H.pack_weight(w.detach().float().contiguous(), dst, H.wmap(2 if flip else 1, Co, Ci, (1, Co, Cop), (1, Ci, Cip)))
    return dst


@torch.library.custom_op("kair::conv3x3", mutates_args=(), device_types="cuda")
def conv3x3(x: Tensor, weight: Tensor, bias: Optional[Tensor], compute: int) -> Tensor:
    B, C, Hh, Ww = x.shape
    Co = weight.shape[0]
    if weight.shape[1:] != (C, 3, 3):
        raise RuntimeError("kair::conv3x3: weight must be [Cout, Cin, 3, 3]")
    T = _tdt(compute)
    Cip, Cop = _rup(C, 8), _rup(Co, 8)
    A = _nhwc(x.float(), Cip, T)
    Wf = _conv_packed(weight, Cop, Cip, T)
    M = B * Hh * Ww
    y = torch.empty(M, Cop, device=x.device)
    bp = torch.zeros(Cop, device=x.device)
    if bias is not None:
        bp[:Co] = bias.detach().float()
    H.gemm_nt(H.im2col(A, Hh, Ww, Cip), H.rows(Wf), H.epilogue(y, bias=bp), M, Cop, 9 * Cip, _cd(compute))
    return y.view(B, Hh, Ww, Cop)[..., :Co].permute(0, 3, 1, 2).contiguous()


@conv3x3.register_fake
def _(x, weight, bias, compute):
    return x.new_empty(x.shape[0], weight.shape[0], x.shape[2], x.shape[3])


@torch.library.custom_op("kair::conv3x3_bwd", mutates_args=(), device_types="cuda")
def conv3x3_bwd(gy: Tensor, x: Tensor, weight: Tensor, compute: int, has_bias: bool) -> Tuple[Tensor, Tensor, Tensor]:
    B, C, Hh, Ww = x.shape
    Co = weight.shape[0]
    T = _tdt(compute)
    Cip, Cop = _rup(C, 8), _rup(Co, 8)
    M = B * Hh * Ww
    G32 = _nhwc(gy.float(), Cop, torch.float32)
    G = G32.to(T) if T != torch.float32 else G32
    Wd = _conv_packed(weight, Cop, Cip, T, flip=True)
    gx = torch.empty(M, Cip, device=x.device)
    H.gemm_nt(H.im2col(G, Hh, Ww, Cop, flip=True), H.rows(Wd), H.epilogue(gx), M, Cip, 9 * Cop, _cd(compute))
    A = _nhwc(x.float(), Cip, T)
    gw = torch.empty_like(weight, dtype=torch.float32)
    _wgrad(H.rows(G), H.im2col(A, Hh, Ww, Cip), M, Cop, 9 * Cip, H.wmap(1, Co, C, (1, Co, Cop), (1, C, Cip)), gw, compute)
    gb = torch.empty(Co, device=x.device)
    if has_bias:
        _colsum(G32, M, Cop, Co, gb)
    return gx.view(B, Hh, Ww, Cip)[..., :C].permute(0, 3, 1, 2).contiguous(), gw, gb


@conv3x3_bwd.register_fake
def _(gy, x, weight, compute, has_bias):
    return x.new_empty(x.shape), weight.new_empty(weight.shape), weight.new_empty(weight.shape[0])


def _conv_setup(ctx, inputs, output):
    x, weight, bias, compute = inputs
    ctx.save_for_backward(x, weight)
    ctx.compute, ctx.has_bias = compute, bias is not None


def _conv_backward(ctx, gy):
    x, weight = ctx.saved_tensors
    gx, gw, gb = torch.ops.kair.conv3x3_bwd(gy, x, weight, ctx.compute, ctx.has_bias)
    return gx, gw, (gb if ctx.has_bias else None), None


torch.library.register_autograd("kair::conv3x3", _conv_backward, setup_context=_conv_setup)


def registered_ops() -> List[str]:
    return ["linear", "linear_bwd", "window_attn", "window_attn_bwd", "layernorm", "layernorm_bwd", "conv3x3",
            "conv3x3_bwd"]
