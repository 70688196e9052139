"""SwinIR on MI355X — drop-in for /root/reference/models/network_swinir.py.

The module tree, parameter names/shapes, buffers (relative_position_index int64, attn_mask on
shifted blocks) and initialisation follow the reference (network_swinir.py:65-773), so reference
checkpoints load strictly and define_G() callers see the same object.

Two ways in:
  * SwinIR.forward hands the whole network to the HIP step program in
    kair_amd/engine/swinir_engine.py (fused window attention, implicit-GEMM convs, fused
    epilogues, one autograd node) -- the training / inference hot path;
  * every submodule is also callable on its own, as in the reference -- Mlp.forward,
    WindowAttention.forward(x, mask), SwinTransformerBlock.forward(x, x_size),
    BasicLayer/RSTB.forward(x, x_size), PatchEmbed/PatchUnEmbed, SwinIR.forward_features /
    check_image_size -- dispatching to the torch.ops.kair.* custom ops (kair_amd/ops.py) with
    autograd per op.
There is no CPU path; a CPU input raises.  Module-level ops compute in exact fp32 unless the
owning SwinIR was built with compute_dtype 'bf16' (attribute `compute` on each op module).
"""
import logging
import math

import torch
import torch.nn as nn

from .. import ops as kops  # noqa: F401  (registers torch.ops.kair.*)
from ..engine.swinir_engine import SwinIREngine, SwinIRFunction


def _need_device(x):
    if not x.is_cuda:
        raise RuntimeError("kair_amd SwinIR modules run on the MI355X (HIP) only; got a CPU tensor (no CPU fallback)")


class Linear(nn.Linear):
    """nn.Linear whose forward is torch.ops.kair.linear (same parameters / state_dict)."""
    compute = 0

    def forward(self, x):
        _need_device(x)
        shp = x.shape
        y, _ = torch.ops.kair.linear(x.reshape(-1, shp[-1]), self.weight, self.bias, 0, self.compute)
        return y.view(*shp[:-1], self.out_features)


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm whose forward is torch.ops.kair.layernorm."""

    def forward(self, x):
        _need_device(x)
        shp = x.shape
        y, _, _ = torch.ops.kair.layernorm(x.reshape(-1, shp[-1]), self.weight, self.bias, self.eps)
        return y.view(shp)


class Conv3x3(nn.Conv2d):
    """nn.Conv2d(C, C, 3, 1, 1) whose forward is torch.ops.kair.conv3x3."""
    compute = 0

    def forward(self, x):
        _need_device(x)
        return torch.ops.kair.conv3x3(x, self.weight, self.bias, self.compute)


def _drop_path(x, rate, training):
    """timm DropPath (network_swinir.py:204): per-sample keep mask / keep."""
    if rate == 0.0 or not training:
        return x
    keep = 1.0 - rate
    m = (torch.rand((x.shape[0],) + (1,) * (x.dim() - 1), device=x.device) < keep).to(x.dtype)
    return x * m / keep


def _pair(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, x)


def _trunc_normal(t, std=0.02):
    return nn.init.trunc_normal_(t, std=std, a=-2.0, b=2.0)


def _relative_position_index(ws):
    """network_swinir.py:92-102."""
    ys, xs = torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")
    ys, xs = ys.flatten(), xs.flatten()
    return (ys[:, None] - ys[None, :] + ws - 1) * (2 * ws - 1) + (xs[:, None] - xs[None, :] + ws - 1)


def _shift_mask(H, W, ws, shift):
    """network_swinir.py:216-237 (calculate_mask), kept only as the state_dict buffer."""
    def region(n):
        r = torch.zeros(n, dtype=torch.long)
        r[n - ws:n - shift] = 1
        r[n - shift:] = 2
        return r
    rid = region(H)[:, None] * 3 + region(W)[None, :]
    win = rid.view(H // ws, ws, W // ws, ws).permute(0, 2, 1, 3).reshape(-1, ws * ws)
    d = win[:, None, :] - win[:, :, None]
    return torch.zeros(d.shape).masked_fill(d != 0, -100.0)


class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0):
        super().__init__()
        self.fc1 = Linear(in_features, hidden_features or in_features)
        self.act = act_layer()
        self.fc2 = Linear(hidden_features or in_features, out_features or in_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        """network_swinir.py:24-30: fc1 -> GELU (fused in the fc1 epilogue) -> fc2 (dropout p=0)."""
        _need_device(x)
        shp = x.shape
        h, _ = torch.ops.kair.linear(x.reshape(-1, shp[-1]), self.fc1.weight, self.fc1.bias, 1, self.fc1.compute)
        return self.drop(self.fc2(self.drop(h))).view(*shp[:-1], self.fc2.out_features)


class WindowAttention(nn.Module):
    def __init__(self, dim, window_size, num_heads, qkv_bias=True, qk_scale=None, attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.dim, self.window_size, self.num_heads = dim, _pair(window_size), num_heads
        self.scale = qk_scale or (dim // num_heads) ** -0.5
        ws = self.window_size[0]
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) * (2 * ws - 1), num_heads))
        self.register_buffer("relative_position_index", _relative_position_index(ws))
        self.qkv = Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)
        _trunc_normal(self.relative_position_bias_table)
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, x, mask=None):
        """network_swinir.py:114-145.  x [num_windows*B, 64, C]; mask (0/-100) [num_windows, 64, 64] or
        None.  q*scale @ k^T + rel-pos bias (+ mask), softmax, @ v in one HIP kernel per (window, head);
        the relative-position gather is computed from indices (relative_position_index is the buffer
        of :92-103, kept for checkpoints)."""
        _need_device(x)
        B_, N, C = x.shape
        qkv = self.qkv(x)
        o, _, _ = torch.ops.kair.window_attn(qkv, self.relative_position_bias_table, mask, self.num_heads,
                                             float(self.scale), self.qkv.compute)
        return self.proj_drop(self.proj(o))


class SwinTransformerBlock(nn.Module):
    def __init__(self, dim, input_resolution, num_heads, window_size=7, shift_size=0, mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0, act_layer=nn.GELU, norm_layer=LayerNorm):
        super().__init__()
        self.dim, self.input_resolution, self.num_heads = dim, tuple(input_resolution), num_heads
        self.window_size, self.shift_size, self.mlp_ratio = window_size, shift_size, mlp_ratio
        if min(self.input_resolution) <= self.window_size:
            self.shift_size, self.window_size = 0, min(self.input_resolution)
        self.norm1 = norm_layer(dim)
        self.attn = WindowAttention(dim, self.window_size, num_heads, qkv_bias, qk_scale, attn_drop, drop)
        self.drop_path_rate = float(drop_path)
        self.drop_path = nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio), act_layer=act_layer, drop=drop)
        mask = _shift_mask(*self.input_resolution, self.window_size, self.shift_size) if self.shift_size > 0 else None
        self.register_buffer("attn_mask", mask)

    def calculate_mask(self, x_size):
        """network_swinir.py:216-237."""
        return _shift_mask(x_size[0], x_size[1], self.window_size, self.shift_size)

    def forward(self, x, x_size):
        """network_swinir.py:239-279: LN1, cyclic shift, window partition, W-MSA, reverse, residual +
        DropPath, LN2, MLP, residual + DropPath (roll / partition are device tensor views here; the
        engine folds them into address maps)."""
        _need_device(x)
        Hh, Ww = x_size
        B, L, C = x.shape
        ws, sh = self.window_size, self.shift_size
        h = self.norm1(x).view(B, Hh, Ww, C)
        if sh > 0:
            h = torch.roll(h, shifts=(-sh, -sh), dims=(1, 2))
        win = h.view(B, Hh // ws, ws, Ww // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, C)
        if sh > 0:
            mask = self.attn_mask if tuple(x_size) == tuple(self.input_resolution) else self.calculate_mask(x_size).to(x.device)
        else:
            mask = None
        a = self.attn(win, mask=mask)
        a = a.view(B, Hh // ws, Ww // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, Hh, Ww, C)
        if sh > 0:
            a = torch.roll(a, shifts=(sh, sh), dims=(1, 2))
        x = x + _drop_path(a.reshape(B, Hh * Ww, C), self.drop_path_rate, self.training)
        return x + _drop_path(self.mlp(self.norm2(x)), self.drop_path_rate, self.training)


class BasicLayer(nn.Module):
    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0, norm_layer=LayerNorm, downsample=None,
                 use_checkpoint=False):
        super().__init__()
        self.dim, self.input_resolution, self.depth = dim, input_resolution, depth
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim, input_resolution, num_heads, window_size, 0 if i % 2 == 0 else window_size // 2,
                                 mlp_ratio, qkv_bias, qk_scale, drop, attn_drop,
                                 drop_path[i] if isinstance(drop_path, list) else drop_path, norm_layer=norm_layer)
            for i in range(depth)])
        self.downsample = None

    def forward(self, x, x_size):
        for blk in self.blocks:
            x = blk(x, x_size)
        return x


class PatchEmbed(nn.Module):
    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__()
        img_size, patch_size = _pair(img_size), _pair(patch_size)
        self.img_size, self.patch_size = img_size, patch_size
        self.patches_resolution = [img_size[0] // patch_size[0], img_size[1] // patch_size[1]]
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans, self.embed_dim = in_chans, embed_dim
        self.norm = norm_layer(embed_dim) if norm_layer is not None else None

    def forward(self, x):
        """network_swinir.py:524-528: [B, C, H, W] -> [B, HW, C] (+ LayerNorm)."""
        x = x.flatten(2).transpose(1, 2)
        return self.norm(x) if self.norm is not None else x


class PatchUnEmbed(PatchEmbed):
    def __init__(self, img_size=224, patch_size=4, in_chans=3, embed_dim=96, norm_layer=None):
        super().__init__(img_size, patch_size, in_chans, embed_dim, None)

    def forward(self, x, x_size):
        """network_swinir.py:562-565: [B, HW, C] -> [B, C, H, W]."""
        B, HW, C = x.shape
        return x.transpose(1, 2).reshape(B, self.embed_dim, x_size[0], x_size[1])


class Conv1x1(nn.Conv2d):
    """nn.Conv2d(Ci, Co, 1, 1, 0) whose forward is torch.ops.kair.linear over NHWC pixel rows."""
    compute = 0

    def forward(self, x):
        _need_device(x)
        B, C, Hh, Ww = x.shape
        rows = x.permute(0, 2, 3, 1).reshape(B * Hh * Ww, C)
        y, _ = torch.ops.kair.linear(rows, self.weight.view(self.out_channels, C), self.bias, 0, self.compute)
        return y.view(B, Hh, Ww, -1).permute(0, 3, 1, 2).contiguous()


def resi_conv(dim, resi_connection):
    """The residual-connection conv of RSTB (network_swinir.py:464-471) and conv_after_body (:727-737):
    '1conv' one 3x3 C->C; '3conv' 3x3 C->C/4, LeakyReLU 0.2, 1x1 C/4->C/4, LeakyReLU 0.2, 3x3 C/4->C
    (the same Sequential indices as the reference, so the state_dict keys match)."""
    if resi_connection == "1conv":
        return Conv3x3(dim, dim, 3, 1, 1)
    if resi_connection == "3conv":
        return nn.Sequential(Conv3x3(dim, dim // 4, 3, 1, 1), nn.LeakyReLU(negative_slope=0.2, inplace=True),
                             Conv1x1(dim // 4, dim // 4, 1, 1, 0), nn.LeakyReLU(negative_slope=0.2, inplace=True),
                             Conv3x3(dim // 4, dim, 3, 1, 1))
    raise ValueError(f"resi_connection {resi_connection!r}")


class RSTB(nn.Module):
    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, drop=0.0, attn_drop=0.0, drop_path=0.0, norm_layer=LayerNorm, downsample=None,
                 use_checkpoint=False, img_size=224, patch_size=4, resi_connection="1conv"):
        super().__init__()
        self.dim, self.input_resolution = dim, input_resolution
        self.residual_group = BasicLayer(dim, input_resolution, depth, num_heads, window_size, mlp_ratio, qkv_bias,
                                         qk_scale, drop, attn_drop, drop_path, norm_layer)
        self.conv = resi_conv(dim, resi_connection)
        self.patch_embed = PatchEmbed(img_size, patch_size, 0, dim, None)
        self.patch_unembed = PatchUnEmbed(img_size, patch_size, 0, dim, None)

    def forward(self, x, x_size):
        """network_swinir.py:481-482."""
        return self.patch_embed(self.conv(self.patch_unembed(self.residual_group(x, x_size), x_size))) + x


class Upsample(nn.Sequential):
    def __init__(self, scale, num_feat):
        m = []
        if scale & (scale - 1) == 0:
            for _ in range(int(math.log2(scale))):
                m += [nn.Conv2d(num_feat, 4 * num_feat, 3, 1, 1), nn.PixelShuffle(2)]
        elif scale == 3:
            m += [nn.Conv2d(num_feat, 9 * num_feat, 3, 1, 1), nn.PixelShuffle(3)]
        else:
            raise ValueError(f"scale {scale} is not supported. Supported scales: 2^n and 3.")
        super().__init__(*m)


class UpsampleOneStep(nn.Sequential):
    def __init__(self, scale, num_feat, num_out_ch, input_resolution=None):
        self.num_feat, self.input_resolution = num_feat, input_resolution
        super().__init__(nn.Conv2d(num_feat, scale ** 2 * num_out_ch, 3, 1, 1), nn.PixelShuffle(scale))


class SwinIR(nn.Module):
    """Same constructor signature as the reference SwinIR (network_swinir.py:646-652).

    Extra (engine) options, all keyword-only and absent from the reference:
      compute_dtype  'bf16' (default, MFMA bf16 with fp32 accumulation/master weights) or 'fp32'
                     (exact fp32 MFMA; the parity mode)
      split_conv     bf16 only (default True): forward 3x3 convs use hi/lo bf16 weight pairs, which
                     removes the output bias of bf16 weight rounding (DESIGN.md "parity at bf16")
      fused_blocks   bf16 only (default True): fused Swin-block kernels where the geometry allows
    """

    def __init__(self, img_size=64, patch_size=1, in_chans=3, embed_dim=96, depths=(6, 6, 6, 6),
                 num_heads=(6, 6, 6, 6), window_size=7, mlp_ratio=4.0, qkv_bias=True, qk_scale=None, drop_rate=0.0,
                 attn_drop_rate=0.0, drop_path_rate=0.1, norm_layer=LayerNorm, ape=False, patch_norm=True,
                 use_checkpoint=False, upscale=2, img_range=1.0, upsampler="", resi_connection="1conv",
                 compute_dtype="fp32", split_conv=True, fused_blocks=True, **kwargs):
        super().__init__()
        if ape or not patch_norm or patch_size != 1 or not qkv_bias or qk_scale is not None:
            raise NotImplementedError("kair_amd SwinIR: ape / patch_norm=False / patch_size!=1 / custom qk are off-path")
        num_in_ch = num_out_ch = in_chans
        num_feat = 64
        self.img_range = img_range
        self.mean = torch.Tensor((0.4488, 0.4371, 0.4040)).view(1, 3, 1, 1) if in_chans == 3 else torch.zeros(1, 1, 1, 1)
        self.upscale, self.upsampler, self.window_size = upscale, upsampler, window_size
        self.conv_first = nn.Conv2d(num_in_ch, embed_dim, 3, 1, 1)
        self.num_layers, self.embed_dim, self.ape, self.patch_norm = len(depths), embed_dim, ape, patch_norm
        self.num_features, self.mlp_ratio = embed_dim, mlp_ratio
        self.patch_embed = PatchEmbed(img_size, patch_size, embed_dim, embed_dim, norm_layer if patch_norm else None)
        self.patches_resolution = self.patch_embed.patches_resolution
        self.patch_unembed = PatchUnEmbed(img_size, patch_size, embed_dim, embed_dim, None)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]   # network_swinir.py:701
        self.layers = nn.ModuleList()
        for i in range(self.num_layers):
            self.layers.append(RSTB(embed_dim, tuple(self.patches_resolution), depths[i], num_heads[i], window_size,
                                    mlp_ratio, qkv_bias, qk_scale, drop_rate, attn_drop_rate,
                                    dpr[sum(depths[:i]):sum(depths[:i + 1])], norm_layer, None, use_checkpoint,
                                    img_size, patch_size, resi_connection))
        self.norm = norm_layer(self.num_features)
        self.conv_after_body = resi_conv(embed_dim, resi_connection)
        if upsampler == "pixelshuffle":
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(embed_dim, num_feat, 3, 1, 1), nn.LeakyReLU(inplace=True))
            self.upsample = Upsample(upscale, num_feat)
            self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
        elif upsampler == "pixelshuffledirect":
            self.upsample = UpsampleOneStep(upscale, embed_dim, num_out_ch, tuple(self.patches_resolution))
        elif upsampler == "nearest+conv":   # real-world SR (network_swinir.py:751-760)
            assert self.upscale == 4, "only support x4 now."
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(embed_dim, num_feat, 3, 1, 1), nn.LeakyReLU(inplace=True))
            self.conv_up1 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
            self.conv_up2 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
            self.conv_hr = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
            self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)
            self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)
        else:   # denoising / JPEG artifact reduction, upsampler None or '' (network_swinir.py:761-763)
            self.conv_last = nn.Conv2d(embed_dim, num_out_ch, 3, 1, 1)
        self.apply(self._init_weights)
        self.compute_dtype = compute_dtype
        self._set_op_compute()
        self.split_conv = split_conv
        self.fused_blocks = fused_blocks
        self._engine = None
        # evaluation numerics of the bf16 engine: the Swin-block linears also multiply hi/lo split weight
        # pairs (SwinIREngine split_linear) in eval-mode forwards, on top of the training step's split conv
        # weights and activations -- the bf16 rounding of the linear weights is half of the forward's
        # remaining output error (profiles/r04_drift_ablation.txt); eval is not on the timed path
        self.eval_split_linear = True
        self._engine_eval = None

    @staticmethod
    def _init_weights(m):
        """network_swinir.py:766-773."""
        if isinstance(m, nn.Linear):
            _trunc_normal(m.weight)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    @torch.jit.ignore
    def no_weight_decay(self):
        return {"absolute_pos_embed"}

    @torch.jit.ignore
    def no_weight_decay_keywords(self):
        return {"relative_position_bias_table"}

    # ------------------------------------------------------------------------------------
    def engine(self):
        if self._engine is None or self._engine.net_ref() is not self:
            self._engine = SwinIREngine(self, self.compute_dtype, self.split_conv, self.fused_blocks)
            logging.getLogger("kair_amd").info("SwinIR: %s engine (%s)", self.compute_dtype, {
                "fp32": "exact-fp32 MFMA; compute_dtype='fp32x3' is the same precision class at ~2.7x the speed",
                "fp32x3": "fp16-pair products, fp32 accumulation", "bf16": "split-operand bf16"}[self.compute_dtype])
        return self._engine

    def eval_engine(self):
        """The engine of eval-mode forwards: the training engine, or for bf16 with eval_split_linear its
        split-linear twin (same kernels, hi/lo weight pairs in the fused block kernels)."""
        if self.compute_dtype != "bf16" or not self.eval_split_linear:
            return self.engine()
        if self._engine_eval is None or self._engine_eval.net_ref() is not self:
            self._engine_eval = SwinIREngine(self, self.compute_dtype, self.split_conv, self.fused_blocks, split_linear=True,
                                             side_stream=False)
            self._engine_eval.repack_always = True   # the trainer's Adam kernel leaves parameter versions alone
        return self._engine_eval

    def _apply(self, fn, *args, **kwargs):
        self._engine = None     # packed buffers live on the old device / dtype
        self._engine_eval = None
        return super()._apply(fn, *args, **kwargs)

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        self._engine = None
        self._engine_eval = None
        self._set_op_compute()
        return self

    def _set_op_compute(self):
        for m in self.modules():
            if isinstance(m, (Linear, Conv3x3, Conv1x1)):
                m.compute = 1 if self.compute_dtype == "bf16" else 0

    def check_image_size(self, x):
        """network_swinir.py:783-788: reflect-pad H, W up to multiples of window_size."""
        _, _, h, w = x.size()
        ph = (self.window_size - h % self.window_size) % self.window_size
        pw = (self.window_size - w % self.window_size) % self.window_size
        return torch.nn.functional.pad(x, (0, pw, 0, ph), "reflect") if (ph or pw) else x

    def forward_features(self, x):
        """network_swinir.py:790-803 on the torch.ops.kair.* module path: x [B, C, H, W] (after
        conv_first) -> normalised deep features [B, C, H, W]."""
        _need_device(x)
        x_size = (x.shape[2], x.shape[3])
        x = self.pos_drop(self.patch_embed(x))
        for layer in self.layers:
            x = layer(x, x_size)
        return self.patch_unembed(self.norm(x), x_size)

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("kair_amd SwinIR runs on the MI355X (HIP) only; got a CPU tensor (no CPU fallback)")
        params = [p for p in self.parameters()]
        eng = self.engine() if self.training else self.eval_engine()
        return SwinIRFunction.run(eng, x, params)

    def flops(self):
        """Training FLOPs are tracked by kair_amd.engine.swinir_engine.swinir_flops()."""
        from ..engine.swinir_engine import swinir_flops
        H, W = self.patches_resolution
        return swinir_flops(self, H, W)["fwd"]
