"""Oracle (test infrastructure only): fp32 CPU restatement of SwinIR.

Follows /root/reference/models/network_swinir.py.  Parameter/buffer names match the reference
state_dict exactly (550 entries for classical x4), so golden state_dicts load strictly.
DropPath is expressed as an explicit per-sample keep mask argument (None = identity), which makes
the oracle deterministic; the reference draws the mask from timm's DropPath (network_swinir.py:204).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def relative_position_index(ws):
    """network_swinir.py:92-102 — index into the (2ws-1)^2 bias table for each token pair."""
    ys, xs = torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")
    ys, xs = ys.flatten(), xs.flatten()
    dy = ys[:, None] - ys[None, :] + ws - 1
    dx = xs[:, None] - xs[None, :] + ws - 1
    return dy * (2 * ws - 1) + dx


def shift_region_mask(H, W, ws, shift):
    """network_swinir.py:216-237 — {0,-100} mask between tokens of different shifted regions."""
    def region(n):
        r = torch.zeros(n, dtype=torch.long)
        r[n - ws:n - shift] = 1
        r[n - shift:] = 2
        return r
    rid = region(H)[:, None] * 3 + region(W)[None, :]           # H, W
    win = rid.view(H // ws, ws, W // ws, ws).permute(0, 2, 1, 3).reshape(-1, ws * ws)
    diff = win[:, None, :] - win[:, :, None]
    return torch.where(diff != 0, torch.tensor(-100.0), torch.tensor(0.0))


def to_windows(x, ws):
    """network_swinir.py:33-45  (B,H,W,C) -> (B*nW, ws*ws, C)."""
    B, H, W, C = x.shape
    return x.view(B, H // ws, ws, W // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, C)


def from_windows(w, ws, B, H, W):
    """network_swinir.py:48-62."""
    C = w.shape[-1]
    return w.view(B, H // ws, W // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, H, W, C)


class Mlp(nn.Module):
    """network_swinir.py:14-30 (dropout p=0)."""

    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))


class WindowAttention(nn.Module):
    """network_swinir.py:65-145."""

    def __init__(self, dim, ws, heads):
        super().__init__()
        self.dim, self.ws, self.heads = dim, ws, heads
        self.scale = (dim // heads) ** -0.5
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) ** 2, heads))
        self.register_buffer("relative_position_index", relative_position_index(ws))
        self.qkv = nn.Linear(dim, 3 * dim)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x, mask=None):
        Bn, N, C = x.shape
        hd = C // self.heads
        q, k, v = self.qkv(x).view(Bn, N, 3, self.heads, hd).permute(2, 0, 3, 1, 4)
        s = (q * self.scale) @ k.transpose(-2, -1)                       # :124-125
        bias = self.relative_position_bias_table[self.relative_position_index.view(-1)]
        s = s + bias.view(N, N, self.heads).permute(2, 0, 1).unsqueeze(0)  # :127-130
        if mask is not None:                                              # :132-135
            nW = mask.shape[0]
            s = (s.view(Bn // nW, nW, self.heads, N, N) + mask[None, :, None]).view(Bn, self.heads, N, N)
        p = torch.softmax(s, dim=-1)
        o = (p @ v).transpose(1, 2).reshape(Bn, N, C)
        return self.proj(o)


class SwinTransformerBlock(nn.Module):
    """network_swinir.py:164-279."""

    def __init__(self, dim, res, heads, ws, shift, mlp_ratio):
        super().__init__()
        self.res, self.ws, self.shift = tuple(res), ws, shift
        if min(self.res) <= ws:                                           # :193-196
            self.shift, self.ws = 0, min(self.res)
        self.norm1 = nn.LayerNorm(dim)
        self.attn = WindowAttention(dim, self.ws, heads)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))
        mask = shift_region_mask(self.res[0], self.res[1], self.ws, self.shift) if self.shift > 0 else None
        self.register_buffer("attn_mask", mask)

    def forward(self, x, size, keep=None):
        H, W = size
        B, L, C = x.shape
        h = self.norm1(x).view(B, H, W, C)
        if self.shift:
            h = torch.roll(h, (-self.shift, -self.shift), (1, 2))
        if self.shift == 0:
            mask = None
        elif tuple(size) == self.res:
            mask = self.attn_mask
        else:
            mask = shift_region_mask(H, W, self.ws, self.shift)
        a = from_windows(self.attn(to_windows(h, self.ws), mask), self.ws, B, H, W)
        if self.shift:
            a = torch.roll(a, (self.shift, self.shift), (1, 2))
        a = a.reshape(B, L, C)
        if keep is not None:                                              # DropPath (train only)
            # timm DropPath draws the two branches' masks independently (:268, :275): keep may be
            # one per-sample scale for both branches or an (attn, mlp) pair
            ka, km = keep if isinstance(keep, (tuple, list)) else (keep, keep)
            x = x + a * ka
            return x + self.mlp(self.norm2(x)) * km
        x = x + a
        return x + self.mlp(self.norm2(x))


class _Group(nn.Module):
    def __init__(self, blocks):
        super().__init__()
        self.blocks = nn.ModuleList(blocks)


def resi_conv(dim, resi_connection):
    """The residual-connection conv of RSTB (network_swinir.py:464-471) and conv_after_body
    (:727-737): '1conv' = one 3x3 C->C; '3conv' = 3x3 C->C/4, LeakyReLU 0.2, 1x1 C/4->C/4,
    LeakyReLU 0.2, 3x3 C/4->C (same Sequential indices, so the state_dict keys match)."""
    if resi_connection == "1conv":
        return nn.Conv2d(dim, dim, 3, 1, 1)
    if resi_connection == "3conv":
        return nn.Sequential(nn.Conv2d(dim, dim // 4, 3, 1, 1), nn.LeakyReLU(0.2),
                             nn.Conv2d(dim // 4, dim // 4, 1, 1, 0), nn.LeakyReLU(0.2),
                             nn.Conv2d(dim // 4, dim, 3, 1, 1))
    raise ValueError(resi_connection)


class RSTB(nn.Module):
    """network_swinir.py:419-482."""

    def __init__(self, dim, res, depth, heads, ws, mlp_ratio, resi_connection="1conv"):
        super().__init__()
        self.residual_group = _Group([SwinTransformerBlock(dim, res, heads, ws, 0 if i % 2 == 0 else ws // 2,
                                                           mlp_ratio) for i in range(depth)])
        self.conv = resi_conv(dim, resi_connection)

    def forward(self, x, size, keeps=None):
        h = x
        for i, blk in enumerate(self.residual_group.blocks):
            h = blk(h, size, None if keeps is None else keeps[i])
        B, L, C = h.shape
        img = h.transpose(1, 2).reshape(B, C, size[0], size[1])         # PatchUnEmbed :562-565
        return self.conv(img).flatten(2).transpose(1, 2) + x            # PatchEmbed :524-528


class _Norm(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.norm = nn.LayerNorm(dim)


class SwinIR(nn.Module):
    """network_swinir.py:618-839.  Supports upsampler 'pixelshuffle', 'pixelshuffledirect',
    'nearest+conv' and '' (denoise / JPEG)."""

    def __init__(self, upscale=2, in_chans=3, img_size=64, window_size=7, img_range=1.0,
                 depths=(6, 6, 6, 6), embed_dim=96, num_heads=(6, 6, 6, 6), mlp_ratio=4.0,
                 upsampler="", resi_connection="1conv"):
        super().__init__()
        self.upscale, self.upsampler, self.window_size, self.img_range = upscale, upsampler, window_size, img_range
        self.mean = (torch.tensor([0.4488, 0.4371, 0.4040]) if in_chans == 3 else torch.zeros(1)).view(1, -1, 1, 1)
        img_size = img_size if isinstance(img_size, (tuple, list)) else (img_size, img_size)
        self.res = tuple(img_size)
        self.depths = list(depths)
        C, nf = embed_dim, 64
        self.conv_first = nn.Conv2d(in_chans, C, 3, 1, 1)
        self.patch_embed = _Norm(C)
        self.layers = nn.ModuleList([RSTB(C, self.res, d, h, window_size, mlp_ratio, resi_connection)
                                     for d, h in zip(depths, num_heads)])
        self.norm = nn.LayerNorm(C)
        self.conv_after_body = resi_conv(C, resi_connection)
        if upsampler == "pixelshuffle":
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(C, nf, 3, 1, 1), nn.LeakyReLU(0.01))
            ups = []
            if scale_is_pow2(upscale):
                for _ in range(int(math.log2(upscale))):
                    ups += [nn.Conv2d(nf, 4 * nf, 3, 1, 1), nn.PixelShuffle(2)]
            else:
                ups += [nn.Conv2d(nf, 9 * nf, 3, 1, 1), nn.PixelShuffle(3)]
            self.upsample = nn.Sequential(*ups)
            self.conv_last = nn.Conv2d(nf, in_chans, 3, 1, 1)
        elif upsampler == "pixelshuffledirect":
            self.upsample = nn.Sequential(nn.Conv2d(C, upscale ** 2 * in_chans, 3, 1, 1), nn.PixelShuffle(upscale))
        elif upsampler == "nearest+conv":
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(C, nf, 3, 1, 1), nn.LeakyReLU(0.01))
            self.conv_up1 = nn.Conv2d(nf, nf, 3, 1, 1)
            self.conv_up2 = nn.Conv2d(nf, nf, 3, 1, 1)
            self.conv_hr = nn.Conv2d(nf, nf, 3, 1, 1)
            self.conv_last = nn.Conv2d(nf, in_chans, 3, 1, 1)
        else:
            self.conv_last = nn.Conv2d(C, in_chans, 3, 1, 1)

    def features(self, x, keeps=None):
        """forward_features :790-803."""
        size = (x.shape[2], x.shape[3])
        h = self.patch_embed.norm(x.flatten(2).transpose(1, 2))
        i0 = 0
        for layer, d in zip(self.layers, self.depths):
            h = layer(h, size, None if keeps is None else keeps[i0:i0 + d])
            i0 += d
        h = self.norm(h)
        B, L, C = h.shape
        return h.transpose(1, 2).reshape(B, C, size[0], size[1])

    def forward(self, x, keeps=None):
        H, W = x.shape[2:]
        ws = self.window_size
        ph, pw = (ws - H % ws) % ws, (ws - W % ws) % ws
        x = F.pad(x, (0, pw, 0, ph), "reflect")                         # check_image_size :783-788
        mean = self.mean.type_as(x)
        x = (x - mean) * self.img_range
        lrelu = lambda t: F.leaky_relu(t, 0.2)
        if self.upsampler == "pixelshuffle":
            f = self.conv_first(x)
            f = self.conv_after_body(self.features(f, keeps)) + f
            x = self.conv_last(self.upsample(self.conv_before_upsample(f)))
        elif self.upsampler == "pixelshuffledirect":
            f = self.conv_first(x)
            x = self.upsample(self.conv_after_body(self.features(f, keeps)) + f)
        elif self.upsampler == "nearest+conv":
            f = self.conv_first(x)
            f = self.conv_before_upsample(self.conv_after_body(self.features(f, keeps)) + f)
            f = lrelu(self.conv_up1(F.interpolate(f, scale_factor=2, mode="nearest")))
            f = lrelu(self.conv_up2(F.interpolate(f, scale_factor=2, mode="nearest")))
            x = self.conv_last(lrelu(self.conv_hr(f)))
        else:
            f = self.conv_first(x)
            x = x + self.conv_last(self.conv_after_body(self.features(f, keeps)) + f)
        x = x / self.img_range + mean
        return x[:, :, :H * self.upscale, :W * self.upscale]


def scale_is_pow2(s):
    return s & (s - 1) == 0
