"""Image utilities on the parity-defining path (mirror of /root/reference/utils/utils_image.py).

calculate_psnr  utils_image.py:629-644   (uint8 HxW[xC], float64 MSE, border shave)
tensor2uint     utils_image.py:296-300
single2uint     utils_image.py:261-263
uint2tensor3/4  utils_image.py:281-292
imresize        utils_image.py:938-1005  MATLAB bicubic (a = -0.5, antialias when shrinking,
                symmetric border).  Written as two separable resampling-matrix products so it runs
                batched on the device (the data-synthesis step feeding the hot path).
"""
import math

import numpy as np
import torch


def _cubic(x):
    ax = x.abs()
    return ((1.5 * ax ** 3 - 2.5 * ax ** 2 + 1) * (ax <= 1).to(x.dtype)
            + (-0.5 * ax ** 3 + 2.5 * ax ** 2 - 4 * ax + 2) * ((ax > 1) & (ax <= 2)).to(x.dtype))


_MAT_CACHE = {}


def resize_matrix(n_in, n_out, scale, antialias=True, device="cpu"):
    key = (n_in, n_out, float(scale), antialias, str(device))
    if key in _MAT_CACHE:
        return _MAT_CACHE[key]
    kw = 4.0 / scale if (scale < 1 and antialias) else 4.0
    u = torch.arange(1, n_out + 1, dtype=torch.float64) / scale + 0.5 * (1 - 1 / scale)
    left = torch.floor(u - kw / 2)
    P = math.ceil(kw) + 2
    idx = left[:, None] + torch.arange(P, dtype=torch.float64)[None]
    d = u[:, None] - idx
    w = (scale * _cubic(d * scale)) if (scale < 1 and antialias) else _cubic(d)
    w = (w / w.sum(1, keepdim=True)).float()
    # the reference drops an all-zero first/last column (same result either way)
    i = idx.long() - 1
    i = torch.where(i < 0, -i - 1, i)
    i = torch.where(i >= n_in, 2 * n_in - 1 - i, i)
    M = torch.zeros(n_out, n_in, dtype=torch.float32)
    M.index_put_((torch.arange(n_out)[:, None].expand_as(i), i), w, accumulate=True)
    M = M.to(device)
    _MAT_CACHE[key] = M
    return M


def imresize(img, scale, antialiasing=True):
    """img: [..., H, W] float tensor in [0, 1] (CHW, HW or a batch NCHW), any device."""
    Hh, Ww = img.shape[-2:]
    oh, ow = math.ceil(Hh * scale), math.ceil(Ww * scale)
    Mh = resize_matrix(Hh, oh, scale, antialiasing, img.device)
    Mw = resize_matrix(Ww, ow, scale, antialiasing, img.device)
    return torch.matmul(torch.matmul(Mh, img.float()), Mw.T)


def single2uint(img):
    return np.uint8((img.clip(0, 1) * 255.0).round())


def uint2single(img):
    return np.float32(img / 255.0)


def uint2tensor3(img):
    if img.ndim == 2:
        img = np.expand_dims(img, axis=2)
    return torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1).float().div(255.0)


def uint2tensor4(img):
    return uint2tensor3(img).unsqueeze(0)


def tensor2uint(img):
    img = img.detach().squeeze().float().clamp(0, 1).cpu().numpy()
    if img.ndim == 3:
        img = np.transpose(img, (1, 2, 0))
    return np.uint8((img * 255.0).round())


def calculate_psnr(img1, img2, border=0):
    if img1.shape != img2.shape:
        raise ValueError("Input images must have the same dimensions.")
    h, w = img1.shape[:2]
    a = img1[border:h - border, border:w - border].astype(np.float64)
    b = img2[border:h - border, border:w - border].astype(np.float64)
    mse = np.mean((a - b) ** 2)
    return float("inf") if mse == 0 else 20 * math.log10(255.0 / math.sqrt(mse))


def psnr_float(E, H):
    mse = torch.mean((E.double().clamp(0, 1) - H.double()) ** 2).item()
    return float("inf") if mse == 0 else -10 * math.log10(mse)


def synth_sr_batch(B, lq, scale, seed=0, device="cpu"):
    """Seeded synthetic SR patches: HR = clamp(bicubic-up(U[0,1) at HR/8) + 0.02 N, 0, 1),
    LQ = MATLAB-bicubic x1/scale of HR.  Generated on CPU with a torch.Generator, then moved."""
    g = torch.Generator().manual_seed(seed)
    hr = lq * scale
    base = torch.rand(B, 3, max(1, hr // 8), max(1, hr // 8), generator=g)
    Hh = torch.nn.functional.interpolate(base, size=(hr, hr), mode="bicubic", align_corners=False)
    Hh = (Hh + 0.02 * torch.randn(Hh.shape, generator=g)).clamp(0, 1)
    L = imresize(Hh, 1.0 / scale)
    return L.to(device), Hh.to(device)
