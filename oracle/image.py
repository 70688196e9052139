"""Oracle (test infrastructure only): image utilities on the parity-defining path.

imresize_matlab  — /root/reference/utils/utils_image.py:872-1005 (MATLAB bicubic, a=-0.5, antialias
                   when downscaling, symmetric border extension); written as two separable
                   weight-matrix products instead of the reference's per-row loops.
calculate_psnr   — utils_image.py:629-644 (uint8 inputs, float64 MSE, border shave)
tensor2uint      — utils_image.py:296-300
"""
import math

import numpy as np
import torch


def _cubic(x):
    ax = x.abs()
    ax2, ax3 = ax * ax, ax * ax * ax
    return ((1.5 * ax3 - 2.5 * ax2 + 1) * (ax <= 1).to(x.dtype)
            + (-0.5 * ax3 + 2.5 * ax2 - 4 * ax + 2) * ((ax > 1) & (ax <= 2)).to(x.dtype))


def resize_matrix(n_in, n_out, scale, antialias=True):
    """Dense (n_out, n_in) resampling matrix equal to calculate_weights_indices (:880-932)
    followed by the symmetric padding of imresize (:956-975)."""
    kw = 4.0
    if scale < 1 and antialias:
        kw = kw / scale
    x = torch.linspace(1, n_out, n_out)
    u = x / scale + 0.5 * (1 - 1 / scale)
    left = torch.floor(u - kw / 2)
    P = math.ceil(kw) + 2
    idx = left[:, None] + torch.arange(P, dtype=torch.float32)[None, :]
    dist = u[:, None] - idx
    w = scale * _cubic(dist * scale) if (scale < 1 and antialias) else _cubic(dist)
    w = w / w.sum(1, keepdim=True)
    zeros = (w == 0).sum(0)
    if zeros[0] != 0:
        idx, w = idx[:, 1:], w[:, 1:]
    if zeros[-1] != 0:
        idx, w = idx[:, :-1], w[:, :-1]
    # 1-based input index i -> symmetric reflection into [1, n_in] (MATLAB 'symmetric')
    i = idx.long() - 1
    i = torch.where(i < 0, -i - 1, i)
    i = torch.where(i >= n_in, 2 * n_in - 1 - i, i)
    M = torch.zeros(n_out, n_in, dtype=torch.float32)
    M.index_put_((torch.arange(n_out)[:, None].expand_as(i), i), w.float(), accumulate=True)
    return M


def imresize_matlab(img, scale, antialias=True):
    """img: CHW or HW float tensor in [0,1]; returns the resized tensor (no rounding)."""
    squeeze = img.dim() == 2
    if squeeze:
        img = img[None]
    C, H, W = img.shape
    oh, ow = math.ceil(H * scale), math.ceil(W * scale)
    Mh = resize_matrix(H, oh, scale, antialias)
    Mw = resize_matrix(W, ow, scale, antialias)
    out = torch.einsum("oh,chw->cow", Mh, img.float())
    out = torch.einsum("pw,cow->cop", Mw, out)
    return out[0] if squeeze else out


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
    """Float PSNR on [0,1] tensors (SURVEY §8d PSNR parity form 1)."""
    mse = torch.mean((E.double().clamp(0, 1) - H.double()) ** 2).item()
    return float("inf") if mse == 0 else -10 * math.log10(mse)
