"""Image utilities on the parity-defining path (mirror of /root/reference/utils/utils_image.py).

calculate_psnr  utils_image.py:629-644   (uint8 HxW[xC], float64 MSE, border shave)
calculate_ssim  utils_image.py:650-697   (11x11 Gaussian sigma 1.5, 'valid' window; cv2.filter2D is
                a correlation whose border never enters the valid region, restated with numpy)
rgb2ycbcr / bgr2ycbcr / ycbcr2rgb  utils_image.py:536-602 (MATLAB coefficients)
augment_img / augment_img_tensor4  utils_image.py:387-426 (the 8 flip/rot90 modes)
modcrop / shave utils_image.py:501-531
imread_uint / imsave  utils_image.py:192-221 (PIL instead of cv2: cv2 is not in this image;
                grayscale is ITU-R 601-2 luma in both)
tensor2uint     utils_image.py:296-300
single2uint     utils_image.py:261-263
uint2tensor3/4  utils_image.py:281-292
imresize        utils_image.py:938-1005  MATLAB bicubic (a = -0.5, antialias when shrinking,
                symmetric border).  Written as two separable resampling-matrix products so it runs
                batched on the device (the data-synthesis step feeding the hot path).
"""
import math
import os

import numpy as np
import torch

IMG_EXTENSIONS = [".jpg", ".JPG", ".jpeg", ".JPEG", ".png", ".PNG", ".ppm", ".PPM", ".bmp", ".BMP", ".tif"]


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


def bicubic_taps(n_in, n_out, scale, antialias=True):
    """calculate_weights_indices (utils_image.py:880-932) in the reference's float32 arithmetic, as
    per-output-pixel taps: (indices int32 [n_out, P] with the symmetric border already reflected,
    weights fp32 [n_out, P]).  Zero-weight border taps are kept (they add 0)."""
    kw = 4.0 / scale if (scale < 1 and antialias) else 4.0
    x = torch.linspace(1, n_out, n_out)
    u = x / scale + 0.5 * (1 - 1 / scale)
    left = torch.floor(u - kw / 2)
    P = math.ceil(kw) + 2
    idx = left.view(n_out, 1).expand(n_out, P) + torch.linspace(0, P - 1, P).view(1, P).expand(n_out, P)
    d = u.view(n_out, 1).expand(n_out, P) - idx
    w = (scale * _cubic(d * scale)) if (scale < 1 and antialias) else _cubic(d)
    w = w / torch.sum(w, 1).view(n_out, 1)
    i = idx.long() - 1
    i = torch.where(i < 0, -i - 1, i)
    i = torch.where(i >= n_in, 2 * n_in - 1 - i, i)
    return i.int().contiguous(), w.float().contiguous()


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


# ------------------------------------------------------------------------------------------
# files
# ------------------------------------------------------------------------------------------
def is_image_file(filename):
    return any(filename.endswith(ext) for ext in IMG_EXTENSIONS)


def get_image_paths(dataroot):
    """utils_image.py:70-91: sorted image files under a directory (or a list of directories)."""
    if dataroot is None:
        return None
    roots = [dataroot] if isinstance(dataroot, str) else list(dataroot)
    paths = []
    for root in roots:
        if not os.path.isdir(root):
            raise AssertionError(f"{root} is not a valid directory")
        found = [os.path.join(d, f) for d, _, fs in sorted(os.walk(root)) for f in sorted(fs) if is_image_file(f)]
        if not found:
            raise AssertionError(f"{root} has no valid image file")
        paths += sorted(found)
    return paths


def imread_uint(path, n_channels=3):
    """HxWx3 RGB (or GGG) / HxWx1 gray uint8."""
    from PIL import Image
    im = Image.open(path)
    if n_channels == 1:
        return np.expand_dims(np.asarray(im.convert("L")), axis=2)
    return np.asarray(im.convert("RGB"))


def imsave(img, img_path):
    from PIL import Image
    Image.fromarray(np.squeeze(img)).save(img_path)


# ------------------------------------------------------------------------------------------
# layout / augmentation
# ------------------------------------------------------------------------------------------
def single2tensor3(img):
    return torch.from_numpy(np.ascontiguousarray(img)).permute(2, 0, 1).float()


def tensor2single(img):
    img = img.detach().squeeze().float().cpu().numpy()
    return np.transpose(img, (1, 2, 0)) if img.ndim == 3 else img


def augment_img(img, mode=0):
    """numpy HxW[xC]: the 8 dihedral modes of utils_image.py:387-405."""
    if mode == 0:
        return img
    if mode == 1:
        return np.flipud(np.rot90(img))
    if mode == 2:
        return np.flipud(img)
    if mode == 3:
        return np.rot90(img, k=3)
    if mode == 4:
        return np.flipud(np.rot90(img, k=2))
    if mode == 5:
        return np.rot90(img)
    if mode == 6:
        return np.rot90(img, k=2)
    if mode == 7:
        return np.flipud(np.rot90(img, k=3))
    raise ValueError(mode)


def augment_img_tensor4(img, mode=0):
    """NCHW tensor, utils_image.py:408-426."""
    if mode == 0:
        return img
    if mode == 1:
        return img.rot90(1, [2, 3]).flip([2])
    if mode == 2:
        return img.flip([2])
    if mode == 3:
        return img.rot90(3, [2, 3])
    if mode == 4:
        return img.rot90(2, [2, 3]).flip([2])
    if mode == 5:
        return img.rot90(1, [2, 3])
    if mode == 6:
        return img.rot90(2, [2, 3])
    if mode == 7:
        return img.rot90(3, [2, 3]).flip([2])
    raise ValueError(mode)


def modcrop(img_in, scale):
    img = np.copy(img_in)
    if img.ndim not in (2, 3):
        raise ValueError("Wrong img ndim: [{:d}].".format(img.ndim))
    H, W = img.shape[:2]
    return img[:H - H % scale, :W - W % scale, ...]


def shave(img_in, border=0):
    img = np.copy(img_in)
    h, w = img.shape[:2]
    return img[border:h - border, border:w - border]


# ------------------------------------------------------------------------------------------
# colour (MATLAB rgb2ycbcr coefficients)
# ------------------------------------------------------------------------------------------
_YCC = np.array([[65.481, -37.797, 112.0], [128.553, -74.203, -93.786], [24.966, 112.0, -18.214]])


def _ycbcr(img, only_y, coef):
    in_type = img.dtype
    x = img.astype(np.float64) if in_type == np.uint8 else img.astype(np.float64) * 255.0
    if only_y:
        rlt = np.dot(x, coef[:, 0]) / 255.0 + 16.0
    else:
        rlt = np.matmul(x, coef) / 255.0 + [16, 128, 128]
    rlt = rlt.round() if in_type == np.uint8 else rlt / 255.0
    return rlt.astype(in_type)


def rgb2ycbcr(img, only_y=True):
    return _ycbcr(img, only_y, _YCC)


def bgr2ycbcr(img, only_y=True):
    return _ycbcr(img, only_y, _YCC[::-1])


def ycbcr2rgb(img):
    in_type = img.dtype
    x = img.astype(np.float64) if in_type == np.uint8 else img.astype(np.float64) * 255.0
    rlt = np.matmul(x, [[0.00456621, 0.00456621, 0.00456621], [0, -0.00153632, 0.00791071],
                        [0.00625893, -0.00318811, 0]]) * 255.0 + [-222.921, 135.576, -276.836]
    rlt = np.clip(rlt, 0, 255)
    rlt = rlt.round() if in_type == np.uint8 else rlt / 255.0
    return rlt.astype(in_type)


# ------------------------------------------------------------------------------------------
# SSIM
# ------------------------------------------------------------------------------------------
def _gauss_window(k=11, sigma=1.5):
    x = np.arange(k, dtype=np.float64) - (k - 1) / 2
    g = np.exp(-x * x / (2 * sigma * sigma))
    g /= g.sum()
    return np.outer(g, g)


def _filter_valid(img, win):
    """correlation of img with win over the fully-overlapping region (cv2.filter2D(...)[5:-5, 5:-5])."""
    k = win.shape[0]
    from numpy.lib.stride_tricks import sliding_window_view
    v = sliding_window_view(img, (k, k))
    return np.einsum("ijkl,kl->ij", v, win)


def ssim(img1, img2):
    C1, C2 = (0.01 * 255) ** 2, (0.03 * 255) ** 2
    a, b = img1.astype(np.float64), img2.astype(np.float64)
    w = _gauss_window()
    mu1, mu2 = _filter_valid(a, w), _filter_valid(b, w)
    mu1_sq, mu2_sq, mu12 = mu1 ** 2, mu2 ** 2, mu1 * mu2
    s1 = _filter_valid(a * a, w) - mu1_sq
    s2 = _filter_valid(b * b, w) - mu2_sq
    s12 = _filter_valid(a * b, w) - mu12
    m = ((2 * mu12 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    return m.mean()


def calculate_ssim(img1, img2, border=0):
    if img1.shape != img2.shape:
        raise ValueError("Input images must have the same dimensions.")
    h, w = img1.shape[:2]
    a, b = img1[border:h - border, border:w - border], img2[border:h - border, border:w - border]
    if a.ndim == 2:
        return ssim(a, b)
    if a.ndim == 3:
        if a.shape[2] in (2, 3):
            return np.array([ssim(a[:, :, i], b[:, :, i]) for i in range(a.shape[2])]).mean()
        if a.shape[2] == 1:
            return ssim(np.squeeze(a), np.squeeze(b))
    raise ValueError("Wrong input image dimensions.")
