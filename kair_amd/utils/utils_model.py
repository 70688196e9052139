"""Full-image inference helpers (restatement of /root/reference/utils/utils_model.py:51-230 and the
tiling / padding of /root/reference/main_test_swinir.py:66-72, 256-284), SURVEY §8f rank 4.

test_mode(model, L, mode, refield, min_size, sf, modulo)   utils_model.py:51-89
    0 plain, 1 replicate-pad to `modulo`, 2 recursive 4-way split, 3 x8 self-ensemble,
    4 split + x8
pad_to_window(L, window_size)   main_test_swinir.py:66-72 (mirror pad to the next multiple + 1 window)
test_tiled(model, L, tile, tile_overlap, sf, window_size, tile_batch)   main_test_swinir.py:256-284
    overlapping tiles blended by their coverage count.  MI355X: the tiles of one image are run as
    batches of `tile_batch` (one forward per batch instead of one per tile); every network on
    this path is per-sample independent, so the blend is the reference's.

The model is any callable NCHW -> NCHW (the define_G networks); no_grad is the caller's business,
as in the reference.
"""
import math

import torch

from . import utils_image as util


def test_mode(model, L, mode=0, refield=32, min_size=256, sf=1, modulo=1):
    if mode == 0:
        return test(model, L)
    if mode == 1:
        return test_pad(model, L, modulo, sf)
    if mode == 2:
        return test_split(model, L, refield, min_size, sf, modulo)
    if mode == 3:
        return test_x8(model, L, modulo, sf)
    if mode == 4:
        return test_split_x8(model, L, refield, min_size, sf, modulo)
    raise ValueError(f"test_mode: mode {mode}")


def test(model, L):
    return model(L)


def test_pad(model, L, modulo=16, sf=1):
    h, w = L.shape[-2:]
    pb, pr = int(math.ceil(h / modulo) * modulo - h), int(math.ceil(w / modulo) * modulo - w)
    E = model(torch.nn.functional.pad(L, (0, pr, 0, pb), mode="replicate") if (pb or pr) else L)
    return E[..., :h * sf, :w * sf]


def test_split_fn(model, L, refield=32, min_size=256, sf=1, modulo=1):
    h, w = L.shape[-2:]
    if h * w <= min_size ** 2:
        return test_pad(model, L, modulo, sf)
    th, tw = (h // 2 // refield + 1) * refield, (w // 2 // refield + 1) * refield
    top, bottom = slice(0, th), slice(h - th, h)
    left, right = slice(0, tw), slice(w - tw, w)
    Ls = [L[..., top, left], L[..., top, right], L[..., bottom, left], L[..., bottom, right]]
    if h * w <= 4 * min_size ** 2:
        Es = [model(x) for x in Ls]
    else:
        Es = [test_split_fn(model, x, refield, min_size, sf, modulo) for x in Ls]
    b, c = Es[0].shape[:2]
    E = torch.zeros(b, c, sf * h, sf * w, dtype=L.dtype, device=L.device)
    h2, w2 = h // 2 * sf, w // 2 * sf
    E[..., :h2, :w2] = Es[0][..., :h2, :w2]
    E[..., :h2, w2:w * sf] = Es[1][..., :h2, (-w + w // 2) * sf:]
    E[..., h2:h * sf, :w2] = Es[2][..., (-h + h // 2) * sf:, :w2]
    E[..., h2:h * sf, w2:w * sf] = Es[3][..., (-h + h // 2) * sf:, (-w + w // 2) * sf:]
    return E


def test_split(model, L, refield=32, min_size=256, sf=1, modulo=1):
    return test_split_fn(model, L, refield, min_size, sf, modulo)


def _unaugment(E, i):
    return util.augment_img_tensor4(E, mode=8 - i if i in (3, 5) else i)


def test_x8(model, L, modulo=1, sf=1):
    Es = [_unaugment(test_pad(model, util.augment_img_tensor4(L, mode=i), modulo, sf), i) for i in range(8)]
    return torch.stack(Es, 0).mean(0)


def test_split_x8(model, L, refield=32, min_size=256, sf=1, modulo=1):
    Es = [_unaugment(test_split_fn(model, util.augment_img_tensor4(L, mode=i), refield, min_size, sf, modulo), i)
          for i in range(8)]
    return torch.stack(Es, 0).mean(0)


def pad_to_window(L, window_size):
    """main_test_swinir.py:66-72: mirror-extend to (h // ws + 1) * ws (always at least one row)."""
    h, w = L.shape[-2:]
    hp = (h // window_size + 1) * window_size - h
    wp = (w // window_size + 1) * window_size - w
    L = torch.cat([L, torch.flip(L, [2])], 2)[:, :, :h + hp, :]
    return torch.cat([L, torch.flip(L, [3])], 3)[:, :, :, :w + wp]


def test_tiled(model, L, tile=None, tile_overlap=32, sf=1, window_size=8, tile_batch=16):
    if tile is None:
        return model(L)
    b, c, h, w = L.shape
    tile = min(tile, h, w)
    if tile % window_size:
        raise AssertionError("tile size should be a multiple of window_size")
    stride = tile - tile_overlap
    hs = list(range(0, h - tile, stride)) + [h - tile]
    ws = list(range(0, w - tile, stride)) + [w - tile]
    pos = [(y, x) for y in hs for x in ws]
    E = W = None
    for i in range(0, len(pos), tile_batch):
        chunk = pos[i:i + tile_batch]
        batch = torch.cat([L[..., y:y + tile, x:x + tile] for y, x in chunk], 0)
        out = model(batch)
        if E is None:
            E = torch.zeros(b, out.shape[1], h * sf, w * sf, dtype=out.dtype, device=out.device)
            W = torch.zeros_like(E)
        for j, (y, x) in enumerate(chunk):
            E[..., y * sf:(y + tile) * sf, x * sf:(x + tile) * sf].add_(out[j * b:(j + 1) * b])
            W[..., y * sf:(y + tile) * sf, x * sf:(x + tile) * sf].add_(1.0)
    return E.div_(W)


def find_last_checkpoint(save_dir, net_type="G", pretrained_path=None):
    from .utils_option import find_last_checkpoint as f
    return f(save_dir, net_type, pretrained_path)
