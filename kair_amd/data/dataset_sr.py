"""DatasetSR (restatement of /root/reference/data/dataset_sr.py:17-105): bicubic SR pairs.

H: modcrop(sf) of the image (dataset_sr.py:51); L: read from dataroot_L, or MATLAB-bicubic x1/sf of
the WHOLE H image (66; the fork's imresize_np is broken, SURVEY §0 gotcha 5 -- the same maths runs
here through utils_image.imresize).  train: random L crop of H_size // sf and the aligned H crop
(71-86), one of the 8 flip/rot modes on both (91-92).

kair_amd.data.gpu_synth.PatchSynth produces the same pairs from an HBM-resident image pool with
one HIP kernel per batch.
"""
import random

import numpy as np
import torch
import torch.utils.data as data

from ..utils import utils_image as util


class DatasetSR(data.Dataset):
    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        self.n_channels = opt.get("n_channels") or 3
        self.sf = opt.get("scale") or 4
        self.patch_size = opt.get("H_size") or 96
        self.L_size = self.patch_size // self.sf
        self.paths_H = util.get_image_paths(opt["dataroot_H"])
        self.paths_L = util.get_image_paths(opt.get("dataroot_L"))
        assert self.paths_H, "Error: H path is empty."
        if self.paths_L and self.paths_H:
            assert len(self.paths_L) == len(self.paths_H), f"L/H mismatch - {len(self.paths_L)}, {len(self.paths_H)}."

    def __getitem__(self, index):
        H_path = self.paths_H[index]
        img_H = util.modcrop(util.uint2single(util.imread_uint(H_path, self.n_channels)), self.sf)
        L_path = None
        if self.paths_L:
            L_path = self.paths_L[index]
            img_L = util.uint2single(util.imread_uint(L_path, self.n_channels))
        else:
            t = torch.from_numpy(np.ascontiguousarray(img_H)).permute(2, 0, 1)
            img_L = util.imresize(t, 1 / self.sf, True).permute(1, 2, 0).numpy()
        if self.opt["phase"] == "train":
            H, W, _ = img_L.shape
            rnd_h = random.randint(0, max(0, H - self.L_size))
            rnd_w = random.randint(0, max(0, W - self.L_size))
            img_L = img_L[rnd_h:rnd_h + self.L_size, rnd_w:rnd_w + self.L_size, :]
            rh, rw = int(rnd_h * self.sf), int(rnd_w * self.sf)
            img_H = img_H[rh:rh + self.patch_size, rw:rw + self.patch_size, :]
            mode = random.randint(0, 7)
            img_L, img_H = util.augment_img(img_L, mode=mode), util.augment_img(img_H, mode=mode)
        img_H, img_L = util.single2tensor3(img_H), util.single2tensor3(img_L)
        return {"L": img_L, "H": img_H, "L_path": L_path or H_path, "H_path": H_path}

    def __len__(self):
        return len(self.paths_H)
