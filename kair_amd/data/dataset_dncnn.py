"""DatasetDnCNN (restatement of /root/reference/data/dataset_dncnn.py:19-101): AWGN denoising pairs.

train: random 'H_size' crop (dataset_dncnn.py:59-61), one of the 8 flip/rot modes (66-67),
       L = H + N(0, 1) * sigma / 255 from torch's global RNG (74-75);
test:  whole image, L = H + numpy N(0, sigma_test / 255) after np.random.seed(0) (88-90).

The GPU-resident equivalent that feeds the fused trainer without a host loader is
kair_amd.data.gpu_synth.PatchSynth (HIP kernel).
"""
import random

import numpy as np
import torch
import torch.utils.data as data

from ..utils import utils_image as util


class DatasetDnCNN(data.Dataset):
    def __init__(self, opt):
        super().__init__()
        self.opt = opt
        self.n_channels = opt.get("n_channels") or 3
        self.patch_size = opt.get("H_size") or 64
        self.sigma = opt.get("sigma") or 25
        self.sigma_test = opt.get("sigma_test") or self.sigma
        self.paths_H = util.get_image_paths(opt["dataroot_H"])

    def __getitem__(self, index):
        H_path = self.paths_H[index]
        img_H = util.imread_uint(H_path, self.n_channels)
        if self.opt["phase"] == "train":
            H, W, _ = img_H.shape
            rnd_h = random.randint(0, max(0, H - self.patch_size))
            rnd_w = random.randint(0, max(0, W - self.patch_size))
            patch = img_H[rnd_h:rnd_h + self.patch_size, rnd_w:rnd_w + self.patch_size, :]
            patch = util.augment_img(patch, mode=random.randint(0, 7))
            img_H = util.uint2tensor3(patch)
            img_L = img_H.clone()
            img_L.add_(torch.randn(img_L.size()).mul_(self.sigma / 255.0))
        else:
            img_H = util.uint2single(img_H)
            img_L = np.copy(img_H)
            np.random.seed(seed=0)
            img_L += np.random.normal(0, self.sigma_test / 255.0, img_L.shape)
            img_L, img_H = util.single2tensor3(img_L), util.single2tensor3(img_H)
        return {"L": img_L, "H": img_H, "H_path": H_path, "L_path": H_path}

    def __len__(self):
        return len(self.paths_H)
