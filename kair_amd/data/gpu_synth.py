"""HBM-resident training-patch synthesis: DatasetSR / DatasetDnCNN batches made
by one HIP launch from an image pool on the device, so 8 GPUs are not fed by Python loaders.

    synth = PatchSynth(pool, task="sr", scale=4, H_size=192, seed=0)    # pool [N, C, Hs, Ws] fp32 [0, 1]
    L, H = synth.next(32)                                               # device tensors, NCHW

Sampling follows the reference loaders: the image order is a seeded shuffled epoch
(DataLoader(shuffle=True), main_train_psnr.py:122-130; with `rank`/`world` the DistributedSampler's
rank-strided slice of it), then per sample random.randint for the crop rows / columns and the
augment mode in the order __getitem__ draws them (data/dataset_sr.py:78-91,
data/dataset_dncnn.py:59-66).  The per-sample geometry is drawn on the host (a few ints), the
pixels are produced on the device (kair_synth_sr / kair_synth_dn in csrc/synth.hip).
"""
import random

import torch

from .. import _hip as H
from ..utils import utils_image as util


class PatchSynth:
    def __init__(self, pool, task="sr", scale=4, H_size=96, sigma=25, seed=0, rank=0, world=1):
        if pool.dim() != 4 or not pool.is_cuda:
            raise ValueError("PatchSynth: pool must be a device tensor [N, C, Hs, Ws]")
        self.task = task
        self.sf = scale if task == "sr" else 1
        Hs, Ws = pool.shape[-2:]
        if task == "sr":   # modcrop (dataset_sr.py:51)
            pool = pool[..., :Hs - Hs % self.sf, :Ws - Ws % self.sf]
        self.pool = pool.float().contiguous()
        self.N, self.C, self.Hs, self.Ws = self.pool.shape
        self.PS = H_size
        if self.PS > min(self.Hs, self.Ws):
            raise ValueError("PatchSynth: H_size larger than the pool images")
        self.sigma = sigma / 255.0
        self.seed = seed
        self.rng = random.Random(seed)
        self.rank, self.world = rank, world
        self.epoch, self.order, self.pos = 0, [], 0
        self.step = 0
        dev = self.pool.device
        if task == "sr":
            ih, wh = util.bicubic_taps(self.Hs, self.Hs // self.sf, 1.0 / self.sf)
            iw, ww = util.bicubic_taps(self.Ws, self.Ws // self.sf, 1.0 / self.sf)
            self.taps_h = (ih.to(dev), wh.to(dev))
            self.taps_w = (iw.to(dev), ww.to(dev))
        elif task != "dn":
            raise ValueError(task)
        self._par_host = None
        self._par_ev = None

    def _next_index(self):
        if self.pos >= len(self.order):
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            perm = torch.randperm(self.N, generator=g).tolist()
            self.order = perm[self.rank::self.world] if self.world > 1 else perm
            self.epoch += 1
            self.pos = 0
        i = self.order[self.pos]
        self.pos += 1
        return i

    def draw(self, B):
        """Host-side geometry of the next batch: [B, 4] int32 {image, rnd_h, rnd_w, mode}."""
        rows = []
        ls = self.PS // self.sf
        hl, wl = self.Hs // self.sf, self.Ws // self.sf
        for _ in range(B):
            img = self._next_index()
            rh = self.rng.randint(0, max(0, hl - ls))
            rw = self.rng.randint(0, max(0, wl - ls))
            mode = self.rng.randint(0, 7)
            rows.append((img, rh, rw, mode))
        return torch.tensor(rows, dtype=torch.int32)

    def next(self, B, out=None):
        """The next batch (L, H), produced on the current stream.  The per-sample geometry goes up
        through a pinned staging buffer with an async copy, so a training loop that calls next()
        every step never blocks the host on the device."""
        dev = self.pool.device
        host = self.draw(B)
        if self._par_host is None or self._par_host.shape[0] < B:
            self._par_host = torch.empty(B, 4, dtype=torch.int32).pin_memory()
            self._par_ev = None
        if self._par_ev is not None:
            self._par_ev.synchronize()   # the previous batch's copy has read the staging buffer
        self._par_host[:B].copy_(host)
        par = self._par_host[:B].to(dev, non_blocking=True)
        self._par_ev = torch.cuda.Event()
        self._par_ev.record()
        ls = self.PS // self.sf
        if out is None:
            Hp = torch.empty(B, self.C, self.PS, self.PS, device=dev)
            Lp = torch.empty(B, self.C, ls, ls, device=dev)
        else:
            Lp, Hp = out
        if self.task == "sr":
            H.synth_sr(self.pool, par, B, self.PS, self.sf, self.taps_h, self.taps_w, Hp, Lp)
        else:
            H.synth_dn(self.pool, par, B, self.PS, self.sigma, self.seed, self.step, Hp, Lp)
        self.step += 1
        self.last_params = par
        return Lp, Hp


def synthetic_pool(N, C, Hs, Ws, seed=0, device="cuda"):
    """Seeded natural-ish images for the pool when no dataset is on the box (SURVEY §8d recipe:
    bicubic-upsampled uniform noise + 0.02 N, clamped to [0, 1])."""
    g = torch.Generator().manual_seed(seed)
    base = torch.rand(N, C, max(1, Hs // 8), max(1, Ws // 8), generator=g)
    img = torch.nn.functional.interpolate(base, size=(Hs, Ws), mode="bicubic", align_corners=False)
    img = (img + 0.02 * torch.randn(img.shape, generator=g)).clamp(0, 1)
    return img.to(device)
