"""USRNet — module tree of /root/reference/models/network_usrnet.py:191-344 (the class define_G
binds, select_network.py:167-178) with the maths of its torch.fft restatement
network_usrnet_v1.py:109-262 (the legacy file calls torch.rfft, removed in torch 1.8; SURVEY.md §0
gotcha 3).

Same submodule names and parameter shapes (p.* ResUNet, h.* HyPaNet; DataNet has no parameters), so
`state_dict` and checkpoints interchange with the reference.  `forward(x, k, sf, sigma)` runs the
whole unfolded network as one autograd node on the HIP step program
(kair_amd/engine/usrnet_engine.py); there is no CPU path.
"""
import torch.nn as nn

from ..engine.usrnet_engine import USRNetEngine, USRNetFunction


class ResBlock(nn.Module):
    """basicblock.ResBlock (basicblock.py:211-223), mode 'C' + act + 'C', no bias: x + res(x)."""

    def __init__(self, c, act_mode="R"):
        super().__init__()
        if act_mode != "R":
            raise NotImplementedError("kair_amd USRNet: act_mode 'R' only (options/train_usrnet.json)")
        self.res = nn.Sequential(nn.Conv2d(c, c, 3, 1, 1, bias=False), nn.ReLU(inplace=True),
                                 nn.Conv2d(c, c, 3, 1, 1, bias=False))


def _seq(*mods):
    """basicblock.sequential (basicblock.py:15-35): a single module is returned as it is."""
    return mods[0] if len(mods) == 1 else nn.Sequential(*mods)


class ResUNet(nn.Module):
    """network_usrnet_v1.py:109-145 with strideconv down / convtranspose up, no bias."""

    def __init__(self, in_nc=4, out_nc=3, nc=(64, 128, 256, 512), nb=2, act_mode="R", downsample_mode="strideconv",
                 upsample_mode="convtranspose"):
        super().__init__()
        if downsample_mode != "strideconv" or upsample_mode != "convtranspose":
            raise NotImplementedError("kair_amd USRNet: strideconv / convtranspose only (options/train_usrnet.json)")
        if nb < 1:
            raise NotImplementedError("kair_amd USRNet: nb >= 1")
        rb = lambda c: [ResBlock(c, act_mode) for _ in range(nb)]   # noqa: E731
        self.m_head = nn.Conv2d(in_nc, nc[0], 3, 1, 1, bias=False)
        self.m_down1 = _seq(*rb(nc[0]), nn.Conv2d(nc[0], nc[1], 2, 2, 0, bias=False))
        self.m_down2 = _seq(*rb(nc[1]), nn.Conv2d(nc[1], nc[2], 2, 2, 0, bias=False))
        self.m_down3 = _seq(*rb(nc[2]), nn.Conv2d(nc[2], nc[3], 2, 2, 0, bias=False))
        self.m_body = _seq(*rb(nc[3]))
        self.m_up3 = _seq(nn.ConvTranspose2d(nc[3], nc[2], 2, 2, 0, bias=False), *rb(nc[2]))
        self.m_up2 = _seq(nn.ConvTranspose2d(nc[2], nc[1], 2, 2, 0, bias=False), *rb(nc[1]))
        self.m_up1 = _seq(nn.ConvTranspose2d(nc[1], nc[0], 2, 2, 0, bias=False), *rb(nc[0]))
        self.m_tail = nn.Conv2d(nc[0], out_nc, 3, 1, 1, bias=False)


class DataNet(nn.Module):
    """network_usrnet_v1.py:179-194: parameter-free closed form; runs inside the engine
    (kair_usr_fft_rows / _cols / _ifft_rows)."""


class HyPaNet(nn.Module):
    """network_usrnet_v1.py:204-216."""

    def __init__(self, in_nc=2, out_nc=8, channel=64):
        super().__init__()
        self.mlp = nn.Sequential(nn.Conv2d(in_nc, channel, 1, padding=0, bias=True), nn.ReLU(inplace=True),
                                 nn.Conv2d(channel, channel, 1, padding=0, bias=True), nn.ReLU(inplace=True),
                                 nn.Conv2d(channel, out_nc, 1, padding=0, bias=True), nn.Softplus())


class USRNet(nn.Module):
    """network_usrnet_v1.py:228-262 (same constructor signature; compute_dtype is the engine option:
    'bf16' MFMA operands with fp32 accumulation, or 'fp32' exact-MFMA parity mode)."""

    def __init__(self, n_iter=8, h_nc=64, in_nc=4, out_nc=3, nc=(64, 128, 256, 512), nb=2, act_mode="R",
                 downsample_mode="strideconv", upsample_mode="convtranspose", compute_dtype="fp32"):
        super().__init__()
        self.d = DataNet()
        self.p = ResUNet(in_nc=in_nc, out_nc=out_nc, nc=nc, nb=nb, act_mode=act_mode, downsample_mode=downsample_mode,
                         upsample_mode=upsample_mode)
        self.h = HyPaNet(in_nc=2, out_nc=n_iter * 2, channel=h_nc)
        self.n = n_iter
        self.compute_dtype = compute_dtype
        self._engine = None

    def engine(self):
        if self._engine is None or self._engine.net_ref() is not self:
            self._engine = USRNetEngine(self, self.compute_dtype)
        return self._engine

    def _apply(self, fn, *args, **kwargs):
        self._engine = None
        return super()._apply(fn, *args, **kwargs)

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        self._engine = None
        return self

    def forward(self, x, k, sf, sigma):
        if not x.is_cuda:
            raise RuntimeError("kair_amd USRNet runs on the MI355X (HIP) only; got a CPU tensor (no CPU fallback)")
        return USRNetFunction.run(self.engine(), x, k, int(sf), sigma, list(self.parameters()))
