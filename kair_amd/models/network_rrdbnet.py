"""RRDBNet (ESRGAN generator) — module tree of /root/reference/models/network_rrdbnet.py:35-157.

Same submodule names, parameter shapes and initialisation (ResidualDenseBlock_5C convs:
kaiming-normal fan_in x 0.1, zero bias, network_rrdbnet.py:8-25/49; the rest torch defaults), so
`state_dict` and checkpoints interchange with the reference (702 keys at nb=23).  `forward` runs
the whole network as one autograd node on the HIP step program
(kair_amd/engine/rrdbnet_engine.py); there is no CPU path.
"""
import functools

import torch
import torch.nn as nn
import torch.nn.init as init

from ..engine.rrdbnet_engine import RRDBNetEngine, ConvNetFunction


def initialize_weights(net_l, scale=1):
    """network_rrdbnet.py:8-25."""
    if not isinstance(net_l, list):
        net_l = [net_l]
    for net in net_l:
        for m in net.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                init.kaiming_normal_(m.weight, a=0, mode="fan_in")
                m.weight.data *= scale
                if m.bias is not None:
                    m.bias.data.zero_()
            elif isinstance(m, nn.BatchNorm2d):
                init.constant_(m.weight, 1)
                init.constant_(m.bias.data, 0.0)


class ResidualDenseBlock_5C(nn.Module):
    """network_rrdbnet.py:35-58: five 3x3 convs over the growing concatenation, LeakyReLU 0.2,
    out = 0.2 * conv5 + x."""

    def __init__(self, nf=64, gc=32, bias=True):
        super().__init__()
        self.conv1 = nn.Conv2d(nf, gc, 3, 1, 1, bias=bias)
        self.conv2 = nn.Conv2d(nf + gc, gc, 3, 1, 1, bias=bias)
        self.conv3 = nn.Conv2d(nf + 2 * gc, gc, 3, 1, 1, bias=bias)
        self.conv4 = nn.Conv2d(nf + 3 * gc, gc, 3, 1, 1, bias=bias)
        self.conv5 = nn.Conv2d(nf + 4 * gc, nf, 3, 1, 1, bias=bias)
        self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)
        initialize_weights([self.conv1, self.conv2, self.conv3, self.conv4, self.conv5], 0.1)


class RRDB(nn.Module):
    """network_rrdbnet.py:61-75: three RDBs, out = 0.2 * RDB3(RDB2(RDB1(x))) + x."""

    def __init__(self, nf, gc=32):
        super().__init__()
        self.RDB1 = ResidualDenseBlock_5C(nf, gc)
        self.RDB2 = ResidualDenseBlock_5C(nf, gc)
        self.RDB3 = ResidualDenseBlock_5C(nf, gc)


def make_layer(block, n_layers):
    return nn.Sequential(*[block() for _ in range(n_layers)])


class RRDBNet(nn.Module):
    """network_rrdbnet.py:78-119."""

    def __init__(self, in_nc=3, out_nc=3, nf=64, nb=23, gc=32, sf=4, compute_dtype="fp32"):
        super().__init__()
        self.sf = sf
        self.conv_first = nn.Conv2d(in_nc, nf, 3, 1, 1, bias=True)
        self.RRDB_trunk = make_layer(functools.partial(RRDB, nf=nf, gc=gc), nb)
        self.trunk_conv = nn.Conv2d(nf, nf, 3, 1, 1, bias=True)
        self.upconv1 = nn.Conv2d(nf, nf, 3, 1, 1, bias=True)
        if self.sf == 4:
            self.upconv2 = nn.Conv2d(nf, nf, 3, 1, 1, bias=True)
        self.HRconv = nn.Conv2d(nf, nf, 3, 1, 1, bias=True)
        self.conv_last = nn.Conv2d(nf, out_nc, 3, 1, 1, bias=True)
        self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)
        self.compute_dtype = compute_dtype
        self._engine = None

    def engine(self):
        if self._engine is None or self._engine.net_ref() is not self:
            self._engine = RRDBNetEngine(self, self.compute_dtype)
        return self._engine

    def _apply(self, fn, *args, **kwargs):
        self._engine = None
        return super()._apply(fn, *args, **kwargs)

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        self._engine = None
        return self

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("kair_amd RRDBNet runs on the MI355X (HIP) only; got a CPU tensor (no CPU fallback)")
        return ConvNetFunction.run(self.engine(), x, list(self.parameters()))
