"""DnCNN / FDnCNN — module trees of /root/reference/models/network_dncnn.py:40-71 / 128-149.

`model` is the flattened Sequential basicblock.sequential builds (basicblock.py:61-98): conv,
act, [conv, BatchNorm2d(momentum 0.9, eps 1e-4), act] x (nb-2), conv — so state_dict keys
(model.0.weight, model.3.running_mean, ...) match the reference.

`forward` on a HIP tensor runs the whole network as one autograd node on the HIP step program
(kair_amd/engine/dncnn_engine.py); it raises if libkair_hip.so is missing.  On a CPU tensor it
runs the module list itself: that is BASELINE config 1 ("DnCNN sigma=25, main_train_dncnn.py on
CPU, plumbing, no GPU"), the one configuration the reference specifies for the host -- never a
substitute for a device call.
"""
import torch
import torch.nn as nn

from ..engine.dncnn_engine import DnCNNEngine
from ..engine.rrdbnet_engine import ConvNetFunction


def _act(a, slope=0.2):
    if a in "Rr":
        return nn.ReLU(inplace=a == "R")
    if a in "Ll":
        return nn.LeakyReLU(negative_slope=slope, inplace=a == "L")
    raise NotImplementedError(f"kair_amd DnCNN: activation {a!r}")


def _layers(in_nc, out_nc, nc, nb, act_mode):
    if "R" not in act_mode and "L" not in act_mode:
        raise AssertionError("Examples of activation function: R, L, BR, BL, IR, IL")
    if "I" in act_mode:
        raise NotImplementedError("kair_amd DnCNN: InstanceNorm ('I') is not on the MI355X path")
    act = act_mode[-1]
    mods = [nn.Conv2d(in_nc, nc, 3, 1, 1, bias=True), _act(act)]
    for _ in range(nb - 2):
        mods.append(nn.Conv2d(nc, nc, 3, 1, 1, bias=True))
        if "B" in act_mode:
            mods.append(nn.BatchNorm2d(nc, momentum=0.9, eps=1e-4, affine=True))
        mods.append(_act(act))
    mods.append(nn.Conv2d(nc, out_nc, 3, 1, 1, bias=True))
    return nn.Sequential(*mods)


class _Base(nn.Module):
    residual = True

    def __init__(self, in_nc, out_nc, nc, nb, act_mode, compute_dtype):
        super().__init__()
        self.model = _layers(in_nc, out_nc, nc, nb, act_mode)
        self.compute_dtype = compute_dtype
        self._engine = None

    def engine(self):
        if self._engine is None or self._engine.net_ref() is not self:
            self._engine = DnCNNEngine(self, self.compute_dtype, residual=self.residual)
        return self._engine

    def invalidate_engine(self):
        """The module list changed (utils_bnorm.merge_bn / tidy_sequential): rebuild on next use."""
        self._engine = None

    def _apply(self, fn, *args, **kwargs):
        self._engine = None
        return super()._apply(fn, *args, **kwargs)

    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        self._engine = None
        return self

    def forward(self, x):
        if x.is_cuda:
            return ConvNetFunction.run(self.engine(), x, list(self.parameters()))
        if next(self.parameters()).is_cuda:
            raise RuntimeError("kair_amd DnCNN: CPU input for a network on the HIP device")
        n = self.model(x)                                   # config 1: host execution (network_dncnn.py:69-71)
        return x - n if self.residual else n


class DnCNN(_Base):
    """network_dncnn.py:40-71: out = x - model(x)."""

    def __init__(self, in_nc=1, out_nc=1, nc=64, nb=17, act_mode="BR", compute_dtype="fp32"):
        super().__init__(in_nc, out_nc, nc, nb, act_mode, compute_dtype)


class FDnCNN(_Base):
    """network_dncnn.py:128-149: out = model(x) (x carries the noise-level map channel)."""
    residual = False

    def __init__(self, in_nc=2, out_nc=1, nc=64, nb=20, act_mode="R", compute_dtype="fp32"):
        super().__init__(in_nc, out_nc, nc, nb, act_mode, compute_dtype)
