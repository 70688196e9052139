"""RRDB (option net_type 'rrdb') — module tree of /root/reference/models/network_rrdb.py:14-54.

basicblock.sequential flattening is reproduced so state_dict keys match the reference:
model.0 head conv; model.1 = ShortcutBlock(sub = [RRDB x nb, LR conv]) whose RDB convs 1-4 are
Sequential(conv, act) ('conv1.0.weight') and conv5 a bare conv (basicblock.py:393-409, gc fixed at
32 by network_rrdb.py:29); then per x2 stage Upsample + conv + act (upsample_upconv,
basicblock.py:455-465), then conv + act, conv.  Runs on the RRDB step program
(kair_amd/engine/rrdbnet_engine.py).
"""
import math

import torch.nn as nn

from ..engine.rrdbnet_engine import ConvNetFunction, RRDBNetEngine


def _act(a, slope=0.2):
    if a in "Rr":
        return nn.ReLU(inplace=a == "R")
    if a in "Ll":
        return nn.LeakyReLU(negative_slope=slope, inplace=a == "L")
    raise NotImplementedError(f"kair_amd RRDB: activation {a!r}")


class ResidualDenseBlock_5C(nn.Module):
    def __init__(self, nc=64, gc=32, act="R"):
        super().__init__()
        self.conv1 = nn.Sequential(nn.Conv2d(nc, gc, 3, 1, 1), _act(act))
        self.conv2 = nn.Sequential(nn.Conv2d(nc + gc, gc, 3, 1, 1), _act(act))
        self.conv3 = nn.Sequential(nn.Conv2d(nc + 2 * gc, gc, 3, 1, 1), _act(act))
        self.conv4 = nn.Sequential(nn.Conv2d(nc + 3 * gc, gc, 3, 1, 1), _act(act))
        self.conv5 = nn.Conv2d(nc + 4 * gc, nc, 3, 1, 1)


class RRDBBlock(nn.Module):
    def __init__(self, nc=64, gc=32, act="R"):
        super().__init__()
        self.RDB1 = ResidualDenseBlock_5C(nc, gc, act)
        self.RDB2 = ResidualDenseBlock_5C(nc, gc, act)
        self.RDB3 = ResidualDenseBlock_5C(nc, gc, act)


class ShortcutBlock(nn.Module):
    def __init__(self, submodule):
        super().__init__()
        self.sub = submodule


class RRDB(nn.Module):
    def __init__(self, in_nc=3, out_nc=3, nc=64, nb=23, gc=32, upscale=4, act_mode="L", upsample_mode="upconv",
                 compute_dtype="fp32"):
        super().__init__()
        if "R" not in act_mode and "L" not in act_mode:
            raise AssertionError("Examples of activation function: R, L, BR, BL, IR, IL")
        if upsample_mode != "upconv":
            raise NotImplementedError(f"kair_amd RRDB: upsample_mode {upsample_mode!r} (upconv only on the MI355X path)")
        if upscale not in (2, 4):
            raise NotImplementedError("kair_amd RRDB: upscale 2 or 4")
        if act_mode not in ("R", "L"):
            raise NotImplementedError("kair_amd RRDB: act_mode 'R' or 'L'")
        act = act_mode
        n_up = int(math.log(upscale, 2))
        body = [RRDBBlock(nc, 32, act) for _ in range(nb)]      # gc hard-coded 32 (network_rrdb.py:29)
        body.append(nn.Conv2d(nc, nc, 3, 1, 1))
        mods = [nn.Conv2d(in_nc, nc, 3, 1, 1), ShortcutBlock(nn.Sequential(*body))]
        for _ in range(n_up):
            mods += [nn.Upsample(scale_factor=2, mode="nearest"), nn.Conv2d(nc, nc, 3, 1, 1), _act(act)]
        mods += [nn.Conv2d(nc, nc, 3, 1, 1), _act(act), nn.Conv2d(nc, out_nc, 3, 1, 1)]
        self.model = nn.Sequential(*mods)
        self.compute_dtype = compute_dtype
        self._engine = None
        self._act = act

    def _spec(self):
        m = list(self.model)
        body = list(m[1].sub)
        ups = [mm for mm in m[2:-3] if isinstance(mm, nn.Conv2d)]
        return {"first": m[0], "rrdbs": [(b.RDB1, b.RDB2, b.RDB3) for b in body[:-1]],
                "rdb_convs": lambda d: [d.conv1[0], d.conv2[0], d.conv3[0], d.conv4[0], d.conv5], "trunk": body[-1],
                "up": ups, "hr": m[-3], "last": m[-1], "act": 1 if self._act == "R" else 2,
                "slope": 0.0 if self._act == "R" else 0.2}

    def engine(self):
        if self._engine is None or self._engine.net_ref() is not self:
            self._engine = RRDBNetEngine(self, self.compute_dtype, spec=self._spec())
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
            raise RuntimeError("kair_amd RRDB runs on the MI355X (HIP) only; got a CPU tensor (no CPU fallback)")
        return ConvNetFunction.run(self.engine(), x, list(self.parameters()))
