"""Oracle (test infrastructure only): fp32 CPU restatements of the conv networks on the path.

DnCNN      — /root/reference/models/network_dncnn.py:40-71 with basicblock.conv (basicblock.py:61-98)
RRDB       — /root/reference/models/network_rrdb.py:14-54 (option net_type 'rrdb'; gc hard-coded 32 :29)
RRDBNet    — /root/reference/models/network_rrdbnet.py:89-157 (option net_type 'rrdbnet')
USRNet     — /root/reference/models/network_usrnet_v1.py:33-262 (torch.fft maths; the option file
             binds network_usrnet.py whose torch.rfft API no longer exists — same parameters)
State-dict keys match the reference so golden weights load strictly.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def _bn(c):
    # basicblock.py:69 — momentum 0.9, eps 1e-4
    return nn.BatchNorm2d(c, momentum=0.9, eps=1e-4, affine=True)


class DnCNN(nn.Module):
    """network_dncnn.py:40-71: conv+act, (nb-2) x [conv(+BN)+act], conv;  out = x - model(x)."""

    def __init__(self, in_nc=1, out_nc=1, nc=64, nb=17, act_mode="BR"):
        super().__init__()
        act = act_mode[-1]
        mods = [nn.Conv2d(in_nc, nc, 3, 1, 1), _act(act)]
        for _ in range(nb - 2):
            mods.append(nn.Conv2d(nc, nc, 3, 1, 1))
            if "B" in act_mode:
                mods.append(_bn(nc))
            mods.append(_act(act))
        mods.append(nn.Conv2d(nc, out_nc, 3, 1, 1))
        self.model = nn.Sequential(*mods)

    def forward(self, x):
        return x - self.model(x)


def _act(a, slope=0.2):
    if a in "Rr":
        return nn.ReLU()
    if a in "Ll":
        return nn.LeakyReLU(slope)
    raise ValueError(a)


class _ConvAct(nn.Sequential):
    """basicblock.conv(mode='C'+act): Sequential(conv, act) — keys '<name>.0.weight'."""

    def __init__(self, cin, cout, act):
        super().__init__(nn.Conv2d(cin, cout, 3, 1, 1), _act(act))


class RDB5(nn.Module):
    """Residual dense block, 5 convs (basicblock.py:393-409 / network_rrdbnet.py:89-109)."""

    def __init__(self, nc, gc, act, seq_keys):
        super().__init__()
        mk = (lambda ci, co: _ConvAct(ci, co, act)) if seq_keys else (lambda ci, co: nn.Conv2d(ci, co, 3, 1, 1))
        self.conv1 = mk(nc, gc)
        self.conv2 = mk(nc + gc, gc)
        self.conv3 = mk(nc + 2 * gc, gc)
        self.conv4 = mk(nc + 3 * gc, gc)
        self.conv5 = nn.Conv2d(nc + 4 * gc, nc, 3, 1, 1)
        self.seq_keys = seq_keys
        self.act = _act(act)

    def forward(self, x):
        a = (lambda t: t) if self.seq_keys else self.act
        x1 = a(self.conv1(x))
        x2 = a(self.conv2(torch.cat((x, x1), 1)))
        x3 = a(self.conv3(torch.cat((x, x1, x2), 1)))
        x4 = a(self.conv4(torch.cat((x, x1, x2, x3), 1)))
        x5 = self.conv5(torch.cat((x, x1, x2, x3, x4), 1))
        return x5 * 0.2 + x


class RRDBlock(nn.Module):
    """basicblock.py:416-428 / network_rrdbnet.py:112-125."""

    def __init__(self, nc, gc, act, seq_keys):
        super().__init__()
        self.RDB1 = RDB5(nc, gc, act, seq_keys)
        self.RDB2 = RDB5(nc, gc, act, seq_keys)
        self.RDB3 = RDB5(nc, gc, act, seq_keys)

    def forward(self, x):
        return self.RDB3(self.RDB2(self.RDB1(x))) * 0.2 + x


class RRDBNet(nn.Module):
    """network_rrdbnet.py:128-157 (LeakyReLU 0.2 everywhere)."""

    def __init__(self, in_nc=3, out_nc=3, nf=64, nb=23, gc=32, sf=4):
        super().__init__()
        self.sf = sf
        self.conv_first = nn.Conv2d(in_nc, nf, 3, 1, 1)
        self.RRDB_trunk = nn.Sequential(*[RRDBlock(nf, gc, "L", False) for _ in range(nb)])
        self.trunk_conv = nn.Conv2d(nf, nf, 3, 1, 1)
        self.upconv1 = nn.Conv2d(nf, nf, 3, 1, 1)
        if sf == 4:
            self.upconv2 = nn.Conv2d(nf, nf, 3, 1, 1)
        self.HRconv = nn.Conv2d(nf, nf, 3, 1, 1)
        self.conv_last = nn.Conv2d(nf, out_nc, 3, 1, 1)

    def forward(self, x):
        lr = lambda t: F.leaky_relu(t, 0.2)
        fea = self.conv_first(x)
        fea = fea + self.trunk_conv(self.RRDB_trunk(fea))
        fea = lr(self.upconv1(F.interpolate(fea, scale_factor=2, mode="nearest")))
        if self.sf == 4:
            fea = lr(self.upconv2(F.interpolate(fea, scale_factor=2, mode="nearest")))
        return self.conv_last(lr(self.HRconv(fea)))


class _Shortcut(nn.Module):
    def __init__(self, sub):
        super().__init__()
        self.sub = sub

    def forward(self, x):
        return x + self.sub(x)


class _Up(nn.Sequential):
    """basicblock.upsample_upconv(mode='2'+act): Sequential(Upsample(nearest x2), conv, act)."""

    def __init__(self, nc, act):
        super().__init__(nn.Upsample(scale_factor=2, mode="nearest"), nn.Conv2d(nc, nc, 3, 1, 1), _act(act))


class RRDB(nn.Module):
    """network_rrdb.py:14-54 with upsample_mode 'upconv' (option train_rrdb_psnr.json)."""

    def __init__(self, in_nc=3, out_nc=3, nc=64, nb=23, gc=32, upscale=4, act_mode="R", upsample_mode="upconv"):
        super().__init__()
        assert upsample_mode == "upconv" and upscale in (2, 4)
        act = act_mode[-1]
        body = [RRDBlock(nc, 32, act, True) for _ in range(nb)] + [nn.Conv2d(nc, nc, 3, 1, 1)]
        mods = [nn.Conv2d(in_nc, nc, 3, 1, 1), _Shortcut(nn.Sequential(*body))]
        for _ in range(2 if upscale == 4 else 1):
            mods += list(_Up(nc, act).children())
        mods += [nn.Conv2d(nc, nc, 3, 1, 1), _act(act), nn.Conv2d(nc, out_nc, 3, 1, 1)]
        self.model = nn.Sequential(*mods)

    def forward(self, x):
        return self.model(x)


# ------------------------------------------------------------------------------------------
# USRNet (network_usrnet_v1.py)
# ------------------------------------------------------------------------------------------
def splits(a, sf):
    """v1:33-45 — (N,C,W,H) -> (N,C,W/sf,H/sf,sf*sf), block order as the reference."""
    b = torch.stack(torch.chunk(a, sf, dim=2), dim=4)
    return torch.cat(torch.chunk(b, sf, dim=3), dim=4)


def p2o(psf, shape):
    """v1:48-69 — PSF to OTF: zero-pad to shape, circularly centre, fft2."""
    otf = torch.zeros(psf.shape[:-2] + tuple(shape), dtype=psf.dtype)
    otf[..., :psf.shape[2], :psf.shape[3]] = psf
    otf = torch.roll(otf, (-(psf.shape[2] // 2), -(psf.shape[3] // 2)), dims=(2, 3))
    return torch.fft.fftn(otf, dim=(-2, -1))


def zero_upsample(x, sf):
    """v1:72-82."""
    z = x.new_zeros(x.shape[0], x.shape[1], x.shape[2] * sf, x.shape[3] * sf)
    z[..., ::sf, ::sf] = x
    return z


def datanet(x, FB, FBC, F2B, FBFy, alpha, sf):
    """v1:179-192 closed-form data step."""
    FR = FBFy + torch.fft.fftn(alpha * x, dim=(-2, -1))
    FBR = splits(FB * FR, sf).mean(-1)
    invW = splits(F2B, sf).mean(-1)
    invWBR = FBR / (invW + alpha)
    FX = (FR - FBC * invWBR.repeat(1, 1, sf, sf)) / alpha
    return torch.real(torch.fft.ifftn(FX, dim=(-2, -1)))


class _ResBlock(nn.Module):
    """basicblock.py:211-223 — x + conv(relu(conv(x))), keys 'res.0' / 'res.2' (no bias)."""

    def __init__(self, c):
        super().__init__()
        self.res = nn.Sequential(nn.Conv2d(c, c, 3, 1, 1, bias=False), nn.ReLU(), nn.Conv2d(c, c, 3, 1, 1, bias=False))

    def forward(self, x):
        return x + self.res(x)


class ResUNet(nn.Module):
    """v1:109-170 with act 'R', strideconv down, convtranspose up, no bias."""

    def __init__(self, in_nc=4, out_nc=3, nc=(64, 128, 256, 512), nb=2):
        super().__init__()
        self.m_head = nn.Conv2d(in_nc, nc[0], 3, 1, 1, bias=False)
        down = lambda a, b: nn.Sequential(*[_ResBlock(a) for _ in range(nb)], nn.Conv2d(a, b, 2, 2, 0, bias=False))
        up = lambda a, b: nn.Sequential(nn.ConvTranspose2d(a, b, 2, 2, 0, bias=False), *[_ResBlock(b) for _ in range(nb)])
        self.m_down1 = down(nc[0], nc[1])
        self.m_down2 = down(nc[1], nc[2])
        self.m_down3 = down(nc[2], nc[3])
        self.m_body = nn.Sequential(*[_ResBlock(nc[3]) for _ in range(nb)])
        self.m_up3 = up(nc[3], nc[2])
        self.m_up2 = up(nc[2], nc[1])
        self.m_up1 = up(nc[1], nc[0])
        self.m_tail = nn.Conv2d(nc[0], out_nc, 3, 1, 1, bias=False)

    def forward(self, x):
        h, w = x.shape[-2:]
        x = F.pad(x, (0, (8 - w % 8) % 8, 0, (8 - h % 8) % 8), mode="replicate")
        x1 = self.m_head(x)
        x2 = self.m_down1(x1)
        x3 = self.m_down2(x2)
        x4 = self.m_down3(x3)
        x = self.m_body(x4)
        x = self.m_up3(x + x4)
        x = self.m_up2(x + x3)
        x = self.m_up1(x + x2)
        x = self.m_tail(x + x1)
        return x[..., :h, :w]


class HyPaNet(nn.Module):
    """v1:204-216."""

    def __init__(self, in_nc=2, out_nc=8, channel=64):
        super().__init__()
        self.mlp = nn.Sequential(nn.Conv2d(in_nc, channel, 1), nn.ReLU(), nn.Conv2d(channel, channel, 1), nn.ReLU(),
                                 nn.Conv2d(channel, out_nc, 1), nn.Softplus())

    def forward(self, x):
        return self.mlp(x) + 1e-6


class USRNet(nn.Module):
    """v1:228-262."""

    def __init__(self, n_iter=8, h_nc=64, in_nc=4, out_nc=3, nc=(64, 128, 256, 512), nb=2, **_):
        super().__init__()
        self.p = ResUNet(in_nc, out_nc, nc, nb)
        self.h = HyPaNet(2, n_iter * 2, h_nc)
        self.n = n_iter

    def forward(self, x, k, sf, sigma):
        w, h = x.shape[-2:]
        FB = p2o(k, (w * sf, h * sf))
        FBC = torch.conj(FB)
        F2B = torch.abs(FB) ** 2
        FBFy = FBC * torch.fft.fftn(zero_upsample(x, sf), dim=(-2, -1))
        x = F.interpolate(x, scale_factor=sf, mode="nearest")
        ab = self.h(torch.cat((sigma, torch.tensor(sf).type_as(sigma).expand_as(sigma)), dim=1))
        for i in range(self.n):
            x = datanet(x, FB, FBC, F2B, FBFy, ab[:, i:i + 1], sf)
            x = self.p(torch.cat((x, ab[:, i + self.n:i + self.n + 1].repeat(1, 1, x.size(2), x.size(3))), dim=1))
        return x
