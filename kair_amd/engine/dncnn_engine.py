"""DnCNN / FDnCNN step program for MI355X.

Reference: /root/reference/models/network_dncnn.py:40-71 (DnCNN, out = x - model(x)), 128-149
(FDnCNN, out = model(x)); layers from basicblock.conv (basicblock.py:61-98).  SURVEY §8 row a14.

Per body layer: implicit-GEMM 3x3 conv (bias in the epilogue) -> fp32 pre-norm rows z ->
BatchNorm (batch statistics + running-stat update in train mode, running statistics in eval) with
the activation fused into the normalise pass -> compute-dtype activation rows for the next conv.
Without BN the activation is fused into the conv epilogue.  Backward: BN backward fuses the
activation gate and the two per-channel reductions; conv input / weight / bias gradients as in the
other conv programs.
"""
import torch
import torch.nn as nn

from .. import _hip as H
from .rrdbnet_engine import ConvEngineBase
from .swinir_engine import _Conv


def _rup(x, m):
    return (x + m - 1) // m * m


class DnCNNEngine(ConvEngineBase):
    def __init__(self, net, compute_dtype="bf16", residual=True):
        super().__init__(net, compute_dtype)
        self.residual = residual
        mods = list(net.model)
        self.device = mods[0].weight.device
        layers, i = [], 0
        while i < len(mods):
            conv = mods[i]
            if not isinstance(conv, nn.Conv2d) or conv.kernel_size != (3, 3) or conv.stride != (1, 1) or conv.padding != (1, 1):
                raise NotImplementedError("kair_amd DnCNN: 3x3 / stride 1 / pad 1 convs only")
            i += 1
            bn, act, slope = None, 0, 0.0
            if i < len(mods) and isinstance(mods[i], nn.BatchNorm2d):
                bn = mods[i]
                i += 1
            if i < len(mods) and isinstance(mods[i], (nn.ReLU, nn.LeakyReLU)):
                act = 1 if isinstance(mods[i], nn.ReLU) else 2
                slope = mods[i].negative_slope if act == 2 else 0.0
                i += 1
            layers.append((conv, bn, act, slope))
        self.in_ch = layers[0][0].in_channels
        self.out_ch = layers[-1][0].out_channels
        self.nc = layers[0][0].out_channels
        if self.nc % 8 or self.out_ch > 16:
            raise NotImplementedError("kair_amd DnCNN: nc multiple of 8, out_nc <= 16")
        self.Cin_p = _rup(self.in_ch, 8)
        self.layers = []
        for li, (conv, bn, act, slope) in enumerate(layers):
            cop = 16 if li == len(layers) - 1 else conv.out_channels
            cip = self.Cin_p if li == 0 else conv.in_channels
            self.layers.append((_Conv(self, conv, cop, cip, need_dgrad=li > 0), bn, act, slope))

    def convs(self):
        return [c for c, _, _, _ in self.layers]

    def _build_plan(self, key, infer):
        B, Hh, Ww = key
        T, e, nc = self.tdt, self._e, self.nc
        M = B * Hh * Ww
        P = {"B": B, "H": Hh, "W": Ww, "M": M}
        P["xin"] = e(M, self.Cin_p, dt=T)
        n_mid = len(self.layers) - 1
        P["a"] = [e(M, nc, dt=T) for _ in range(n_mid)]
        P["z"] = [e(M, nc) if bn is not None else None for _, bn, _, _ in self.layers[:n_mid]]
        P["mean"] = [e(nc) if bn is not None else None for _, bn, _, _ in self.layers[:n_mid]]
        P["rstd"] = [e(nc) if bn is not None else None for _, bn, _, _ in self.layers[:n_mid]]
        P["E"] = e(B, self.out_ch, Hh, Ww)
        P["dEf"] = torch.zeros(M, 16, device=self.device)
        P["dn"] = e(M, 16, dt=T)
        P["G"], P["dz"] = e(M, nc), e(M, nc, dt=T)
        P["dzf"] = e(M, nc)   # fp32 gradient rows before the compute-dtype cast (bias gradients)
        P["bn_ws"] = e(H.bn_ws(nc))
        P["loss"], P["loss_ws"] = e(1), e(1024)
        P["colsum_ws"] = e(1024 * 256)
        shapes = [(M, c.Cop, 9 * c.Cip) for c, _, _, _ in self.layers]
        P["wg_ws"] = e(self.wgrad_ws_size(shapes))
        return P

    def forward(self, x, drop_scales=None):
        B, _, Hh, Ww = x.shape
        P = self.plan(B, Hh, Ww)
        self.pack()
        cd, nc = self.cd, self.nc
        M = P["M"]
        x = x.contiguous()
        self.cur = P
        P["x"] = x
        training = self.net_ref().training
        H.image_to_nhwc(x, P["xin"], self.Cin_p, None, 1.0, B, self.in_ch, Hh, Ww)
        src, ldsrc, Cs = P["xin"], self.Cin_p, self.Cin_p
        for li, (c, bn, act, slope) in enumerate(self.layers[:-1]):
            a = P["a"][li]
            if bn is None:
                H.gemm_nt(H.im2col(src, Hh, Ww, Cs, ld=ldsrc), c.fwd(),
                          H.epilogue(a, bias=c.bp, act=(H.ACT_RELU if act == 1 else H.ACT_LEAKY) if act else H.ACT_NONE,
                                     slope=slope), M, nc, 9 * c.Cip, cd)
            else:
                z = P["z"][li]
                H.gemm_nt(H.im2col(src, Hh, Ww, Cs, ld=ldsrc), c.fwd(), H.epilogue(z, bias=c.bp), M, nc, 9 * c.Cip, cd)
                H.bn_fwd(z, nc, a, nc, M, nc, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum, bn.eps,
                         training, P["mean"][li], P["rstd"][li], act, slope, P["bn_ws"])
                if training:
                    bn.num_batches_tracked.add_(1)
            src, ldsrc, Cs = a, nc, nc
        c = self.layers[-1][0]
        H.gemm_nt(H.im2col(src, Hh, Ww, nc), c.fwd(),
                  H.epilogue(P["E"], mode=H.OUT_NCHW, ldo=0, bias=c.bp, img=(None, 1.0, self.out_ch, Hh, Ww)), M, c.Cop,
                  9 * nc, cd)
        if self.residual:
            H.axpby(P["E"], x, 1.0, -1.0)     # x - model(x)
        return P["E"]

    def backward_from_loss(self, H_img, grads, loss_weight=1.0, charb_eps=None):
        P = self.cur
        H.l1_loss(P["E"], H_img, P["loss"], P["dEf"], 16, loss_weight, P["B"], self.out_ch, P["H"], P["W"], P["loss_ws"], charb_eps=charb_eps)
        self.backward(grads, P)
        return P["loss"]

    def backward_from_grad(self, gE, grads):
        P = self.cur
        H.image_to_nhwc(gE.contiguous(), P["dEf"], 16, None, 1.0, P["B"], self.out_ch, P["H"], P["W"])
        self.backward(grads, P)

    def backward(self, grads, P):
        cd, nc = self.cd, self.nc
        Hh, Ww, M = P["H"], P["W"], P["M"]
        # d model(x) = -dE for DnCNN (out = x - model(x)), dE for FDnCNN
        H.act_grad_cast(P["dEf"], 16, None, 0, P["dn"], 16, M, 16, 0, 0.0, -1.0 if self.residual else 1.0)
        c = self.layers[-1][0]
        G = P["G"]
        H.gemm_nt(H.im2col(P["dn"], Hh, Ww, 16, flip=True), H.rows(c.Wd), H.epilogue(G), M, nc, 9 * 16, cd)
        self.conv_wgrad(P, c, P["dn"], 16, H.im2col(P["a"][-1], Hh, Ww, nc), M, grads)
        for li in range(len(self.layers) - 2, -1, -1):
            c, bn, act, slope = self.layers[li]
            a, dz = P["a"][li], P["dz"]
            if bn is not None:
                dzf = dz if cd == H.F32 else P["dzf"]
                H.bn_bwd(P["z"][li], nc, a, nc, G, nc, dzf, nc, M, nc, bn.weight, P["mean"][li], P["rstd"][li], act, slope,
                         grads[bn.weight], grads[bn.bias], False, P["bn_ws"])
                if cd != H.F32:
                    H.row_copy(dzf, nc, M, nc, H.copy_desc(dz))
                bs = (dzf, nc)
            else:
                bs = self.gate_cast(P, G, nc, a, nc, dz, nc, M, nc, act, slope)
            if li > 0:
                H.gemm_nt(H.im2col(dz, Hh, Ww, nc, flip=True), H.rows(c.Wd), H.epilogue(G), M, nc, 9 * nc, cd)
                self.conv_wgrad(P, c, dz, nc, H.im2col(P["a"][li - 1], Hh, Ww, nc), M, grads, *bs)
            else:
                self.conv_wgrad(P, c, dz, nc, H.im2col(P["xin"], Hh, Ww, self.Cin_p), M, grads, *bs)
