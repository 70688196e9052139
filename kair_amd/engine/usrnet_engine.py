"""USRNet step program for MI355X.

Reference: /root/reference/models/network_usrnet_v1.py (the torch.fft restatement of the
network_usrnet.py that define_G binds, select_network.py:167-178): p2o :48-69, upsample :72-82,
ResUNet :109-166, DataNet :179-194, HyPaNet :204-216, USRNet.forward :237-262.

Program per forward (B patches, LQ h x w, scale sf, HR H = h*sf, W = w*sf):
  ab = HyPaNet([sigma, sf])                                   one-block kernel, [B, 2n]
  FB = fft2(p2o(k)), invW = alias-mean |FB|^2                 rows pass + column pass
  FBFy = conj(FB) * fft2(upsample(x, sf))                     rows pass + column pass
  x = nearest-upsample(x)
  n times:  z = DataNet(x; alpha_i)     rows -> columns (closed form, inverse columns) -> inverse rows
            xin = [z, beta_i]           NHWC rows of 8 channels (the 4-channel cat, padded)
            x = ResUNet(xin)            -> NCHW image written by the tail conv's epilogue
ResUNet: implicit-GEMM 3x3 convs (im2col address map), the 2x2/stride-2 conv as a space-to-depth
operand (KAIR_LD_S2D), the 2x2/stride-2 transposed conv as a 1x1 GEMM with a pixel-shuffle store,
ReLU fused into the first conv of each ResBlock, the ResBlock residual and the U-Net skip fused
into the second conv's epilogue (two residual operands).  Backward mirrors it: ReLU' gate in the
dgrad epilogue, transposed-conv dgrad through the space-to-depth operand, stride-conv dgrad
through the pixel-shuffle store, skip gradients added by the first ResBlock of each level.  The
ResUNet weights are shared by the n iterations, so their gradients accumulate.

Maps are NHWC fp32 token rows (ReLU outputs and GEMM-only operands in the compute dtype), complex
planes float2 [planes][W][H] (kair_hip.h).  An HR size that is not a multiple of 8 runs the ResUNet on
the replicate-padded grid (v1:148-151) and crops its output (v1:164) -- kair_usr_pad, with the zero pad
(crop adjoint) of the output gradient and the fold (replicate adjoint) of the input gradient in
backward.  B*Hp*Wp < 2^24.
"""
import weakref

import torch
import torch.nn as nn

from .. import _hip as H
from .plans import Lease, PlanPool, autograd_mode, plan_mode

C8 = 8   # channel stride of the ResUNet input (x, beta) and of the tail-output gradient rows


def _mods(m):
    return list(m) if isinstance(m, nn.Sequential) else [m]


class _Conv3:
    """Bias-free 3x3 conv: forward [Cop][9 Cip] (kind 1) and input-gradient [Cip][9 Cop] (kind 2) packs."""

    def __init__(self, eng, mod, Cop=None, Cip=None):
        self.w = mod.weight
        self.Co, self.Ci = self.w.shape[:2]
        self.Cop, self.Cip = Cop or self.Co, Cip or self.Ci
        self.map = H.wmap(1, self.Co, self.Ci, (1, self.Co, self.Cop), (1, self.Ci, self.Cip))
        self.mapd = H.wmap(2, self.Co, self.Ci, (1, self.Co, self.Cop), (1, self.Ci, self.Cip))
        self.Wf = eng._e(self.Cop, 9 * self.Cip, dt=eng.tdt)
        self.Wd = eng._e(self.Cip, 9 * self.Cop, dt=eng.tdt)

    def pack_jobs(self):
        w = self.w.detach()
        return [(w, self.Wf, self.map), (w, self.Wd, self.mapd)]


class _Down:
    """Conv2d(Ci, Co, 2, stride 2, bias=False) (basicblock.downsample_strideconv, basicblock.py:495-501):
    forward through the space-to-depth operand with the [Co][4 Ci] pack (kind 7); input gradient as a
    1x1 GEMM into a pixel-shuffle store with the [4 Ci][Co] pack (kind 8); weight gradient kind 7."""

    def __init__(self, eng, mod):
        self.w = mod.weight
        self.Co, self.Ci = self.w.shape[:2]
        self.map = H.wmap(7, self.Co, self.Ci)
        self.mapd = H.wmap(8, self.Co, self.Ci)
        self.Wf = eng._e(self.Co, 4 * self.Ci, dt=eng.tdt)
        self.Wd = eng._e(4 * self.Ci, self.Co, dt=eng.tdt)

    def pack_jobs(self):
        w = self.w.detach()
        return [(w, self.Wf, self.map), (w, self.Wd, self.mapd)]


class _Up:
    """ConvTranspose2d(Ci, Co, 2, stride 2, bias=False) (basicblock.upsample_convtranspose,
    basicblock.py:471-477), weight [Ci][Co][2][2]: forward as a 1x1 GEMM into a pixel-shuffle store
    with the [4 Co][Ci] pack (kind 8 over (Ci, Co)); input gradient through the space-to-depth operand
    with the [Ci][4 Co] pack (kind 7 over (Ci, Co)); weight gradient kind 7 over (Ci, Co)."""

    def __init__(self, eng, mod):
        self.w = mod.weight
        self.Ci, self.Co = self.w.shape[:2]
        self.mapf = H.wmap(8, self.Ci, self.Co)
        self.map = H.wmap(7, self.Ci, self.Co)
        self.Wf = eng._e(4 * self.Co, self.Ci, dt=eng.tdt)
        self.Wd = eng._e(self.Ci, 4 * self.Co, dt=eng.tdt)

    def pack_jobs(self):
        w = self.w.detach()
        return [(w, self.Wf, self.mapf), (w, self.Wd, self.map)]


class _RB:
    def __init__(self, eng, rb):
        self.c1, self.c2 = _Conv3(eng, rb.res[0]), _Conv3(eng, rb.res[2])


class USRNetEngine:
    def __init__(self, net, compute_dtype="bf16"):
        self.net_ref = weakref.ref(net)
        if compute_dtype not in ("bf16", "fp32"):
            raise ValueError(compute_dtype)
        self.cd = H.BF16 if compute_dtype == "bf16" else H.F32
        self.tdt = torch.bfloat16 if compute_dtype == "bf16" else torch.float32
        p = net.p
        self.device = p.m_head.weight.device
        self.n = net.n
        self.in_nc, self.out_nc = p.m_head.in_channels, p.m_tail.out_channels
        if self.in_nc != self.out_nc + 1 or self.in_nc > C8:
            raise NotImplementedError("kair_amd USRNet: in_nc must be out_nc + 1 <= 8")
        self.hyp = [net.h.mlp[0], net.h.mlp[2], net.h.mlp[4]]
        self.hc, self.no = self.hyp[0].out_channels, self.hyp[2].out_channels
        if self.no != 2 * self.n or self.hyp[0].in_channels != 2:
            raise NotImplementedError("kair_amd USRNet: HyPaNet must map 2 -> 2 * n_iter")
        self.head = _Conv3(self, p.m_head, Cip=C8)
        self.tail = _Conv3(self, p.m_tail, Cop=C8)
        self.down_rbs, self.downs = [], []
        for d in (p.m_down1, p.m_down2, p.m_down3):
            ms = _mods(d)
            self.down_rbs.append([_RB(self, m) for m in ms[:-1]])
            self.downs.append(_Down(self, ms[-1]))
        self.body_rbs = [_RB(self, m) for m in _mods(p.m_body)]
        self.ups, self.up_rbs = [], []                 # m_up3 (-> level 2), m_up2 (-> 1), m_up1 (-> 0)
        for u in (p.m_up3, p.m_up2, p.m_up1):
            ms = _mods(u)
            self.ups.append(_Up(self, ms[0]))
            self.up_rbs.append([_RB(self, m) for m in ms[1:]])
        self.nc = [self.head.Co] + [d.Co for d in self.downs]
        if any(c % 8 for c in self.nc):
            raise NotImplementedError("kair_amd USRNet: ResUNet channel counts must be multiples of 8")
        self.plans = PlanPool(self._build_plan)
        self.plan_mode = "primary"
        self._packed_version = None
        self._pack_table = None
        self.blocks = []

    def _e(self, *shape, dt=torch.float32):
        return torch.empty(*shape, device=self.device, dtype=dt)

    def convs(self):
        cs = [self.head, self.tail] + self.downs + self.ups
        for rbs in self.down_rbs + [self.body_rbs] + self.up_rbs:
            for rb in rbs:
                cs += [rb.c1, rb.c2]
        return cs

    def pack(self, force=False):
        net = self.net_ref()
        ver = None if force else tuple(p._version for p in net.parameters())
        if ver is not None and ver == self._packed_version:
            return
        ptrs = tuple(p.data_ptr() for p in net.parameters())
        if self._pack_table is None or self._pack_table[0] != ptrs:
            jobs = [j for c in self.convs() for j in c.pack_jobs()]
            self._pack_table = (ptrs, H.PackTable(jobs))
        self._pack_table[1].run()
        self._packed_version = ver

    def _hyp(self):
        return [t for m in self.hyp for t in (m.weight, m.bias)]

    # ------------------------------------------------------------------------------------
    def _chain(self, M, c, n):
        return [{"h": self._e(M, c, dt=self.tdt), "out": self._e(M, c)} for _ in range(n)]

    def plan(self, B, h, w, sf, kh, kw):
        return self.plans.get((B, h, w, sf, kh, kw), self.plan_mode)

    def _build_plan(self, key, infer):
        B, h, w, sf, kh, kw = key
        Hh, Ww = h * sf, w * sf
        Hp, Wp = -(-Hh // 8) * 8, -(-Ww // 8) * 8   # the ResUNet's grid (ReplicationPad2d, v1:148-151)
        pad = (Hp, Wp) != (Hh, Ww)
        M = [B * (Hp >> l) * (Wp >> l) for l in range(4)]
        if M[0] >= 1 << 24:
            raise NotImplementedError("kair_amd USRNet: B*Hp*Wp must be < 2^24")
        T, e, nc, C = self.tdt, self._e, self.nc, self.out_nc
        planes = B * C
        P = {"B": B, "h": h, "w": w, "sf": sf, "H": Hh, "W": Ww, "Hp": Hp, "Wp": Wp, "pad": pad, "M": M}
        Mu = B * Hh * Ww   # pixels of the HR grid
        cplx = planes * Hh * Ww * 2
        P["T"], P["FBFy"] = e(cplx), e(cplx)
        P["FB"] = e(B * Hh * Ww * 2)
        P["invW"] = e(B * (Hh // sf) * (Ww // sf))
        P["ab"], P["gab"], P["sig"] = e(B, self.no), e(B, self.no), e(B)
        P["x0"], P["z"] = e(B, C, Hh, Ww), e(B, C, Hh, Ww)
        its = []
        for _ in range(self.n):
            its.append({"FR": e(cplx), "xin": e(M[0], C8, dt=T), "xout": e(B, C, Hh, Ww),
                        "xin_u": e(Mu, C8, dt=T) if pad else None, "xout_p": e(B, C, Hp, Wp) if pad else None,
                        "X": [e(M[l], nc[l]) for l in range(4)],
                        "down": [self._chain(M[l], nc[l], len(self.down_rbs[l])) for l in range(3)],
                        "body": self._chain(M[3], nc[3], len(self.body_rbs)),
                        "t": [e(M[l], nc[l]) for l in range(3)],
                        "up": [self._chain(M[l], nc[l], len(self.up_rbs[2 - l])) for l in range(3)]})
        P["it"] = its
        P["gE"] = torch.zeros(Mu, C8, device=self.device, dtype=T)
        P["gxin"] = e(M[0], C8)
        if pad:   # the output gradient on the padded grid (zeros outside), the input gradient folded back
            P["gE_p"], P["gxin_u"] = e(M[0], C8, dt=T), e(Mu, C8)
        P["G"] = [{"gS": e(M[l], nc[l]), "gc": e(M[l], nc[l]), "ga": e(M[l], nc[l]), "gb": e(M[l], nc[l]),
                   "gz": e(M[l], nc[l], dt=T)} for l in range(4)]
        P["a_ws"] = e(planes * (Ww // sf))
        P["cs_ws"] = e(B * H.USR_CHAN_CHUNKS)
        P["loss"], P["loss_ws"] = e(1), e(1024)
        shapes = [(M[0], nc[0], 9 * C8), (M[0], C8, 9 * nc[0])]
        shapes += [(M[l], nc[l], 9 * nc[l]) for l in range(4)]
        shapes += [(M[l + 1], nc[l + 1], 4 * nc[l]) for l in range(3)]
        P["wg_ws"] = e(max(H.wgrad_splits(m, n, k) * n * k for m, n, k in shapes))
        return P

    # ------------------------------------------------------------------------------------
    # forward
    # ------------------------------------------------------------------------------------
    def forward(self, x, k, sf, sigma):
        """x [B, C, h, w], k [B, 1, kh, kw], sigma [B, 1, 1, 1] (device fp32).  Returns the NCHW
        output buffer of the last iteration."""
        B, C, h, w = x.shape
        if C != self.out_nc:
            raise ValueError(f"kair_amd USRNet: {C} input channels, network has {self.out_nc}")
        if k.dim() != 4 or k.shape[0] != B or k.shape[1] != 1:
            raise NotImplementedError("kair_amd USRNet: one blur kernel per image, k of shape [B, 1, kh, kw]")
        kh, kw = k.shape[-2:]
        P = self.plan(B, h, w, sf, kh, kw)
        self.pack()
        self.cur = P
        x = x.contiguous().float()
        k = k.contiguous().float()
        P["x_in"], P["k_in"] = x, k
        P["sig"].copy_(sigma.reshape(B).float())
        Hh, Ww, planes = P["H"], P["W"], B * C
        H.hypanet_fwd(P["sig"], float(sf), *self._hyp(), self.hc, self.no, B, P["ab"])
        H.usr_fft_rows(k, H.USR_SRC_PSF, 1, 0, kh, kw, 1, P["FB"], B, Hh, Ww)
        H.usr_fft_cols(H.USR_COL_FB, P["FB"], P["FB"], None, None, None, P["invW"], None, 0, None, B, 1, Hh, Ww, sf)
        H.usr_fft_rows(x, H.USR_SRC_ZUP, C, 0, 0, 0, sf, P["FBFy"], planes, Hh, Ww)
        H.usr_fft_cols(H.USR_COL_FBFY, P["FBFy"], P["FBFy"], P["FB"], None, None, P["invW"], None, 0, None, planes, C,
                       Hh, Ww, sf)
        H.usr_upsample_nearest(x, P["x0"], planes, h, w, sf)
        xc = P["x0"]
        for i in range(self.n):
            S = P["it"][i]
            self._datanet_fwd(P, S, xc, i)
            self._unet_fwd(P, S)
            xc = S["xout"]
        return xc

    def _datanet_fwd(self, P, S, xc, i):
        B, C, Hh, Ww, sf = P["B"], self.out_nc, P["H"], P["W"], P["sf"]
        planes, ab = B * C, P["ab"]
        H.usr_fft_rows(xc, H.USR_SRC_NCHW, C, 0, 0, 0, 1, P["T"], planes, Hh, Ww)
        H.usr_fft_cols(H.USR_COL_DATA_FWD, P["T"], P["T"], P["FB"], P["FBFy"], S["FR"], P["invW"], ab[:, i], self.no, None,
                       planes, C, Hh, Ww, sf)
        H.usr_ifft_rows(P["T"], P["z"], False, C, 0, 1.0 / (Hh * Ww), planes, Hh, Ww)
        if P["pad"]:
            H.usr_pack_input(P["z"], ab[:, self.n + i], self.no, S["xin_u"], C8, B, C, Hh * Ww)
            H.usr_pad(S["xin_u"], S["xin"], H.USR_PAD_REPLICATE, C8, B, Hh, Ww, P["Hp"], P["Wp"])
        else:
            H.usr_pack_input(P["z"], ab[:, self.n + i], self.no, S["xin"], C8, B, C, Hh * Ww)

    def _grid(self, P, l):
        """The ResUNet's level-l grid (the replicate-padded HR grid at l = 0)."""
        return P["Hp"] >> l, P["Wp"] >> l

    def _chain_fwd(self, rbs, bufs, x, Hl, Wl, M, c, skip=None):
        """ResBlocks x + conv2(relu(conv1(x))); the last adds `skip` (the U-Net skip) too."""
        cd, cur = self.cd, x
        for j, (rb, S) in enumerate(zip(rbs, bufs)):
            H.gemm_nt(H.im2col(cur, Hl, Wl, c), H.rows(rb.c1.Wf), H.epilogue(S["h"], act=H.ACT_RELU), M, c, 9 * c, cd)
            last = j == len(rbs) - 1
            H.gemm_nt(H.im2col(S["h"], Hl, Wl, c), H.rows(rb.c2.Wf),
                      H.epilogue(S["out"], resid=cur, resid2=skip if last else None), M, c, 9 * c, cd)
            cur = S["out"]
        return cur

    def _unet_fwd(self, P, S):
        cd, nc, M = self.cd, self.nc, P["M"]
        H0, W0 = self._grid(P, 0)
        H.gemm_nt(H.im2col(S["xin"], H0, W0, C8), H.rows(self.head.Wf), H.epilogue(S["X"][0]), M[0], nc[0], 9 * C8, cd)
        cur = S["X"][0]
        for l in range(3):
            Hl, Wl = self._grid(P, l)
            a = self._chain_fwd(self.down_rbs[l], S["down"][l], cur, Hl, Wl, M[l], nc[l])
            Hn, Wn = self._grid(P, l + 1)
            H.gemm_nt(H.s2d(a, Hn, Wn, nc[l]), H.rows(self.downs[l].Wf), H.epilogue(S["X"][l + 1]), M[l + 1], nc[l + 1],
                      4 * nc[l], cd)
            cur = S["X"][l + 1]
        H3, W3 = self._grid(P, 3)
        s = self._chain_fwd(self.body_rbs, S["body"], cur, H3, W3, M[3], nc[3], skip=S["X"][3])
        for u in range(3):
            l = 2 - u                              # output level of m_up(3-u)
            Hs, Ws = self._grid(P, l + 1)
            H.gemm_nt(H.rows(s), H.rows(self.ups[u].Wf), H.epilogue(S["t"][l], mode=H.OUT_PSHUF, ldo=nc[l], ps=(2, Hs, Ws)),
                      M[l + 1], 4 * nc[l], nc[l + 1], cd)
            Hl, Wl = self._grid(P, l)
            s = self._chain_fwd(self.up_rbs[u], S["up"][l], S["t"][l], Hl, Wl, M[l], nc[l], skip=S["X"][l])
        xo = S["xout_p"] if P["pad"] else S["xout"]
        H.gemm_nt(H.im2col(s, H0, W0, nc[0]), H.rows(self.tail.Wf),
                  H.epilogue(xo, mode=H.OUT_NCHW, ldo=0, img=(None, 1.0, self.out_nc, H0, W0)), M[0], C8,
                  9 * nc[0], cd)
        if P["pad"]:   # x[..., :h, :w] (v1:164)
            H.usr_pad(xo, S["xout"], H.USR_CROP_NCHW, 0, P["B"] * self.out_nc, P["H"], P["W"], H0, W0)

    # ------------------------------------------------------------------------------------
    # backward
    # ------------------------------------------------------------------------------------
    def backward_from_loss(self, H_img, grads, loss_weight=1.0, charb_eps=None):
        P = self.cur
        H.l1_loss(P["it"][-1]["xout"], H_img, P["loss"], P["gE"], C8, loss_weight, P["B"], self.out_nc, P["H"], P["W"],
                  P["loss_ws"], charb_eps=charb_eps)
        self.backward(grads, P)
        return P["loss"]

    def backward_from_grad(self, gE, grads):
        P = self.cur
        H.image_to_nhwc(gE.contiguous(), P["gE"], C8, None, 1.0, P["B"], self.out_nc, P["H"], P["W"])
        self.backward(grads, P)

    def backward(self, grads, P):
        B, C, Hh, Ww, sf, n = P["B"], self.out_nc, P["H"], P["W"], P["sf"], self.n
        planes, inv_n = B * C, 1.0 / (Hh * Ww)
        ab, gab = P["ab"], P["gab"]
        for i in range(n - 1, -1, -1):
            S = P["it"][i]
            self._unet_bwd(P, S, grads, acc=i < n - 1)
            gxin = P["gxin"]
            if P["pad"]:   # adjoint of the replicate pad: pad pixels' gradients onto the edge they copied
                gxin = P["gxin_u"]
                H.usr_pad(P["gxin"], gxin, H.USR_PAD_FOLD, C8, B, Hh, Ww, P["Hp"], P["Wp"])
            # beta_i: channel C of the ResUNet input gradient, summed over pixels
            H.usr_chan_sum(gxin, C8, C, Hh * Ww, B, P["cs_ws"], gab[:, n + i], self.no)
            # DataNet_i backward: dL/dx_{i-1} (skipped for i = 0: the upsampled LQ needs none) and dL/dalpha_i
            H.usr_fft_rows(gxin, H.USR_SRC_NHWC, C, C8, 0, 0, 1, P["T"], planes, Hh, Ww)
            H.usr_fft_cols(H.USR_COL_DATA_BWD, P["T"], P["T"] if i > 0 else None, P["FB"], P["FBFy"], S["FR"], P["invW"],
                           ab[:, i], self.no, P["a_ws"], planes, C, Hh, Ww, sf)
            H.usr_seg_sum(P["a_ws"], C * (Ww // sf), B, inv_n, gab[:, i], self.no)
            if i > 0:
                H.usr_ifft_rows(P["T"], P["gE"], True, C, C8, inv_n, planes, Hh, Ww)
        hp = self._hyp()
        H.hypanet_bwd(P["sig"], float(sf), *hp, self.hc, self.no, B, gab, *[grads[t] for t in hp])

    def _wgrad(self, P, A, Bop, M, N, K, m, grad, acc):
        S = H.wgrad_splits(M, N, K)
        H.gemm_tn(A, Bop, P["wg_ws"], S, M, N, K, self.cd)
        H.wgrad_finalize(P["wg_ws"], S, m, grad, accumulate=acc)

    def _chain_bwd(self, P, rbs, bufs, x_in, g, Hl, Wl, M, c, G, grads, acc, skip_g=None):
        """g: fp32 dL/d(chain output) -> returns fp32 dL/d(chain input) (+ skip_g, the U-Net skip)."""
        cd, cur = self.cd, g
        for j in range(len(rbs) - 1, -1, -1):
            rb, S = rbs[j], bufs[j]
            r_in = bufs[j - 1]["out"] if j > 0 else x_in
            H.gemm_nt(H.im2col(cur, Hl, Wl, c, flip=True), H.rows(rb.c2.Wd), H.epilogue(G["gz"], gate=S["h"], gate_kind=3),
                      M, c, 9 * c, cd)
            self._wgrad(P, H.rows(cur), H.im2col(S["h"], Hl, Wl, c), M, c, 9 * c, rb.c2.map, grads[rb.c2.w], acc)
            out = G["ga"] if cur is not G["ga"] else G["gb"]
            H.gemm_nt(H.im2col(G["gz"], Hl, Wl, c, flip=True), H.rows(rb.c1.Wd),
                      H.epilogue(out, resid=cur, resid2=skip_g if j == 0 else None), M, c, 9 * c, cd)
            self._wgrad(P, H.rows(G["gz"]), H.im2col(r_in, Hl, Wl, c), M, c, 9 * c, rb.c1.map, grads[rb.c1.w], acc)
            cur = out
        return cur

    def _unet_bwd(self, P, S, grads, acc):
        cd, nc, M, Gs = self.cd, self.nc, P["M"], P["G"]
        H0, W0 = self._grid(P, 0)
        gE = P["gE"]
        if P["pad"]:   # adjoint of the crop: the output gradient on the padded grid, zeros outside
            H.usr_pad(gE, P["gE_p"], H.USR_PAD_ZERO, C8, P["B"], P["H"], P["W"], H0, W0)
            gE = P["gE_p"]
        H.gemm_nt(H.im2col(gE, H0, W0, C8, flip=True), H.rows(self.tail.Wd), H.epilogue(Gs[0]["gS"]), M[0], nc[0],
                  9 * C8, cd)
        s1 = S["up"][0][-1]["out"]
        self._wgrad(P, H.rows(gE), H.im2col(s1, H0, W0, nc[0]), M[0], C8, 9 * nc[0], self.tail.map, grads[self.tail.w],
                    acc)
        g = Gs[0]["gS"]
        for u in (2, 1, 0):                        # m_up1, m_up2, m_up3
            l = 2 - u
            Hl, Wl = self._grid(P, l)
            gt = self._chain_bwd(P, self.up_rbs[u], S["up"][l], S["t"][l], g, Hl, Wl, M[l], nc[l], Gs[l], grads, acc)
            up = self.ups[u]
            Hs, Ws = self._grid(P, l + 1)
            s_next = S["body"][-1]["out"] if l == 2 else S["up"][l + 1][-1]["out"]
            H.gemm_nt(H.s2d(gt, Hs, Ws, nc[l]), H.rows(up.Wd), H.epilogue(Gs[l + 1]["gS"]), M[l + 1], nc[l + 1],
                      4 * nc[l], cd)
            self._wgrad(P, H.rows(s_next), H.s2d(gt, Hs, Ws, nc[l]), M[l + 1], nc[l + 1], 4 * nc[l], up.map,
                        grads[up.w], acc)
            g = Gs[l + 1]["gS"]
        H3, W3 = self._grid(P, 3)
        gx = self._chain_bwd(P, self.body_rbs, S["body"], S["X"][3], Gs[3]["gS"], H3, W3, M[3], nc[3], Gs[3], grads, acc,
                             skip_g=Gs[3]["gS"])
        for l in (2, 1, 0):
            d = self.downs[l]
            Hn, Wn = self._grid(P, l + 1)
            Hl, Wl = self._grid(P, l)
            a = S["down"][l][-1]["out"]
            H.gemm_nt(H.rows(gx), H.rows(d.Wd), H.epilogue(Gs[l]["gc"], mode=H.OUT_PSHUF, ldo=nc[l], ps=(2, Hn, Wn)),
                      M[l + 1], 4 * nc[l], nc[l + 1], cd)
            self._wgrad(P, H.rows(gx), H.s2d(a, Hn, Wn, nc[l]), M[l + 1], nc[l + 1], 4 * nc[l], d.map, grads[d.w], acc)
            gx = self._chain_bwd(P, self.down_rbs[l], S["down"][l], S["X"][l], Gs[l]["gc"], Hl, Wl, M[l], nc[l], Gs[l],
                                 grads, acc, skip_g=Gs[l]["gS"])
        H.gemm_nt(H.im2col(gx, H0, W0, nc[0], flip=True), H.rows(self.head.Wd), H.epilogue(P["gxin"]), M[0], C8,
                  9 * nc[0], cd)
        self._wgrad(P, H.rows(gx), H.im2col(S["xin"], H0, W0, C8), M[0], nc[0], 9 * C8, self.head.map,
                    grads[self.head.w], acc)


class USRNetFunction(torch.autograd.Function):
    """The whole unfolded USRNet forward/backward as one autograd node (params are inputs); the
    node leases its plan from forward to backward (kair_amd/engine/plans.py)."""

    @classmethod
    def run(cls, engine, x, k, sf, sigma, params):
        return cls.apply(engine, autograd_mode(params), x, k, sf, sigma, *params)

    @staticmethod
    def forward(ctx, engine, mode, x, k, sf, sigma, *params):
        with plan_mode(engine, mode):
            E = engine.forward(x, k, sf, sigma)
        ctx.engine, ctx.params = engine, params
        ctx.lease = Lease(engine.cur) if mode == "lease" else None
        return E.clone()

    @staticmethod
    def backward(ctx, gE):
        eng = ctx.engine
        if ctx.lease is None or ctx.lease.plan is None:
            raise RuntimeError("kair_amd USRNet: backward through a forward whose activations were released")
        flat = torch.empty(sum(p.numel() for p in ctx.params), device=gE.device)
        grads, off = {}, 0
        for p in ctx.params:
            grads[p] = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        eng.cur = ctx.lease.plan
        eng.backward_from_grad(gE.float(), grads)
        ctx.lease.release()
        return (None,) * 6 + tuple(grads[p] for p in ctx.params)
