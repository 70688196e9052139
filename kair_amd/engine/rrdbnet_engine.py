"""RRDBNet (ESRGAN generator) step program for MI355X.

Reference: /root/reference/models/network_rrdbnet.py:35-119 (ResidualDenseBlock_5C, RRDB,
RRDBNet.forward).  SURVEY §8 row a15.

Layout: NHWC feature rows.  Each residual dense block owns ONE compute-dtype
buffer [M, nf + 4 gc] = [x | x1 | x2 | x3 | x4]: every conv reads a prefix of it through the
im2col address map (pixel stride nf + 4 gc) and its epilogue (bias + LeakyReLU 0.2) writes its
gc output channels straight into the next slice, so torch.cat never materialises.  conv5's
epilogue applies the 0.2-scaled residual in fp32.  The nearest x2 upsamples of the tail are an
im2col address mode (`im_up`); their adjoint is a 2x2 sum-pool.  Backward accumulates the input
gradients of the five convs into one fp32 buffer of the same width (dgrad epilogues add in place),
gates them with LeakyReLU' read from the saved post-activation slices, and reduces weight / bias
gradients with the split-M TN GEMM + deterministic finalize / column sums.
"""
import math
import weakref

import torch

from .. import _hip as H
from .plans import Lease, PlanPool, autograd_mode, plan_mode
from .swinir_engine import _Conv


class ConvEngineBase:
    """Shared plumbing of the conv-net step programs: packed weights (one batched launch), plan
    cache, conv forward / weight-gradient helpers."""

    def __init__(self, net, compute_dtype):
        self.net_ref = weakref.ref(net)
        if compute_dtype not in ("bf16", "fp32", "fp32x3"):
            raise ValueError(compute_dtype)
        # fp32x3 (the reference's fp32 precision class on the 16-bit matrix cores, as SwinIREngine): fp32 activations
        # and gradients in HBM, every conv product as hi.hi + hi.lo + lo.hi of power-of-2-scaled fp16 pairs (the
        # split in the GEMM kernels, weights packed as fp16 pairs), fp32 accumulation; cd stays F32 for the
        # fp32-rows bookkeeping (gate_cast), the launches go through _nt / conv_wgrad with compute KAIR_COMPUTE_X3
        self.x3 = compute_dtype == "fp32x3"
        self.cd = H.BF16 if compute_dtype == "bf16" else H.F32
        self.tdt = torch.bfloat16 if compute_dtype == "bf16" else torch.float32
        self.X3_AEXP = 4          # activation exponent (lowered by x3_backoff)
        self.x3_gexp_off = 4      # gradient exponent over the loss normalisation
        self.x3_backoffs = 0
        self._ax = self.X3_AEXP   # the exponent of the GEMM A operands of the phase being issued
        self.plans = PlanPool(self._build_plan)
        self.plan_mode = "primary"
        self._packed_version = None
        self._pack_table = None
        self.blocks = []          # no stochastic depth in the conv nets (FusedTrainer checks this)
        self.seg_hook = None      # called between the gradient segments of backward() (grad_segments())

    def _segment_done(self):
        if self.seg_hook is not None:
            self.seg_hook()

    X3_BACKOFF_STEP, X3_BACKOFF_MAX = 6, 4

    def _nt(self, A, B, E, M, N, K):
        """kair_gemm_nt in the engine's arithmetic; fp32x3: A carries the phase exponent, B the weight packs'."""
        if self.x3:
            A.x3_exp, B.x3_exp = self._ax, H.X3_WEXP
            H.gemm_nt(A, B, E, M, N, K, H.X3)
        else:
            H.gemm_nt(A, B, E, M, N, K, self.cd)

    def _x3_grad_exp(self, numel, weight=1.0):
        """Data gradients of a mean loss are O(weight / numel): times 2^(log2(numel / weight) + 4) they sit near 2^4."""
        return int(round(math.log2(max(numel, 1) / max(abs(weight), 1e-30)))) + self.x3_gexp_off

    def x3_backoff(self, step=None, act=True, grad=True):
        """The range guard's reaction (FusedTrainer.check_range; SwinIREngine.x3_backoff)."""
        if not self.x3:
            raise RuntimeError("x3_backoff: not an fp32x3 engine")
        if self.x3_backoffs >= self.X3_BACKOFF_MAX:
            raise RuntimeError(f"fp32x3 range guard: the step is still non-finite after {self.x3_backoffs} exponent "
                               f"back-offs: the data is not finite, or a weight left its pack window |w| < "
                               f"2^{16 - H.X3_WEXP}")
        step = self.X3_BACKOFF_STEP if step is None else int(step)
        if act:
            self.X3_AEXP -= step
        if grad:
            self.x3_gexp_off -= step
        self.x3_backoffs += 1
        return self.X3_AEXP, self.x3_gexp_off

    def convs(self):
        raise NotImplementedError

    def plan(self, B, Hh, Ww):
        return self.plans.get((B, Hh, Ww), self.plan_mode)

    def _build_plan(self, key, infer):
        raise NotImplementedError

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

    def _e(self, *shape, dt=torch.float32):
        return torch.empty(*shape, device=self.device, dtype=dt)

    def conv_wgrad(self, P, c, dz, ld_dz, src_op, M, grads, bias_src=None, ld_bias=None):
        """weight + bias gradient of conv c: dz [M, Cop] rows (compute dtype), src_op its im2col input;
        bias_src: the fp32 rows dz was cast from (bias gradient summed before rounding)."""
        K = 9 * c.Cip
        S = H.wgrad_splits(M, c.Cop, K)
        A = H.rows(dz, ld=ld_dz)
        if self.x3:   # (gradient, activation) operands
            A.x3_exp, src_op.x3_exp = P["e_g"], self.X3_AEXP
        H.gemm_tn(A, src_op, P["wg_ws"], S, M, c.Cop, K, H.X3 if self.x3 else self.cd)
        H.wgrad_finalize(P["wg_ws"], S, c.map, grads[c.w])
        if bias_src is None:
            bias_src, ld_bias = dz, ld_dz
        H.colsum(H.rows(bias_src, ld=ld_bias), M, c.Cop, c.mapb, grads[c.b], P["colsum_ws"])

    def gate_cast(self, P, G, ldg, X, ldx, out, ldo, M, C, kind, slope=0.0, scale=1.0):
        """out (compute dtype) = scale * G * act'(X).  Returns the fp32 rows to take the bias gradient
        from: `out` itself in fp32 mode, else an fp32 scratch holding the values before rounding."""
        if self.cd == H.F32:
            H.act_grad_cast(G, ldg, X, ldx, out, ldo, M, C, kind, slope, scale)
            return out, ldo
        f = P["dzf"].view(-1)[:M * C].view(M, C)
        H.act_grad_cast(G, ldg, X, ldx, f, C, M, C, kind, slope, scale)
        H.row_copy(f, C, M, C, H.copy_desc(out, ld=ldo))
        return f, C

    def wgrad_ws_size(self, shapes):
        return max(H.wgrad_splits(m, n, k) * n * k for m, n, k in shapes)


class RRDBNetEngine(ConvEngineBase):
    """Also runs network_rrdb.RRDB (option net_type 'rrdb', basicblock.py:393-428 + upsample_upconv
    455-465): same topology with a configurable activation; see spec_from_rrdb()."""

    def __init__(self, net, compute_dtype="bf16", spec=None):
        super().__init__(net, compute_dtype)
        if spec is None:
            spec = {"first": net.conv_first, "rrdbs": [(r.RDB1, r.RDB2, r.RDB3) for r in net.RRDB_trunk],
                    "rdb_convs": lambda d: [d.conv1, d.conv2, d.conv3, d.conv4, d.conv5], "trunk": net.trunk_conv,
                    "up": [net.upconv1] + ([net.upconv2] if net.sf == 4 else []), "hr": net.HRconv,
                    "last": net.conv_last, "act": 2, "slope": 0.2}
        self.act, self.slope = spec["act"], spec["slope"]
        self._spec_mods = spec   # the modules grad_segments() groups
        self.act_epi = H.ACT_LEAKY if self.act == 2 else H.ACT_RELU
        first = spec["first"]
        self.device = first.weight.device
        self.nf = first.out_channels
        rdb_convs = spec["rdb_convs"]
        self.gc = rdb_convs(spec["rrdbs"][0][0])[0].out_channels
        if self.nf % 8 or self.gc % 8:
            raise NotImplementedError("kair_amd RRDB: nf, gc must be multiples of 8")
        self.in_ch, self.out_ch = first.in_channels, spec["last"].out_channels
        self.Cin_p = 8
        self.CD = self.nf + 4 * self.gc
        nf = self.nf
        self.conv_first = _Conv(self, first, nf, self.Cin_p, need_dgrad=False)
        self.rdbs = []
        for rr in spec["rrdbs"]:
            for rdb in rr:
                self.rdbs.append([_Conv(self, m, m.out_channels, m.in_channels) for m in rdb_convs(rdb)])
        self.nrr = len(spec["rrdbs"])
        self.trunk = _Conv(self, spec["trunk"], nf, nf)
        self.up = [_Conv(self, m, nf, nf) for m in spec["up"]]
        if not self.up:
            raise NotImplementedError("kair_amd RRDB: x2 / x4 upscaling only")
        self.hr = _Conv(self, spec["hr"], nf, nf)
        self.last = _Conv(self, spec["last"], 16, nf)

    def convs(self):
        return [self.conv_first] + [c for r in self.rdbs for c in r] + [self.trunk] + self.up + [self.hr, self.last]

    RRDB_PER_SEGMENT = 3   # RRDBs per data-parallel gradient bucket (~8.6 MB of fp32 gradients at nf 64, gc 32)

    def grad_segments(self):
        """Parameter groups in the order backward() completes their gradients (the data-parallel trainer
        all-reduces each as one bucket while the rest of backward runs; reference DDP: model_base.py:113-119):
        the tail (trunk_conv, upsampling convs, HRconv, conv_last), then the RRDB trunk in groups of
        RRDB_PER_SEGMENT, last to first, the first group together with conv_first."""
        sp = self._spec_mods
        plist = lambda mods: [p for m in mods for p in m.parameters()]
        segs = [plist([sp["trunk"]] + list(sp["up"]) + [sp["hr"], sp["last"]])]
        rr = sp["rrdbs"]
        k = self.RRDB_PER_SEGMENT
        starts = list(range(0, len(rr), k))
        for s0 in reversed(starts[1:]):
            segs.append(plist([m for trip in rr[s0:s0 + k] for m in trip]))
        segs.append(plist([sp["first"]] + [m for trip in rr[:k] for m in trip]))
        return segs

    # ------------------------------------------------------------------------------------
    def _build_plan(self, key, infer):
        B, Hh, Ww = key
        T, e = self.tdt, self._e
        nf, gc, CD = self.nf, self.gc, self.CD
        M = B * Hh * Ww
        nr = len(self.rdbs)
        P = {"B": B, "H": Hh, "W": Ww, "M": M}
        P["xin"] = e(M, self.Cin_p, dt=T)
        P["fea"] = e(M, nf)
        P["dense"] = [e(M, CD, dt=T) for _ in range(nr + 1)]    # +1: slice 0 = trunk_conv input
        P["y"] = [e(M, nf) for _ in range(nr)]
        P["fea2"], P["fea2b"] = e(M, nf), e(M, nf, dt=T)
        levels, h, w = [], Hh, Ww
        for _ in self.up:
            h, w = 2 * h, 2 * w
            levels.append((h, w))
        P["levels"] = levels
        P["upa"] = [e(B * hh * ww, nf, dt=T) for hh, ww in levels]
        HL, WL = levels[-1]
        ML = B * HL * WL
        P["ML"] = ML
        P["hr"] = e(ML, nf, dt=T)
        P["E"] = e(B, self.out_ch, HL, WL)
        P["alpha"] = torch.full((1,), 0.2, device=self.device)
        # backward
        P["dE"] = e(ML, 16, dt=T)
        P["G_hr"], P["dz_hr"], P["G_hi"] = e(ML, nf), e(ML, nf, dt=T), e(ML, nf)
        P["G_lv"] = [e(B * hh * ww, nf) for hh, ww in levels]
        P["Gt"], P["dzt"], P["G_R"] = e(M, nf), e(M, nf, dt=T), e(M, nf)
        P["Gd"], P["dz5"], P["dzg"], P["gy"] = e(M, CD), e(M, nf, dt=T), e(M, gc, dt=T), e(M, nf)
        P["dzf"] = e(ML, nf)   # fp32 gradient rows before the compute-dtype cast (bias gradients)
        P["loss"], P["loss_ws"] = e(1), e(1024)
        P["colsum_ws"] = e(1024 * 256)
        shapes = [(M, nf, 9 * self.Cin_p), (M, nf, 9 * nf), (ML, 16, 9 * nf), (ML, nf, 9 * nf)]
        shapes += [(B * hh * ww, nf, 9 * nf) for hh, ww in levels]
        shapes += [(M, c.Cop, 9 * c.Cip) for c in self.rdbs[0]]
        P["wg_ws"] = e(self.wgrad_ws_size(shapes))
        return P

    # ------------------------------------------------------------------------------------
    def forward(self, x, drop_scales=None):
        B, _, Hh, Ww = x.shape
        P = self.plan(B, Hh, Ww)
        self.pack()
        cd, nf, gc, CD = self.cd, self.nf, self.gc, self.CD
        M = P["M"]
        x = x.contiguous()
        self.cur = P
        self._ax = self.X3_AEXP   # fp32x3: forward operands are activations
        H.image_to_nhwc(x, P["xin"], self.Cin_p, None, 1.0, B, self.in_ch, Hh, Ww)
        c = self.conv_first
        self._nt(H.im2col(P["xin"], Hh, Ww, self.Cin_p), c.fwd(), H.epilogue(P["fea"], bias=c.bp), M, nf,
                  9 * self.Cin_p)
        dense = P["dense"]
        H.row_copy(P["fea"], nf, M, nf, H.copy_desc(dense[0], ld=CD))
        rr_in = P["fea"]
        for r, cs in enumerate(self.rdbs):
            x_in = rr_in if r % 3 == 0 else P["y"][r - 1]
            D = dense[r]
            for j in range(4):          # x_{j+1} = lrelu(conv_{j+1}(cat(x, x1..x_j)))
                c, cin = cs[j], nf + j * gc
                self._nt(H.im2col(D, Hh, Ww, cin, ld=CD), c.fwd(),
                          H.epilogue(D[:, cin:cin + gc], ldo=CD, bias=c.bp, act=self.act_epi, slope=self.slope), M, gc, 9 * cin)
            c = cs[4]                    # y = x + 0.2 * conv5(cat(x, x1..x4))
            y = P["y"][r]
            self._nt(H.im2col(D, Hh, Ww, CD, ld=CD), c.fwd(),
                      H.epilogue(y, bias=c.bp, resid=x_in, rowscale=P["alpha"], rows_per_scale=M), M, nf, 9 * CD)
            if r % 3 == 2:               # RRDB: out = 0.2 * RDB3 + x   (in place over y)
                H.axpby(y, rr_in, 1.0, 0.2)
                rr_in = y
            H.row_copy(y, nf, M, nf, H.copy_desc(dense[r + 1], ld=CD))
        c = self.trunk                   # fea = fea + trunk_conv(trunk)
        self._nt(H.im2col(dense[-1], Hh, Ww, nf, ld=CD), c.fwd(), H.epilogue(P["fea2"], bias=c.bp, resid=P["fea"]),
                  M, nf, 9 * nf)
        H.row_copy(P["fea2"], nf, M, nf, H.copy_desc(P["fea2b"]))
        src = P["fea2b"]
        for c, (hh, ww), dst in zip(self.up, P["levels"], P["upa"]):   # lrelu(upconv(nearest x2))
            self._nt(H.im2col(src, hh, ww, nf, up=2), c.fwd(), H.epilogue(dst, bias=c.bp, act=self.act_epi, slope=self.slope),
                      B * hh * ww, nf, 9 * nf)
            src = dst
        HL, WL = P["levels"][-1]
        ML = P["ML"]
        c = self.hr
        self._nt(H.im2col(src, HL, WL, nf), c.fwd(), H.epilogue(P["hr"], bias=c.bp, act=self.act_epi, slope=self.slope), ML,
                  nf, 9 * nf)
        c = self.last
        self._nt(H.im2col(P["hr"], HL, WL, nf), c.fwd(),
                  H.epilogue(P["E"], mode=H.OUT_NCHW, ldo=0, bias=c.bp, img=(None, 1.0, self.out_ch, HL, WL)), ML, c.Cop,
                  9 * nf)
        return P["E"]

    # ------------------------------------------------------------------------------------
    def backward_from_loss(self, H_img, grads, loss_weight=1.0, charb_eps=None):
        P = self.cur
        HL, WL = P["levels"][-1]
        H.l1_loss(P["E"], H_img, P["loss"], P["dE"], 16, loss_weight, P["B"], self.out_ch, HL, WL, P["loss_ws"], charb_eps=charb_eps)
        P["e_g"] = self._x3_grad_exp(P["B"] * self.out_ch * HL * WL, loss_weight)
        self.backward(grads, P)
        return P["loss"]

    def backward_from_grad(self, gE, grads):
        P = self.cur
        HL, WL = P["levels"][-1]
        H.image_to_nhwc(gE.contiguous(), P["dE"], 16, None, 1.0, P["B"], self.out_ch, HL, WL)
        if self.x3:   # an arbitrary upstream gradient: its exponent from its own range (one host sync)
            mx = float(gE.abs().max())
            P["e_g"] = (8 - int(math.ceil(math.log2(mx)))) if mx > 0 and math.isfinite(mx) else 0
        self.backward(grads, P)

    def backward(self, grads, P):
        cd, nf, gc, CD = self.cd, self.nf, self.gc, self.CD
        self._ax = P.get("e_g", 0)   # fp32x3: backward GEMM A operands are data gradients
        B, Hh, Ww, M, ML = P["B"], P["H"], P["W"], P["M"], P["ML"]
        HL, WL = P["levels"][-1]
        # conv_last
        c = self.last
        self._nt(H.im2col(P["dE"], HL, WL, 16, flip=True), H.rows(c.Wd), H.epilogue(P["G_hr"]), ML, nf, 9 * 16)
        self.conv_wgrad(P, c, P["dE"], 16, H.im2col(P["hr"], HL, WL, nf), ML, grads)
        # HRconv (lrelu)
        c = self.hr
        bs = self.gate_cast(P, P["G_hr"], nf, P["hr"], nf, P["dz_hr"], nf, ML, nf, self.act, self.slope)
        G = P["G_lv"][-1]
        self._nt(H.im2col(P["dz_hr"], HL, WL, nf, flip=True), H.rows(c.Wd), H.epilogue(G), ML, nf, 9 * nf)
        self.conv_wgrad(P, c, P["dz_hr"], nf, H.im2col(P["upa"][-1], HL, WL, nf), ML, grads, *bs)
        # upsampling convs, last to first: G = dL/d(post-lrelu output of up[i])
        for i in range(len(self.up) - 1, -1, -1):
            c, (hh, ww), a = self.up[i], P["levels"][i], P["upa"][i]
            Mi = B * hh * ww
            dz = P["dz_hr"][:Mi]
            bs = self.gate_cast(P, G, nf, a, nf, dz, nf, Mi, nf, self.act, self.slope)
            Ghi = P["G_hi"][:Mi]
            self._nt(H.im2col(dz, hh, ww, nf, flip=True), H.rows(c.Wd), H.epilogue(Ghi), Mi, nf, 9 * nf)
            src = P["upa"][i - 1] if i > 0 else P["fea2b"]
            self.conv_wgrad(P, c, dz, nf, H.im2col(src, hh, ww, nf, up=2), Mi, grads, *bs)
            Gn = P["G_lv"][i - 1] if i > 0 else P["Gt"]
            H.sumpool2x(Ghi, nf, Gn, nf, B, hh // 2, ww // 2, nf)
            G = Gn
        # fea2 = fea + trunk_conv(R):  Gt = dL/d fea2
        c = self.trunk
        H.act_grad_cast(P["Gt"], nf, None, 0, P["dzt"], nf, M, nf, 0)
        self._nt(H.im2col(P["dzt"], Hh, Ww, nf, flip=True), H.rows(c.Wd), H.epilogue(P["G_R"]), M, nf, 9 * nf)
        self.conv_wgrad(P, c, P["dzt"], nf, H.im2col(P["dense"][-1], Hh, Ww, nf, ld=CD), M, grads, P["Gt"], nf)
        self._segment_done()   # the tail's gradients are final
        # RRDB trunk, last to first.  G_R = dL/d(RRDB output)
        gy = P["gy"]
        k = self.RRDB_PER_SEGMENT
        for i in range(self.nrr - 1, -1, -1):
            H.act_grad_cast(P["G_R"], nf, None, 0, gy, nf, M, nf, 0, 0.0, 0.2)     # dL/d RDB3 output
            for r in (3 * i + 2, 3 * i + 1, 3 * i):
                self._rdb_bwd(P, r, grads)                                          # gy -> dL/d RDB input
            H.axpby(P["G_R"], gy, 1.0, 1.0)                                          # + skip
            if i % k == 0 and i > 0:
                self._segment_done()   # RRDBs i .. i + k - 1 are final (the first group joins conv_first)
        # conv_first: dL/d fea = Gt (long skip) + G_R (trunk)
        H.axpby(P["G_R"], P["Gt"], 1.0, 1.0)
        H.act_grad_cast(P["G_R"], nf, None, 0, P["dzt"], nf, M, nf, 0)
        c = self.conv_first
        self.conv_wgrad(P, c, P["dzt"], nf, H.im2col(P["xin"], Hh, Ww, self.Cin_p), M, grads, P["G_R"], nf)

    def _rdb_bwd(self, P, r, grads):
        """gy = dL/dy (y = x + 0.2 conv5(...)) -> replaced by dL/dx."""
        cd, nf, gc, CD = self.cd, self.nf, self.gc, self.CD
        Hh, Ww, M = P["H"], P["W"], P["M"]
        cs, D, Gd, gy = self.rdbs[r], P["dense"][r], P["Gd"], P["gy"]
        c = cs[4]
        bs = self.gate_cast(P, gy, nf, None, 0, P["dz5"], nf, M, nf, 0, 0.0, 0.2)
        self._nt(H.im2col(P["dz5"], Hh, Ww, nf, flip=True), H.rows(c.Wd), H.epilogue(Gd), M, CD, 9 * nf)
        self.conv_wgrad(P, c, P["dz5"], nf, H.im2col(D, Hh, Ww, CD, ld=CD), M, grads, *bs)
        for j in range(3, -1, -1):
            c, cin = cs[j], nf + j * gc
            dz = P["dzg"]
            bs = self.gate_cast(P, Gd[:, cin:], CD, D[:, cin:], CD, dz, gc, M, gc, self.act, self.slope)
            self._nt(H.im2col(dz, Hh, Ww, gc, flip=True), H.rows(c.Wd), H.epilogue(Gd, ldo=CD, resid=Gd, ldr=CD), M, cin,
                      9 * gc)
            self.conv_wgrad(P, c, dz, gc, H.im2col(D, Hh, Ww, cin, ld=CD), M, grads, *bs)
        H.axpby_rows(gy, nf, Gd, CD, M, nf, 1.0, 1.0)


class ConvNetFunction(torch.autograd.Function):
    """A whole conv network (RRDBNet / DnCNN / ...) as one autograd node on its step program; the
    node leases its plan from forward to backward (kair_amd/engine/plans.py)."""

    @classmethod
    def run(cls, engine, x, params):
        return cls.apply(engine, autograd_mode(params), x, *params)

    @staticmethod
    def forward(ctx, engine, mode, x, *params):
        with plan_mode(engine, mode):
            E = engine.forward(x.float().contiguous())
        ctx.engine, ctx.params = engine, params
        ctx.lease = Lease(engine.cur) if mode == "lease" else None
        return E.clone()

    @staticmethod
    def backward(ctx, gE):
        eng = ctx.engine
        if ctx.lease is None or ctx.lease.plan is None:
            raise RuntimeError("kair_amd: backward through a forward whose activations were released")
        flat = torch.empty(sum(p.numel() for p in ctx.params), device=gE.device)
        grads, off = {}, 0
        for p in ctx.params:
            grads[p] = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        eng.cur = ctx.lease.plan
        eng.backward_from_grad(gE.float(), grads)
        ctx.lease.release()
        return (None, None, None) + tuple(grads[p] for p in ctx.params)
