"""kair_conv3x3_wr (csrc/conv_wr.hip): the 3x3 conv with register-streamed weights that runs the SwinIR
RSTB convs (network_swinir.py:263-279) and their input gradients, against float64 torch:
  * split: fp32 image, hi/lo split weights (pack kind 15) and split activations -> ~2^-16 relative
    (vs ~2^-9 for a plain bf16 product), with bias, fp32 residual and the bf16 a_copy of the image;
  * plain: bf16 image with flipped taps over the dgrad-form weight (pack kind 16) = conv_transpose2d,
    fp32 and bf16 outputs, 144-pixel tiles;
  * geometry: rows wider than the tile (row pieces), several images per tile, N < 192."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from kair_amd import _hip as H  # noqa: E402

dev = torch.device("cuda")
F = torch.nn.functional


def rel_err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def nchw(rows, B, Hh, Ww, C):
    return rows.cpu().view(B, Hh, Ww, -1)[..., :C].permute(0, 3, 1, 2)


@pytest.mark.parametrize("shape", [(2, 48, 48, 180, 180), (1, 8, 192, 128, 192), (3, 16, 24, 128, 64), (2, 24, 24, 180, 192),
                                   (8, 48, 48, 180, 180)])
def test_conv_wr_split(shape):
    B, Hh, Ww, C, N = shape
    Cp = (C + 63) // 64 * 64
    # 96-pixel tiles once there are >= 3/4 of a tile per CU (B = 8 here), else 48 (the small batches)
    assert H.conv3x3_wr_tile(1, B, Hh, Ww, Cp, N) in (48, 96)
    g = torch.Generator().manual_seed(C + N + Ww)
    x = torch.randn(B, C, Hh, Ww, generator=g)
    w = torch.randn(N, C, 3, 3, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    M = B * Hh * Ww
    r = torch.randn(M, N, generator=g)
    ref = F.conv2d(x.double(), w.double(), bias.double(), padding=1) + r.double().view(B, Hh, Ww, N).permute(0, 3, 1, 2)
    xin = torch.zeros(M, Cp)
    xin[:, :C] = x.permute(0, 2, 3, 1).reshape(M, C)
    xin = xin.to(dev)
    Wf = torch.empty(192 * 2 * 9 * Cp, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), Wf, H.wmap(15, N, C, (1, N, 192), (1, C, Cp)))
    bp = torch.zeros(192, device=dev)
    bp[:N] = bias.to(dev)
    out = torch.full((M, N), float("nan"), device=dev)
    ac = torch.full((M, Cp), float("nan"), device=dev, dtype=torch.bfloat16)
    H.conv3x3_wr(xin, Cp, 0, Wf, bp, r.to(dev), out, B, Hh, Ww, Cp, N, acopy=ac, acones=C if C < Cp else -1)
    torch.cuda.synchronize()
    assert rel_err(nchw(out, B, Hh, Ww, N), ref) < 3e-5
    # a_copy: the bf16 (hi) image with 1.0 in the ones column
    exp = xin.bfloat16().cpu()
    if C < Cp:
        exp[:, C] = 1.0
    assert torch.equal(ac.cpu(), exp)


@pytest.mark.parametrize("shape,odt,xdt", [((2, 48, 48, 192, 180), torch.float32, torch.bfloat16),
                                           ((2, 48, 48, 192, 192), torch.bfloat16, torch.bfloat16),
                                           ((1, 16, 96, 192, 192), torch.float32, torch.bfloat16),
                                           ((2, 48, 48, 192, 192), torch.float32, torch.float32),
                                           ((2, 24, 24, 192, 192), torch.float32, torch.float32),
                                           ((12, 48, 48, 192, 180), torch.float32, torch.bfloat16)])
def test_conv_wr_dgrad(shape, odt, xdt):
    """input gradient of a forward conv Cin=N_out -> Cout=C: dX = conv_transpose(G, w) over the image G
    (bf16 rows, or fp32 rows rounded to bf16 in the halo fill, with their bf16 copy left in a_copy)"""
    B, Hh, Ww, C, N = shape
    g = torch.Generator().manual_seed(C + N + Ww + 1)
    G = torch.randn(B, C, Hh, Ww, generator=g).bfloat16().float()
    w = (torch.randn(C, N, 3, 3, generator=g) * 0.05).bfloat16().float()   # forward conv N -> C
    ref = F.conv_transpose2d(G.double(), w.double(), padding=1)          # [B, N, H, W]
    M = B * Hh * Ww
    gin = G.permute(0, 2, 3, 1).reshape(M, C).to(dev, xdt).contiguous()
    Wd = torch.empty(192 * 9 * C, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), Wd, H.wmap(16, C, N, (1, C, C), (1, N, 192)))
    tile = H.conv3x3_wr_tile(0, B, Hh, Ww, C, N)
    assert tile in (48, 96, 144)
    out = torch.full((M, N), float("nan"), device=dev, dtype=odt)
    ac = torch.full((M, C), float("nan"), device=dev, dtype=torch.bfloat16) if xdt == torch.float32 else None
    H.conv3x3_wr(gin, C, 1, Wd, None, None, out, B, Hh, Ww, C, N, acopy=ac, split=False)
    torch.cuda.synchronize()
    assert rel_err(nchw(out.float(), B, Hh, Ww, N), ref) < (1e-5 if odt == torch.float32 else 4e-3)
    if ac is not None:
        assert torch.equal(ac.cpu(), gin.bfloat16().cpu())


@pytest.mark.parametrize("hw", [(24, 48), (8, 96)])
def test_conv_wr_pair_pshuf(hw):
    """The x4 upsampling conv under split activations: a bf16 [hi | lo] pair image of 64 channels (two
    halos), 64 -> 256 with hi/lo split weights (kind 15, Np = 256, sub-pixel-major rows), PixelShuffle(2)
    store of a [hi | lo] pair (out_lo) -> ~2^-16 of the fp64 conv + pixel_shuffle."""
    B, r = 2, 2
    Hh, Ww = hw
    g = torch.Generator().manual_seed(Hh + Ww)
    x = torch.randn(B, 64, Hh, Ww, generator=g)
    w = torch.randn(256, 64, 3, 3, generator=g) * 0.05
    b = torch.randn(256, generator=g) * 0.1
    ref = F.pixel_shuffle(F.conv2d(x.double(), w.double(), b.double(), padding=1), r)   # [B, 64, 2H, 2W]
    M = B * Hh * Ww
    rows = x.permute(0, 2, 3, 1).reshape(M, 64)
    hi = rows.bfloat16()
    lo = (rows - hi.float()).bfloat16()
    pair = torch.cat([hi, lo], 1).contiguous().to(dev)
    Wf = torch.empty(256 * 2 * 9 * 64, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), Wf, H.wmap(15, 256, 64, (1, 256, 256), (1, 64, 64), n_perm=r * r))
    bp = torch.empty(256, device=dev)
    H.pack_weight(b.to(dev), bp, H.wmap(4, 256, 0, (1, 256, 256), (1, 1, 1), n_perm=r * r))
    out = torch.full((M * r * r, 128), float("nan"), device=dev, dtype=torch.bfloat16)
    assert H.conv3x3_wr_tile(1, B, Hh, Ww, 64, 256) in (48, 96)
    H.conv3x3_wr(pair, 128, 0, Wf, bp, None, out, B, Hh, Ww, 64, 256, ldo=128, split=True, out_lo=out[:, 64:], ps_r=r)
    torch.cuda.synchronize()
    got = (out[:, :64].double() + out[:, 64:].double()).cpu().view(B, Hh * r, Ww * r, 64).permute(0, 3, 1, 2)
    assert rel_err(got, ref) < 3e-5


def test_conv_wr_cbu_leaky_pair():
    """conv_before_upsample (network_swinir.py:742) under split activations: fp32 image of 180 channels
    (padded 192), 180 -> 64 with split weights (kind 15, Np = 64), LeakyReLU(0.01), stored as a bf16
    [hi | lo] pair (out_lo) -> ~2^-16 of fp64."""
    B, Hh, Ww, C, N = 2, 48, 48, 180, 64
    g = torch.Generator().manual_seed(44)
    x = torch.randn(B, C, Hh, Ww, generator=g)
    w = torch.randn(N, C, 3, 3, generator=g) * 0.05
    b = torch.randn(N, generator=g) * 0.1
    ref = F.leaky_relu(F.conv2d(x.double(), w.double(), b.double(), padding=1), 0.01)
    M = B * Hh * Ww
    xin = torch.zeros(M, 192)
    xin[:, :C] = x.permute(0, 2, 3, 1).reshape(M, C)
    Wc = torch.empty(64 * 2 * 9 * 192, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), Wc, H.wmap(15, N, C, (1, N, 64), (1, C, 192)))
    out = torch.full((M, 128), float("nan"), device=dev, dtype=torch.bfloat16)
    H.conv3x3_wr(xin.to(dev), 192, 0, Wc, b.to(dev), None, out, B, Hh, Ww, 192, N, ldo=128, split=True,
                 out_lo=out[:, 64:], act=H.ACT_LEAKY, slope=0.01)
    torch.cuda.synchronize()
    got = (out[:, :64].double() + out[:, 64:].double()).cpu().view(B, Hh, Ww, N).permute(0, 3, 1, 2)
    assert rel_err(got, ref) < 3e-5


@pytest.mark.parametrize("mode,hw,B", [("punshuf", (24, 96), 2), ("gate", (24, 48), 2), ("punshuf", (48, 48), 2),
                                       ("punshuf", (96, 96), 4), ("gate", (48, 48), 16)])
def test_conv_wr_ups_dgrad(mode, hw, B):
    """The upsampling convs' input gradients (network_swinir.py:584 Upsample, its backward): the 256-channel
    pre-shuffle gradient (bf16) through kind-16 weights (rows = the 64 input channels, columns
    sub-pixel-major), stored PixelUnshuffle(2)-ed into the previous conv's pre-shuffle rows, or gated
    by LeakyReLU'(a0) of the stored [hi | lo] activation -- vs fp64 conv_transpose2d."""
    C, N = 256, 64
    Hh, Ww = hw
    # (96, 96) x 4 has enough pixels for the 192-pixel tile in two channel-half passes (rows of >= 96)
    assert H.conv3x3_wr_tile(0, B, Hh, Ww, C, N) == (192 if B * Hh * Ww >= 36864 and Ww >= 96 else
                                                     96 if B * Hh * Ww >= 18432 else 48)
    g = torch.Generator().manual_seed(31 + Hh)
    x = torch.randn(B, C, Hh, Ww, generator=g).bfloat16().float()
    w = (torch.randn(C, N, 3, 3, generator=g) * 0.03).bfloat16().float()   # forward conv N -> C
    ref = F.conv_transpose2d(x.double(), w.double(), padding=1)            # [B, N, H, W]
    M = B * Hh * Ww
    xin = x.permute(0, 2, 3, 1).contiguous().view(M, C).to(dev, torch.bfloat16)
    Wd = torch.empty(N * 9 * C, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w.to(dev), Wd, H.wmap(16, C, N, (1, C, C), (1, N, N)))
    if mode == "punshuf":
        r = 2
        out = torch.full((M // (r * r), r * r * N), float("nan"), device=dev, dtype=torch.bfloat16)
        H.conv3x3_wr(xin, C, 1, Wd, None, None, out, B, Hh, Ww, C, N, ldo=r * r * N, split=False, ps_r=-r)
        torch.cuda.synchronize()
        got = out.float().cpu().view(B, Hh // r, Ww // r, r, r, N).permute(0, 5, 1, 3, 2, 4).reshape(B, N, Hh, Ww)
    else:
        gate = torch.randn(M, 128, generator=g).bfloat16()
        out = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        H.conv3x3_wr(xin, C, 1, Wd, None, None, out, B, Hh, Ww, C, N, split=False, gate=gate.to(dev), ldg=128, slope=0.01)
        torch.cuda.synchronize()
        got = out.float().cpu().view(B, Hh, Ww, N).permute(0, 3, 1, 2)
        gs = torch.where(gate[:, :N].float() > 0, 1.0, 0.01).view(B, Hh, Ww, N).permute(0, 3, 1, 2)
        ref = ref * gs.double()
    assert rel_err(got, ref) < 4e-3   # bf16 output


def test_conv_wr_rejects():
    x = torch.zeros(2 * 48 * 48, 192, device=dev)
    w = torch.zeros(192 * 2 * 9 * 192, device=dev, dtype=torch.bfloat16)
    out = torch.empty(2 * 48 * 48, 192, device=dev)
    assert H.conv3x3_wr_tile(1, 2, 48, 50, 192, 192) == 0          # 96 % 50 != 0
    with pytest.raises(RuntimeError):
        H.conv3x3_wr(x, 192, 0, w, None, None, out, 2, 48, 50, 192, 192)
    with pytest.raises(RuntimeError):   # C must be a multiple of 64
        H.conv3x3_wr(x, 192, 0, w, None, None, out, 2, 48, 48, 180, 192)
    with pytest.raises(RuntimeError):   # 192 packed rows
        H.conv3x3_wr(x, 192, 0, w, None, None, out, 2, 48, 48, 192, 192, n_blocks=4)


def test_engine_conv_wr_matches_halo():
    """SwinIR classical (embed 180) through the engine with the RSTB / conv_after_body convs on kair_conv3x3_wr
    (forced on at a small batch) against the same engine on the LDS-ring halo kernel: the same three
    products per output summed in another order, so the outputs agree to fp32 summation noise; the
    gradients then differ by bf16 operand-rounding flips downstream (~0.4 %), so both are held against
    the exact-fp32 engine on the same weights and the wr engine must be as close to it as the halo one."""
    from kair_amd.models.network_swinir import SwinIR
    from kair_amd.engine.swinir_engine import SwinIREngine
    torch.manual_seed(3)
    net = SwinIR(upscale=2, in_chans=3, img_size=24, window_size=8, img_range=1.0, depths=[2, 2], embed_dim=180,
                 num_heads=[6, 6], mlp_ratio=2, upsampler="pixelshuffle", drop_path_rate=0.0,
                 compute_dtype="bf16").to(dev).train()
    engs = []
    for wr in (True, False):
        e = SwinIREngine(net, "bf16", side_stream=False, conv_wr=wr)
        e.conv_wr_min_tiles = 0
        engs.append(e)
    engs.append(SwinIREngine(net, "fp32", side_stream=False))
    g = torch.Generator().manual_seed(4)
    x = torch.rand(2, 3, 24, 24, generator=g).to(dev)
    gE = None
    outs, grads = [], []
    params = list(net.parameters())
    for k, e in enumerate(engs):
        E = e.forward(x).clone()
        if k < 2:
            assert e.cur["conv_wr"] == e.conv_wr
        if gE is None:
            gE = torch.randn(E.shape, generator=g).to(dev)
        flat = torch.zeros(sum(p.numel() for p in params), device=dev)
        gd, off = {}, 0
        for p in params:
            gd[p] = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        e.backward_from_grad(gE, gd)
        torch.cuda.synchronize()
        outs.append(E)
        grads.append(flat.clone())
    assert rel_err(outs[0], outs[1]) < 1e-5
    ew, eh = rel_err(grads[0], grads[2]), rel_err(grads[1], grads[2])
    assert ew < 1.2 * eh + 1e-3 and ew < 2e-2, (ew, eh)


def test_halo_dgrad_acopy_matches_wr():
    """The LDS-ring halo kernel's input gradient over an fp32 G with a_copy (the engine's other path) leaves
    the same bf16 copy of G and the same dX as kair_conv3x3_wr."""
    B, Hh, Ww, C = 2, 24, 24, 192
    M = B * Hh * Ww
    g = torch.Generator().manual_seed(12)
    G = torch.randn(M, C, generator=g).to(dev)
    w = torch.randn(180, 180, 3, 3, generator=g).to(dev) * 0.05
    Wd = torch.empty(C, 9 * C, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w, Wd, H.wmap(2, 180, 180, (1, 180, C), (1, 180, C)))
    Wd16 = torch.empty(C * 9 * C, device=dev, dtype=torch.bfloat16)
    H.pack_weight(w, Wd16, H.wmap(16, 180, 180, (1, 180, C), (1, 180, C)))
    outs, acs = [], []
    for wr in (False, True):
        D = torch.full((M, C), float("nan"), device=dev)
        ac = torch.full((M, C), float("nan"), device=dev, dtype=torch.bfloat16)
        if wr:
            H.conv3x3_wr(G, C, 1, Wd16, None, None, D, B, Hh, Ww, C, C, acopy=ac, split=False)
        else:
            H.gemm_nt(H.im2col(G, Hh, Ww, C, flip=True), H.rows(Wd), H.epilogue(D, acopy=(ac, -1)), M, C, 9 * C, H.BF16)
        torch.cuda.synchronize()
        outs.append(D)
        acs.append(ac)
    assert torch.equal(acs[1].cpu(), G.bfloat16().cpu())
    assert torch.equal(acs[0].cpu(), G.bfloat16().cpu())
    assert rel_err(outs[0], outs[1]) < 1e-6
