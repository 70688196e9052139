"""Generate golden vectors from the reference KAIR code (run in the build container only).

This script imports the reference from /root/reference (read-only) and records inputs/outputs
as small .npz fixtures under tests/golden/.  The reference never travels to the GPU box; only the
fixtures do.  Third-party modules the reference imports but this image lacks (timm, cv2, lpips,
torchvision, pytorch_fid) are replaced by in-process ``sys.modules`` stand-ins; nothing is written
to disk except the fixtures.

  timm.layers stand-in:  DropPath (stochastic depth, identical maths to timm's drop_path),
                         to_2tuple, trunc_normal_ (= torch.nn.init.trunc_normal_).
  Fixtures never rely on DropPath randomness (drop_path_rate=0 or eval mode), so timm's exact
  RNG consumption is irrelevant (SURVEY.md §8c "Third-party arithmetic boundary").

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz, *.json)
"""
import collections.abc
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

REF = os.environ.get("KAIR_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    timm = types.ModuleType("timm")
    layers = types.ModuleType("timm.layers")

    class DropPath(nn.Module):
        def __init__(self, drop_prob=0.0):
            super().__init__()
            self.drop_prob = drop_prob

        def forward(self, x):
            if self.drop_prob == 0.0 or not self.training:
                return x
            keep = 1.0 - self.drop_prob
            shape = (x.shape[0],) + (1,) * (x.ndim - 1)
            return x * x.new_empty(shape).bernoulli_(keep) / keep

    def to_2tuple(x):
        if isinstance(x, collections.abc.Iterable) and not isinstance(x, str):
            return tuple(x)
        return (x, x)

    layers.DropPath = DropPath
    layers.to_2tuple = to_2tuple
    layers.trunc_normal_ = nn.init.trunc_normal_
    timm.layers = layers
    sys.modules["timm"] = timm
    sys.modules["timm.layers"] = layers
    for name in ("cv2", "lpips", "torchvision", "pytorch_fid", "pytorch_fid.fid_score"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["pytorch_fid"].fid_score = sys.modules["pytorch_fid.fid_score"]
    if REF not in sys.path:
        sys.path.insert(0, REF)


def _np(t):
    return t.detach().cpu().numpy().astype(np.float32) if t.is_floating_point() else t.detach().cpu().numpy()


def _save(name, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: v for k, v in arrays.items()})
    print("wrote", path, "%.1f KB" % (os.path.getsize(path) / 1024))


def _fwd_bwd(net, inputs, seed_grad=123):
    """Run forward, inject a seeded upstream grad, return (out, grads dict)."""
    for p in net.parameters():
        p.grad = None
    out = net(*inputs)
    g = torch.Generator().manual_seed(seed_grad)
    gout = torch.randn(out.shape, generator=g)
    out.backward(gout)
    grads = {"grad." + k: _np(p.grad) for k, p in net.named_parameters() if p.grad is not None}
    return out, gout, grads


def _state(net):
    return {"param." + k: _np(v) for k, v in net.state_dict().items()}


def gen_window_attention():
    from models.network_swinir import WindowAttention, SwinTransformerBlock
    torch.manual_seed(0)
    attn = WindowAttention(180, (8, 8), 6)
    with torch.no_grad():
        attn.relative_position_bias_table.normal_(0, 0.5)  # make the bias visible
    blk = SwinTransformerBlock(180, (16, 16), 6, window_size=8, shift_size=4, mlp_ratio=2)
    mask = blk.attn_mask.clone()  # (4, 64, 64) region mask of a shifted 16x16 grid
    torch.manual_seed(1)
    x = torch.randn(4, 64, 180, requires_grad=True)
    res = {}
    for tag, m in (("nomask", None), ("mask", mask)):
        x.grad = None
        for p in attn.parameters():
            p.grad = None
        out = attn(x, m)
        gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(7))
        out.backward(gout)
        res.update({
            f"{tag}.out": _np(out), f"{tag}.gout": _np(gout), f"{tag}.dx": _np(x.grad),
            **{f"{tag}.grad.{k}": _np(p.grad) for k, p in attn.named_parameters()},
        })
    _save("window_attention", x=_np(x), mask=_np(mask),
          rel_index=attn.relative_position_index.numpy(), **_state(attn), **res)


def gen_swin_block():
    from models.network_swinir import SwinTransformerBlock
    res = {}
    for shift in (0, 4):
        torch.manual_seed(10 + shift)
        blk = SwinTransformerBlock(180, (16, 16), 6, window_size=8, shift_size=shift, mlp_ratio=2)
        with torch.no_grad():
            blk.attn.relative_position_bias_table.normal_(0, 0.5)
            blk.norm1.weight.uniform_(0.5, 1.5); blk.norm1.bias.normal_(0, 0.1)
            blk.norm2.weight.uniform_(0.5, 1.5); blk.norm2.bias.normal_(0, 0.1)
        torch.manual_seed(20)
        x = torch.randn(1, 256, 180, requires_grad=True)
        for p in blk.parameters():
            p.grad = None
        out = blk(x, (16, 16))
        gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(8))
        out.backward(gout)
        pre = f"s{shift}."
        res.update({pre + "x": _np(x), pre + "out": _np(out), pre + "gout": _np(gout), pre + "dx": _np(x.grad)})
        res.update({pre + k: v for k, v in _state(blk).items()})
        res.update({pre + "grad." + k: _np(p.grad) for k, p in blk.named_parameters()})
    _save("swin_block", **res)


def _small_swinir(upsampler, upscale, embed=60):
    from models.network_swinir import SwinIR
    return SwinIR(upscale=upscale, in_chans=3, img_size=16, window_size=8, img_range=1.0,
                  depths=[2, 2], embed_dim=embed, num_heads=[6, 6], mlp_ratio=2,
                  upsampler=upsampler, resi_connection="1conv", drop_path_rate=0.0)


def gen_swinir_small():
    res = {}
    for tag, ups, sc in (("classical", "pixelshuffle", 4), ("light", "pixelshuffledirect", 2)):
        torch.manual_seed(30)
        net = _small_swinir(ups, sc)
        net.train()
        torch.manual_seed(31)
        L = torch.rand(2, 3, 16, 16)
        H = torch.rand(2, 3, 16 * sc, 16 * sc)
        for p in net.parameters():
            p.grad = None
        E = net(L)
        loss = nn.L1Loss()(E, H)
        loss.backward()
        pre = tag + "."
        res.update({pre + "L": _np(L), pre + "H": _np(H), pre + "E": _np(E), pre + "loss": np.float32(loss.item())})
        res.update({pre + k: v for k, v in _state(net).items()})
        res.update({pre + "grad." + k: _np(p.grad) for k, p in net.named_parameters()})
    _save("swinir_small", **res)


def gen_swinir_variants():
    """The reference's other reconstruction heads and residual connection (network_swinir.py:
    464-471 / 727-737 '3conv', :751-760 / 824-830 'nearest+conv', :761-763 / 831-835 upsampler None:
    denoising / JPEG, with img_range 255 as in options/swinir/train_swinir_car_jpeg.json)."""
    from models.network_swinir import SwinIR
    cfgs = (("realsr3", dict(upscale=4, in_chans=3, img_range=1.0, upsampler="nearest+conv", resi_connection="3conv")),
            ("dngray", dict(upscale=1, in_chans=1, img_range=1.0, upsampler=None, resi_connection="1conv")),
            ("car255", dict(upscale=1, in_chans=3, img_range=255.0, upsampler="", resi_connection="3conv")))
    res = {}
    for i, (tag, kw) in enumerate(cfgs):
        torch.manual_seed(40 + i)
        net = SwinIR(img_size=16, window_size=8, depths=[2], embed_dim=60, num_heads=[6], mlp_ratio=2,
                     drop_path_rate=0.0, **kw)
        net.train()
        torch.manual_seed(50 + i)
        sc, ci = kw["upscale"], kw["in_chans"]
        L = torch.rand(2, ci, 16, 16)
        H = torch.rand(2, ci, 16 * sc, 16 * sc)
        for p in net.parameters():
            p.grad = None
        E = net(L)
        loss = nn.L1Loss()(E, H)
        loss.backward()
        pre = tag + "."
        res.update({pre + "L": _np(L), pre + "H": _np(H), pre + "E": _np(E), pre + "loss": np.float32(loss.item())})
        res.update({pre + k: v for k, v in _state(net).items()})
        res.update({pre + "grad." + k: _np(p.grad) for k, p in net.named_parameters()})
    _save("swinir_variants", **res)


def _opt_dict(netG, train_over=None, E_decay=0.999):
    opt = {
        "model": "plain", "gpu_ids": None, "dist": False, "is_train": True, "scale": netG.get("upscale", 1),
        "path": {"models": "/tmp/_golden_models", "pretrained_netG": None, "pretrained_netE": None,
                 "pretrained_optimizerG": None},
        "netG": netG,
        "train": {"G_lossfn_type": "l1", "G_lossfn_weight": 1.0, "E_decay": E_decay,
                  "G_optimizer_type": "adam", "G_optimizer_lr": 2e-4, "G_optimizer_wd": 0,
                  "G_optimizer_betas": [0.9, 0.999], "G_optimizer_clipgrad": None,
                  "G_optimizer_reuse": True, "G_scheduler_type": "MultiStepLR",
                  "G_scheduler_milestones": [2, 100], "G_scheduler_gamma": 0.5,
                  "G_regularizer_orthstep": None, "G_regularizer_clipstep": None,
                  "G_param_strict": True, "E_param_strict": True, "checkpoint_save": 5000,
                  "lpips_net": "alex"},
    }
    opt["train"].update(train_over or {})
    return opt


def gen_train_trajectory():
    """3 steps of the reference ModelPlain.optimize_parameters on a tiny SwinIR (DropPath off)."""
    import models.network_swinir as ns
    from models.model_plain import ModelPlain
    netG = {"net_type": "swinir", "upscale": 4, "in_chans": 3, "img_size": 16, "window_size": 8,
            "img_range": 1.0, "depths": [2, 2], "embed_dim": 60, "num_heads": [6, 6], "mlp_ratio": 2,
            "upsampler": "pixelshuffle", "resi_connection": "1conv", "init_type": "default"}
    orig_init = ns.SwinIR.__init__

    def init_nodrop(self, *a, **k):
        k["drop_path_rate"] = 0.0
        orig_init(self, *a, **k)
    ns.SwinIR.__init__ = init_nodrop
    os.makedirs("/tmp/_golden_models", exist_ok=True)
    try:
        from utils.utils_option import dict_to_nonedict
        torch.manual_seed(40)
        model = ModelPlain(dict_to_nonedict(_opt_dict(netG)))
        model.init_train()
    finally:
        ns.SwinIR.__init__ = orig_init
    bare = model.get_bare_model(model.netG)
    res = {"init." + k: v for k, v in _state(bare).items()}
    torch.manual_seed(41)
    losses, lrs = [], []
    for step in range(1, 4):
        L = torch.rand(2, 3, 16, 16)
        H = torch.rand(2, 3, 64, 64)
        res[f"step{step}.L"] = _np(L)
        res[f"step{step}.H"] = _np(H)
        model.update_learning_rate(step)      # main_train_psnr.py:176 order: scheduler before step
        model.feed_data({"L": L, "H": H})
        model.optimize_parameters(step)
        losses.append(model.log_dict["G_loss"])
        lrs.append(model.current_learning_rate())
    res["losses"] = np.array(losses, np.float64)
    res["lrs"] = np.array(lrs, np.float64)
    res.update({"final.G." + k: v for k, v in _state(bare).items()})
    res.update({"final.E." + k: v for k, v in _state(model.netE).items()})
    _save("train_trajectory", **res)


def gen_conv_nets():
    from models.network_dncnn import DnCNN
    from models.network_rrdbnet import RRDBNet
    from models.network_rrdb import RRDB
    res = {}
    # DnCNN with BN in train mode (batch statistics + running-stat update, momentum 0.9, eps 1e-4)
    torch.manual_seed(50)
    net = DnCNN(1, 1, 64, 5, "BR")
    from models.select_network import init_weights
    init_weights(net, init_type="orthogonal", init_bn_type="uniform", gain=0.2)
    net.train()
    torch.manual_seed(51)
    x = torch.rand(4, 1, 20, 20)
    res.update({"dncnn." + k: v for k, v in _state(net).items()})  # pre-step state incl. running stats
    out, gout, grads = _fwd_bwd(net, (x,))
    res.update({"dncnn.x": _np(x), "dncnn.out": _np(out), "dncnn.gout": _np(gout)})
    res.update({"dncnn." + k: v for k, v in grads.items()})
    res.update({"dncnn.after." + k: _np(v) for k, v in net.state_dict().items() if "running" in k})
    # RRDBNet (ESRGAN generator), reduced depth
    torch.manual_seed(52)
    net = RRDBNet(3, 3, 32, 1, 16, 4)
    torch.manual_seed(53)
    x = torch.rand(2, 3, 12, 12)
    res.update({"rrdbnet." + k: v for k, v in _state(net).items()})
    out, gout, grads = _fwd_bwd(net, (x,))
    res.update({"rrdbnet.x": _np(x), "rrdbnet.out": _np(out), "rrdbnet.gout": _np(gout)})
    res.update({"rrdbnet." + k: v for k, v in grads.items()})
    # RRDB (option 'rrdb': basicblock RRDB trunk, upconv upsampler), reduced depth, act 'R'
    torch.manual_seed(54)
    net = RRDB(3, 3, 32, 1, 16, 4, "R", "upconv")
    init_weights(net, init_type="orthogonal", init_bn_type="uniform", gain=0.2)
    torch.manual_seed(55)
    x = torch.rand(2, 3, 12, 12)
    res.update({"rrdb." + k: v for k, v in _state(net).items()})
    out, gout, grads = _fwd_bwd(net, (x,))
    res.update({"rrdb.x": _np(x), "rrdb.out": _np(out), "rrdb.gout": _np(gout)})
    res.update({"rrdb." + k: v for k, v in grads.items()})
    _save("conv_nets", **res)


def gen_usrnet():
    from models.network_usrnet_v1 import USRNet, DataNet, p2o, upsample
    torch.manual_seed(60)
    net = USRNet(n_iter=2, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2, act_mode="R",
                 downsample_mode="strideconv", upsample_mode="convtranspose")
    from models.select_network import init_weights
    init_weights(net, init_type="orthogonal", init_bn_type="uniform", gain=0.2)
    torch.manual_seed(61)
    x = torch.rand(1, 3, 16, 16)
    k = torch.rand(1, 1, 25, 25)
    k = k / k.sum()
    sigma = torch.full((1, 1, 1, 1), 10.0 / 255)
    res = {"x": _np(x), "k": _np(k), "sigma": _np(sigma), "sf": np.int64(4)}
    res.update(_state(net))
    for p in net.parameters():
        p.grad = None
    out = net(x, k, 4, sigma)
    gout = torch.randn(out.shape, generator=torch.Generator().manual_seed(9))
    out.backward(gout)
    res.update({"out": _np(out), "gout": _np(gout)})
    res.update({"grad." + n: _np(p.grad) for n, p in net.named_parameters() if p.grad is not None})
    # DataNet alone at a 64x64 HR grid
    torch.manual_seed(62)
    FB = p2o(k, (64, 64))
    FBC = torch.conj(FB)
    F2B = torch.pow(torch.abs(FB), 2)
    y = torch.rand(1, 3, 16, 16)
    STy = upsample(y, sf=4)
    FBFy = FBC * torch.fft.fftn(STy, dim=(-2, -1))
    xin = torch.rand(1, 3, 64, 64)
    alpha = torch.full((1, 1, 1, 1), 0.05)
    z = DataNet()(xin, FB, FBC, F2B, FBFy, alpha, 4)
    res.update({"datanet.y": _np(y), "datanet.x": _np(xin), "datanet.alpha": _np(alpha), "datanet.z": _np(z),
                "datanet.FB_re": _np(FB.real), "datanet.FB_im": _np(FB.imag)})
    _save("usrnet", **res)


def gen_image_utils():
    import utils.utils_image as util
    torch.manual_seed(70)
    img = torch.rand(3, 48, 48)
    img2 = torch.rand(3, 40, 40)
    lr4 = util.imresize(img.clone(), 1 / 4, True)
    lr2 = util.imresize(img.clone(), 1 / 2, True)
    lr3 = util.imresize(img2.clone(), 1 / 3, True)
    up2 = util.imresize(img2.clone(), 2, True)
    gray = util.imresize(img2[0].clone(), 1 / 2, True)
    a = torch.rand(3, 32, 32)
    b = (a + 0.03 * torch.randn(3, 32, 32)).clamp(0, 1)
    ua, ub = util.tensor2uint(a), util.tensor2uint(b)
    psnr0 = util.calculate_psnr(ua, ub, border=0)
    psnr4 = util.calculate_psnr(ua, ub, border=4)
    _save("image_utils", img=_np(img), img2=_np(img2), lr4=_np(lr4), lr2=_np(lr2), lr3=_np(lr3), up2=_np(up2),
          gray=_np(gray), a=_np(a), b=_np(b), ua=ua, ub=ub, psnr0=np.float64(psnr0), psnr4=np.float64(psnr4))


def gen_dncnn_kat():
    """KAT: model_zoo/dncnn_25.pth on utils/test.bmp (PIL grayscale for cv2.imread(...,0)), sigma 25,
    np.random.seed(0) noise (main_test_dncnn.py semantics)."""
    from PIL import Image
    from models.network_dncnn import DnCNN
    import utils.utils_image as util
    net = DnCNN(1, 1, 64, 17, "R")
    sd = torch.load(os.path.join(REF, "model_zoo/dncnn_25.pth"), weights_only=True, map_location="cpu")
    net.load_state_dict(sd, strict=True)
    net.eval()
    img_H = np.array(Image.open(os.path.join(REF, "utils/test.bmp")).convert("L"))
    img_L = util.uint2single(img_H)[..., None]
    np.random.seed(seed=0)
    img_L = img_L + np.random.normal(0, 25 / 255.0, img_L.shape)
    Lt = util.single2tensor4(img_L)
    with torch.no_grad():
        E = net(Lt)
    E_u = util.tensor2uint(E)
    psnr_noisy = util.calculate_psnr(util.single2uint(img_L.squeeze()), img_H)
    psnr_den = util.calculate_psnr(E_u, img_H)
    print("DnCNN KAT noisy %.4f denoised %.4f" % (psnr_noisy, psnr_den))
    # the pretrained weights themselves (weights-only load above), so the HIP DnCNN can run the KAT
    # on the GPU box where the reference does not exist: keys "w/<state_dict key>"
    weights = {"w/" + k: _np(v) for k, v in sd.items()}
    _save("dncnn_kat", img_H=img_H, img_L=img_L.astype(np.float32).squeeze(), E=_np(E).squeeze(),
          psnr_noisy=np.float64(psnr_noisy), psnr_denoised=np.float64(psnr_den), **weights)


def gen_state_dict_layouts():
    """Key names / shapes / dtypes of define_G networks at the FULL option-file configs."""
    from models.select_network import define_G
    import models.network_swinir as ns  # noqa: F401
    cfgs = {
        "swinir_classical_x4": {"net_type": "swinir", "upscale": 4, "in_chans": 3, "img_size": 48,
                                "window_size": 8, "img_range": 1.0, "depths": [6] * 6, "embed_dim": 180,
                                "num_heads": [6] * 6, "mlp_ratio": 2, "upsampler": "pixelshuffle",
                                "resi_connection": "1conv", "init_type": "default"},
        "swinir_light_x2": {"net_type": "swinir", "upscale": 2, "in_chans": 3, "img_size": 64,
                            "window_size": 8, "img_range": 1.0, "depths": [6] * 4, "embed_dim": 60,
                            "num_heads": [6] * 4, "mlp_ratio": 2, "upsampler": "pixelshuffledirect",
                            "resi_connection": "1conv", "init_type": "default"},
        "dncnn": {"net_type": "dncnn", "in_nc": 1, "out_nc": 1, "nc": 64, "nb": 17, "act_mode": "BR",
                  "init_type": "orthogonal", "init_bn_type": "uniform", "init_gain": 0.2},
        "rrdb": {"net_type": "rrdb", "in_nc": 3, "out_nc": 3, "nc": 64, "nb": 23, "gc": 32, "scale": 4,
                 "act_mode": "R", "upsample_mode": "upconv", "init_type": "orthogonal",
                 "init_bn_type": "uniform", "init_gain": 0.2},
        "rrdbnet": {"net_type": "rrdbnet", "in_nc": 3, "out_nc": 3, "nf": 64, "nb": 23, "gc": 32, "scale": 4,
                    "init_type": "default"},
    }
    out = {}
    for name, netG in cfgs.items():
        net = define_G({"netG": netG, "is_train": False})
        out[name] = {"keys": [[k, list(v.shape), str(v.dtype).replace("torch.", "")]
                              for k, v in net.state_dict().items()],
                     "n_params": int(sum(p.numel() for p in net.parameters()))}
    # USRNet option file binds the legacy module; v1 has the identical parameter layout
    from models.network_usrnet_v1 import USRNet
    net = USRNet(n_iter=6, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2, act_mode="R",
                 downsample_mode="strideconv", upsample_mode="convtranspose")
    out["usrnet"] = {"keys": [[k, list(v.shape), str(v.dtype).replace("torch.", "")]
                              for k, v in net.state_dict().items()],
                     "n_params": int(sum(p.numel() for p in net.parameters()))}
    path = os.path.join(OUT, "state_dict_layouts.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print("wrote", path)


if __name__ == "__main__":
    _install_stubs()
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["window_attention", "swin_block", "swinir_small", "train_trajectory",
                             "conv_nets", "usrnet", "swinir_variants", "image_utils", "dncnn_kat", "state_dict_layouts"]
    for w in which:
        globals()["gen_" + w]()
