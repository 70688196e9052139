"""Pin the CPU oracle against golden vectors produced by the reference itself (tests/golden/)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden, sub_grads, sub_state
from oracle import convnets, image, swinir
from oracle.train import OracleTrainer


def close(a, b, rtol=1e-4, atol=1e-5):
    a = a.detach().numpy() if torch.is_tensor(a) else a
    b = b.detach().numpy() if torch.is_tensor(b) else b
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


@pytest.mark.parametrize("tag", ["nomask", "mask"])
def test_window_attention(tag):
    z = load_golden("window_attention")
    m = swinir.WindowAttention(180, 8, 6)
    m.load_state_dict(sub_state(z, ""), strict=True)
    np.testing.assert_array_equal(swinir.relative_position_index(8).numpy(), z["rel_index"])
    x = torch.from_numpy(z["x"]).requires_grad_(True)
    mask = torch.from_numpy(z["mask"]) if tag == "mask" else None
    out = m(x, mask)
    close(out, z[f"{tag}.out"])
    out.backward(torch.from_numpy(z[f"{tag}.gout"]))
    close(x.grad, z[f"{tag}.dx"])
    for k, p in m.named_parameters():
        close(p.grad, z[f"{tag}.grad.{k}"], rtol=1e-4, atol=1e-4)


def test_shift_mask_matches_reference():
    z = load_golden("window_attention")
    np.testing.assert_array_equal(swinir.shift_region_mask(16, 16, 8, 4).numpy(), z["mask"])


@pytest.mark.parametrize("shift", [0, 4])
def test_swin_block(shift):
    z = load_golden("swin_block")
    pre = f"s{shift}."
    blk = swinir.SwinTransformerBlock(180, (16, 16), 6, 8, shift, 2)
    blk.load_state_dict(sub_state(z, pre), strict=True)
    x = torch.from_numpy(z[pre + "x"]).requires_grad_(True)
    out = blk(x, (16, 16))
    close(out, z[pre + "out"])
    out.backward(torch.from_numpy(z[pre + "gout"]))
    close(x.grad, z[pre + "dx"], atol=1e-4)
    g = sub_grads(z, pre)
    for k, p in blk.named_parameters():
        close(p.grad, g[k], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("tag,ups,sc", [("classical", "pixelshuffle", 4), ("light", "pixelshuffledirect", 2)])
def test_swinir_small(tag, ups, sc):
    z = load_golden("swinir_small")
    pre = tag + "."
    net = swinir.SwinIR(upscale=sc, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2, 2],
                        embed_dim=60, num_heads=[6, 6], mlp_ratio=2, upsampler=ups)
    net.load_state_dict(sub_state(z, pre), strict=True)
    E = net(torch.from_numpy(z[pre + "L"]))
    close(E, z[pre + "E"])
    loss = torch.nn.functional.l1_loss(E, torch.from_numpy(z[pre + "H"]))
    assert abs(loss.item() - float(z[pre + "loss"])) < 1e-6
    loss.backward()
    g = sub_grads(z, pre)
    for k, p in net.named_parameters():
        close(p.grad, g[k], rtol=2e-3, atol=2e-5)


VARIANTS = {   # tests/golden/make_golden.py gen_swinir_variants
    "realsr3": dict(upscale=4, in_chans=3, img_range=1.0, upsampler="nearest+conv", resi_connection="3conv"),
    "dngray": dict(upscale=1, in_chans=1, img_range=1.0, upsampler=None, resi_connection="1conv"),
    "car255": dict(upscale=1, in_chans=3, img_range=255.0, upsampler="", resi_connection="3conv"),
}


@pytest.mark.parametrize("tag", sorted(VARIANTS))
def test_swinir_variants(tag):
    """'nearest+conv' / no-upsampler heads, '3conv' residual connections, img_range 255."""
    z = load_golden("swinir_variants")
    pre = tag + "."
    net = swinir.SwinIR(img_size=16, window_size=8, depths=[2], embed_dim=60, num_heads=[6], mlp_ratio=2,
                        **VARIANTS[tag])
    net.load_state_dict(sub_state(z, pre), strict=True)
    E = net(torch.from_numpy(z[pre + "L"]))
    close(E, z[pre + "E"])
    loss = torch.nn.functional.l1_loss(E, torch.from_numpy(z[pre + "H"]))
    assert abs(loss.item() - float(z[pre + "loss"])) < 1e-6
    loss.backward()
    g = sub_grads(z, pre)
    for k, p in net.named_parameters():
        close(p.grad, g[k], rtol=2e-3, atol=2e-5)


def test_train_trajectory():
    """3 reference ModelPlain steps (MultiStepLR before step, Adam, EMA 0.999)."""
    z = load_golden("train_trajectory")
    mk = lambda: swinir.SwinIR(upscale=4, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2, 2],
                               embed_dim=60, num_heads=[6, 6], mlp_ratio=2, upsampler="pixelshuffle")
    net, ema = mk(), mk()
    net.load_state_dict(sub_state(z, "init."), strict=True)
    ema.load_state_dict(sub_state(z, "init."), strict=True)
    tr = OracleTrainer(net, ema, lr=2e-4, milestones=[2, 100], gamma=0.5, E_decay=0.999)
    losses, lrs = [], []
    for s in range(1, 4):
        tr.update_learning_rate()
        _, loss = tr.optimize_parameters(torch.from_numpy(z[f"step{s}.L"]), torch.from_numpy(z[f"step{s}.H"]))
        losses.append(loss)
        lrs.append(tr.lr)
    np.testing.assert_allclose(losses, z["losses"], rtol=1e-5)
    np.testing.assert_allclose(lrs, z["lrs"], rtol=1e-12)
    fg = sub_state(z, "final.G.")
    fe = sub_state(z, "final.E.")
    for k, v in net.state_dict().items():
        close(v, fg[k], rtol=1e-4, atol=2e-6)
    for k, v in ema.state_dict().items():
        close(v, fe[k], rtol=1e-4, atol=2e-6)


def test_dncnn_train_mode_bn():
    z = load_golden("conv_nets")
    net = convnets.DnCNN(1, 1, 64, 5, "BR")
    net.load_state_dict(sub_state(z, "dncnn."), strict=True)
    net.train()
    x = torch.from_numpy(z["dncnn.x"])
    out = net(x)
    close(out, z["dncnn.out"])
    out.backward(torch.from_numpy(z["dncnn.gout"]))
    g = sub_grads(z, "dncnn.")
    for k, p in net.named_parameters():
        close(p.grad, g[k], rtol=1e-3, atol=1e-4)
    sd = net.state_dict()
    for k in z.files:
        if k.startswith("dncnn.after."):
            close(sd[k[len("dncnn.after."):]], z[k])


@pytest.mark.parametrize("name", ["rrdbnet", "rrdb"])
def test_rrdb_nets(name):
    z = load_golden("conv_nets")
    pre = name + "."
    net = convnets.RRDBNet(3, 3, 32, 1, 16, 4) if name == "rrdbnet" else convnets.RRDB(3, 3, 32, 1, 32, 4, "R")
    net.load_state_dict(sub_state(z, pre), strict=True)
    x = torch.from_numpy(z[pre + "x"])
    out = net(x)
    close(out, z[pre + "out"])
    out.backward(torch.from_numpy(z[pre + "gout"]))
    g = sub_grads(z, pre)
    for k, p in net.named_parameters():
        close(p.grad, g[k], rtol=1e-3, atol=1e-4)


def test_usrnet():
    z = load_golden("usrnet")
    net = convnets.USRNet(n_iter=2, h_nc=32, in_nc=4, out_nc=3, nc=[16, 32, 64, 64], nb=2)
    net.load_state_dict(sub_state(z, ""), strict=True)
    out = net(torch.from_numpy(z["x"]), torch.from_numpy(z["k"]), int(z["sf"]), torch.from_numpy(z["sigma"]))
    close(out, z["out"], rtol=1e-4, atol=1e-5)
    out.backward(torch.from_numpy(z["gout"]))
    g = sub_grads(z, "")
    for k, p in net.named_parameters():
        close(p.grad, g[k], rtol=2e-3, atol=1e-4)


def test_datanet():
    z = load_golden("usrnet")
    k = torch.from_numpy(z["k"])
    FB = convnets.p2o(k, (64, 64))
    close(FB.real, z["datanet.FB_re"], atol=1e-6)
    close(FB.imag, z["datanet.FB_im"], atol=1e-6)
    FBC, F2B = torch.conj(FB), torch.abs(FB) ** 2
    FBFy = FBC * torch.fft.fftn(convnets.zero_upsample(torch.from_numpy(z["datanet.y"]), 4), dim=(-2, -1))
    zz = convnets.datanet(torch.from_numpy(z["datanet.x"]), FB, FBC, F2B, FBFy, torch.from_numpy(z["datanet.alpha"]), 4)
    close(zz, z["datanet.z"], atol=1e-5)


@pytest.mark.parametrize("key,src,scale", [("lr4", "img", 1 / 4), ("lr2", "img", 1 / 2), ("lr3", "img2", 1 / 3),
                                           ("up2", "img2", 2)])
def test_imresize(key, src, scale):
    z = load_golden("image_utils")
    out = image.imresize_matlab(torch.from_numpy(z[src]), scale)
    close(out, z[key], rtol=1e-5, atol=1e-6)


def test_imresize_gray_and_psnr():
    z = load_golden("image_utils")
    close(image.imresize_matlab(torch.from_numpy(z["img2"][0]), 1 / 2), z["gray"], rtol=1e-5, atol=1e-6)
    ua = image.tensor2uint(torch.from_numpy(z["a"]))
    ub = image.tensor2uint(torch.from_numpy(z["b"]))
    np.testing.assert_array_equal(ua, z["ua"])
    np.testing.assert_array_equal(ub, z["ub"])
    assert abs(image.calculate_psnr(ua, ub, 0) - float(z["psnr0"])) < 1e-9
    assert abs(image.calculate_psnr(ua, ub, 4) - float(z["psnr4"])) < 1e-9


def test_dncnn_kat():
    """Reference-shipped fixture: dncnn_25.pth (weights recorded as golden E) -> 29.8535 dB."""
    z = load_golden("dncnn_kat")
    E_u = image.tensor2uint(torch.from_numpy(z["E"]))
    assert abs(image.calculate_psnr(E_u, z["img_H"]) - 29.8535) < 5e-5
    noisy = np.uint8((np.clip(z["img_L"], 0, 1) * 255.0).round())
    assert abs(image.calculate_psnr(noisy, z["img_H"]) - 20.3410) < 5e-5


@pytest.mark.parametrize("name", ["swinir_classical_x4", "swinir_light_x2", "dncnn", "rrdb", "rrdbnet", "usrnet"])
def test_oracle_state_dict_layout(name):
    ref = json.load(open(os.path.join(GOLDEN, "state_dict_layouts.json")))[name]
    if name == "swinir_classical_x4":
        net = swinir.SwinIR(4, 3, 48, 8, 1.0, [6] * 6, 180, [6] * 6, 2, "pixelshuffle")
    elif name == "swinir_light_x2":
        net = swinir.SwinIR(2, 3, 64, 8, 1.0, [6] * 4, 60, [6] * 4, 2, "pixelshuffledirect")
    elif name == "dncnn":
        net = convnets.DnCNN(1, 1, 64, 17, "BR")
    elif name == "rrdb":
        net = convnets.RRDB(3, 3, 64, 23, 32, 4, "R")
    elif name == "rrdbnet":
        net = convnets.RRDBNet(3, 3, 64, 23, 32, 4)
    else:
        net = convnets.USRNet(6, 32, 4, 3, [16, 32, 64, 64], 2)
    got = [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in net.state_dict().items()]
    assert got == ref["keys"]
    assert sum(p.numel() for p in net.parameters()) == ref["n_params"]
