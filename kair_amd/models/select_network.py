"""define_G — the drop-in boundary (mirror of /root/reference/models/select_network.py:16-274).

`opt['netG']['net_type']` selects the network; constructor kwargs are taken from opt['netG'] under
the reference's key names, and init_weights() runs when opt['is_train'] (select_network.py:268-272).
Networks on the MI355X path: swinir, dncnn, fdncnn, rrdb, rrdbnet, usrnet.  Everything else the
reference's define_G knows (ffdnet, srmd, dpsr, msrresnet*, imdn, drunet, vrt, rvrt, ...) is out of
scope for this build and raises NotImplementedError naming the type.
"""
import functools
import logging

from torch.nn import init

logger = logging.getLogger("kair_amd")

_ON_PATH = ("swinir", "dncnn", "fdncnn", "rrdb", "rrdbnet", "usrnet")


def define_G(opt):
    o = opt["netG"]
    t = o["net_type"]
    ek = _engine_kwargs(opt)
    if t == "swinir":
        from .network_swinir import SwinIR
        net = SwinIR(upscale=o["upscale"], in_chans=o["in_chans"], img_size=o["img_size"], window_size=o["window_size"],
                     img_range=o["img_range"], depths=o["depths"], embed_dim=o["embed_dim"], num_heads=o["num_heads"],
                     mlp_ratio=o["mlp_ratio"], upsampler=o["upsampler"], resi_connection=o["resi_connection"],
                     **ek, **({"drop_path_rate": o["drop_path_rate"]} if o.get("drop_path_rate") is not None
                                             else {}))
    elif t in ("dncnn", "fdncnn"):
        from .network_dncnn import DnCNN, FDnCNN
        cls = DnCNN if t == "dncnn" else FDnCNN
        net = cls(in_nc=o["in_nc"], out_nc=o["out_nc"], nc=o["nc"], nb=o["nb"], act_mode=o["act_mode"],
                  **ek)
    elif t == "rrdb":
        from .network_rrdb import RRDB
        net = RRDB(in_nc=o["in_nc"], out_nc=o["out_nc"], nc=o["nc"], nb=o["nb"], gc=o["gc"], upscale=o["scale"],
                   act_mode=o["act_mode"], upsample_mode=o["upsample_mode"], **ek)
    elif t == "rrdbnet":
        from .network_rrdbnet import RRDBNet
        net = RRDBNet(in_nc=o["in_nc"], out_nc=o["out_nc"], nf=o["nf"], nb=o["nb"], gc=o["gc"], sf=o["scale"],
                      **ek)
    elif t == "usrnet":
        from .network_usrnet import USRNet
        net = USRNet(n_iter=o["n_iter"], h_nc=o["h_nc"], in_nc=o["in_nc"], out_nc=o["out_nc"], nc=o["nc"], nb=o["nb"],
                     act_mode=o["act_mode"], downsample_mode=o["downsample_mode"], upsample_mode=o["upsample_mode"],
                     **ek)
    else:
        raise NotImplementedError("netG [{:s}] is not on the kair_amd MI355X path (supported: {})".format(
            t, ", ".join(_ON_PATH)))
    logger.info("define_G: %s on the %s engine (%s)", t, ek["compute_dtype"],
                "netG.compute_dtype" if o.get("compute_dtype") else
                ("train.amp_enabled" if (opt.get("train") or {}).get("amp_enabled") else "reference default"))
    if opt.get("is_train"):
        init_weights(net, init_type=o.get("init_type", "default") or "default",
                     init_bn_type=o.get("init_bn_type", "uniform") or "uniform", gain=o.get("init_gain", 1) or 1)
    return net


_X3_NETS = ("swinir", "rrdbnet", "rrdb")   # networks with a split-fp16 (fp32x3) engine


def compute_dtype_of(opt):
    """The engine's arithmetic, decided by the option file as the reference decides it:
      netG.compute_dtype ('bf16' / 'fp32' / 'fp32x3')  explicit choice (build-side key, absent from
                                            reference files);
      train.amp_enabled: true               the reference's reduced-precision mode (model_plain.py:32-35,
                                            261-275: fp16 autocast + GradScaler) -> the bf16 MFMA engine
                                            (fp32 master weights / accumulation; bf16 keeps fp32's exponent
                                            range, so no loss scaling and no {iter}_scaler.pth);
      otherwise                             the reference's default fp32 arithmetic: 'fp32x3' where the
                                            network has that engine (SwinIR: every product on the 16-bit
                                            matrix cores as three fp16 products of power-of-2-scaled hi/lo
                                            pairs, ~2^-21 relative -- it passes the exact-fp32 engine's oracle
                                            bars, tests/test_x3_gpu.py; RRDBNet / RRDB: tests/test_full_configs_gpu.py
                                            test_c5_rrdbnet_full[fp32x3]), else 'fp32' (exact-fp32 MFMA)."""
    o = opt["netG"]
    if o.get("compute_dtype"):
        if o["compute_dtype"] not in ("bf16", "fp32", "fp32x3"):
            raise ValueError(f"netG.compute_dtype must be 'bf16', 'fp32' or 'fp32x3' (got {o['compute_dtype']!r})")
        if o["compute_dtype"] == "fp32x3" and o.get("net_type") not in _X3_NETS:
            raise ValueError(f"netG.compute_dtype 'fp32x3' is available for {_X3_NETS} (got {o.get('net_type')!r})")
        return o["compute_dtype"]
    tr = opt.get("train") or {}
    if tr.get("amp_enabled"):
        return "bf16"
    return "fp32x3" if o.get("net_type") in _X3_NETS else "fp32"


def _engine_kwargs(opt):
    """Constructor kwargs the option file decides beyond the reference's (compute_dtype_of).  (netG.drop_path_rate,
    SwinIR only, is passed through when present; absent, SwinIR's own default 0.1 applies exactly as the
    reference's define_G leaves it.)"""
    return {"compute_dtype": compute_dtype_of(opt)}


def init_weights(net, init_type="xavier_uniform", init_bn_type="uniform", gain=1):
    """select_network.py:370-440 (same initialisers, same Conv/Linear/BatchNorm2d matching by class name)."""

    def init_fn(m, init_type, init_bn_type, gain):
        name = m.__class__.__name__
        if name.find("Conv") != -1 or name.find("Linear") != -1:
            w = m.weight.data
            if init_type == "normal":
                init.normal_(w, 0, 0.1)
                w.clamp_(-1, 1).mul_(gain)
            elif init_type == "uniform":
                init.uniform_(w, -0.2, 0.2)
                w.mul_(gain)
            elif init_type == "xavier_normal":
                init.xavier_normal_(w, gain=gain)
                w.clamp_(-1, 1)
            elif init_type == "xavier_uniform":
                init.xavier_uniform_(w, gain=gain)
            elif init_type == "kaiming_normal":
                init.kaiming_normal_(w, a=0, mode="fan_in", nonlinearity="relu")
                w.clamp_(-1, 1).mul_(gain)
            elif init_type == "kaiming_uniform":
                init.kaiming_uniform_(w, a=0, mode="fan_in", nonlinearity="relu")
                w.mul_(gain)
            elif init_type == "orthogonal":
                init.orthogonal_(w, gain=gain)
            else:
                raise NotImplementedError("Initialization method [{:s}] is not implemented".format(init_type))
            if getattr(m, "bias", None) is not None:
                m.bias.data.zero_()
        elif name.find("BatchNorm2d") != -1:
            if init_bn_type == "uniform":
                if m.affine:
                    init.uniform_(m.weight.data, 0.1, 1.0)
                    init.constant_(m.bias.data, 0.0)
            elif init_bn_type == "constant":
                if m.affine:
                    init.constant_(m.weight.data, 1.0)
                    init.constant_(m.bias.data, 0.0)
            else:
                raise NotImplementedError("Initialization method [{:s}] is not implemented".format(init_bn_type))

    if init_type not in ("default", "none"):
        net.apply(functools.partial(init_fn, init_type=init_type, init_bn_type=init_bn_type, gain=gain))
