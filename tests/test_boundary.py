"""The drop-in boundary, checked without a GPU.

* libkair_hip.so loads and exports every function include/kair_hip.h declares (no compute calls);
* the ctypes binding declares a signature for each of them;
* the product package never imports the oracle (oracle/ is test infrastructure only);
* the HIP path fails loudly instead of falling back to CPU;
* define_G builds the reference module trees (state_dict keys / shapes == reference, golden JSON).
"""
import ctypes
import json
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kair_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?(?:int|long|void|char\s*\*|const char\s*\*)\s*\**\s*(kair_\w+)\s*\(", src,
                       flags=re.M)
    return sorted(set(names))


def test_header_parses():
    names = header_functions()
    assert "kair_gemm_nt" in names and "kair_window_attn_bwd" in names and len(names) >= 20, names


def test_library_exports_every_header_symbol():
    from kair_amd import _hip
    if not os.path.exists(_hip.LIB_PATH):
        from kair_amd import build
        build.build(verbose=False)
    L = ctypes.CDLL(_hip.LIB_PATH)
    missing = [n for n in header_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_binding_covers_header():
    from kair_amd import _hip
    missing = [n for n in header_functions() if n not in _hip._SIGS]
    assert not missing, missing


def test_error_channel_without_gpu():
    """Argument validation runs on the host: a bad call returns an error code + message, no launch."""
    from kair_amd import _hip
    L = _hip.lib()
    rc = L.kair_layernorm_fwd(None, 0, None, 0, 0, None, None, None, None, 0, 0, 1e-5, 0, 0, 0, 0, -1, None)
    assert rc != 0
    assert b"layernorm_fwd" in L.kair_last_error()


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "kair_amd")
    offenders = []
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                txt = open(os.path.join(dp, f)).read()
                if re.search(r"^\s*(from|import)\s+oracle\b", txt, flags=re.M):
                    offenders.append(os.path.join(dp, f))
    assert not offenders, offenders


def test_cpu_input_raises():
    from kair_amd.models.network_swinir import SwinIR
    net = SwinIR(upscale=2, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2], embed_dim=60,
                 num_heads=[6], mlp_ratio=2, upsampler="pixelshuffledirect", resi_connection="1conv")
    with pytest.raises(RuntimeError):
        net(torch.zeros(1, 3, 16, 16))


# the option-file configs tests/golden/make_golden.py:gen_state_dict_layouts recorded the layouts at
NETG_CFGS = {
    "swinir_classical_x4": {"net_type": "swinir", "upscale": 4, "in_chans": 3, "img_size": 48, "window_size": 8,
                            "img_range": 1.0, "depths": [6] * 6, "embed_dim": 180, "num_heads": [6] * 6,
                            "mlp_ratio": 2, "upsampler": "pixelshuffle", "resi_connection": "1conv",
                            "init_type": "default"},
    "swinir_light_x2": {"net_type": "swinir", "upscale": 2, "in_chans": 3, "img_size": 64, "window_size": 8,
                        "img_range": 1.0, "depths": [6] * 4, "embed_dim": 60, "num_heads": [6] * 4, "mlp_ratio": 2,
                        "upsampler": "pixelshuffledirect", "resi_connection": "1conv", "init_type": "default"},
    "dncnn": {"net_type": "dncnn", "in_nc": 1, "out_nc": 1, "nc": 64, "nb": 17, "act_mode": "BR",
              "init_type": "orthogonal", "init_bn_type": "uniform", "init_gain": 0.2},
    "rrdb": {"net_type": "rrdb", "in_nc": 3, "out_nc": 3, "nc": 64, "nb": 23, "gc": 32, "scale": 4, "act_mode": "R",
             "upsample_mode": "upconv", "init_type": "orthogonal", "init_bn_type": "uniform", "init_gain": 0.2},
    "rrdbnet": {"net_type": "rrdbnet", "in_nc": 3, "out_nc": 3, "nf": 64, "nb": 23, "gc": 32, "scale": 4,
                "init_type": "default"},
    "usrnet": {"net_type": "usrnet", "n_iter": 6, "h_nc": 32, "in_nc": 4, "out_nc": 3, "nc": [16, 32, 64, 64], "nb": 2,
               "act_mode": "R", "downsample_mode": "strideconv", "upsample_mode": "convtranspose",
               "init_type": "orthogonal", "init_bn_type": "uniform", "init_gain": 0.2},
}


@pytest.mark.parametrize("name", sorted(NETG_CFGS))
def test_define_G_state_dict_matches_reference(name):
    from kair_amd.models.select_network import define_G
    from kair_amd.utils.utils_option import dict_to_nonedict
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "state_dict_layouts.json")))[name]
    opt = dict_to_nonedict({"is_train": False, "netG": dict(NETG_CFGS[name])})
    net = define_G(opt)
    sd = net.state_dict()
    assert [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()] == ref["keys"]
    assert sum(p.numel() for p in net.parameters()) == ref["n_params"]


def test_custom_ops_registered_and_refuse_cpu():
    """torch.ops.kair.* exist (schema per op) and have no CPU kernel: a host tensor raises."""
    from kair_amd import ops
    for name in ops.registered_ops():
        assert hasattr(torch.ops.kair, name), name
    with pytest.raises(NotImplementedError):
        torch.ops.kair.linear(torch.zeros(4, 8), torch.zeros(4, 8), None, 0, 0)
    from kair_amd.models.network_swinir import WindowAttention
    with pytest.raises(RuntimeError):
        WindowAttention(60, (8, 8), 6)(torch.zeros(1, 64, 60))


def test_precision_is_an_option_file_decision():
    """define_G's arithmetic follows the option file (select_network.compute_dtype_of): the reference's
    fp32 by default (SwinIR, RRDBNet / RRDB: the fp16-pair engine 'fp32x3' that holds the fp32 engine's oracle bars;
    the other conv nets: exact fp32), its amp_enabled reduced-precision mode -> the bf16 engine, netG.compute_dtype
    explicit."""
    from kair_amd.models.select_network import compute_dtype_of
    base = {"netG": {"net_type": "swinir"}}
    assert compute_dtype_of(base) == "fp32x3"
    assert compute_dtype_of({**base, "train": {"amp_enabled": False}}) == "fp32x3"
    assert compute_dtype_of({"netG": {"net_type": "rrdbnet"}}) == "fp32x3"
    assert compute_dtype_of({"netG": {"net_type": "dncnn"}}) == "fp32"
    with pytest.raises(ValueError):
        compute_dtype_of({"netG": {"net_type": "dncnn", "compute_dtype": "fp32x3"}})
    assert compute_dtype_of({**base, "train": {"amp_enabled": True}}) == "bf16"
    assert compute_dtype_of({"netG": {"net_type": "swinir", "compute_dtype": "fp32"}, "train": {"amp_enabled": True}}) == "fp32"
    assert compute_dtype_of({"netG": {"net_type": "swinir", "compute_dtype": "bf16"}}) == "bf16"
    with pytest.raises(ValueError):
        compute_dtype_of({"netG": {"net_type": "swinir", "compute_dtype": "fp16"}})
