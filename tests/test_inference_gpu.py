"""Full-image inference on the HIP path against the CPU oracle: an image whose
sides are not multiples of the window (reflect pad to a window multiple + the analytic shift mask
at that resolution, network_swinir.py:259-262,783-788), the reference's tiled inference
(main_test_swinir.py:256-284) run through the same utils_model.test_tiled with either network,
and test_mode's x8 self-ensemble (utils_model.py:51-230)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from kair_amd.models.network_swinir import SwinIR  # noqa: E402
from kair_amd.utils import utils_model  # noqa: E402
from oracle import swinir as osw  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _pair():
    torch.manual_seed(8)
    net = SwinIR(upscale=2, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2, 2], embed_dim=60,
                 num_heads=[6, 6], mlp_ratio=2, upsampler="pixelshuffle", drop_path_rate=0.0, compute_dtype="fp32")
    ref = osw.SwinIR(2, 3, 16, 8, 1.0, [2, 2], 60, [6, 6], 2, "pixelshuffle")
    ref.load_state_dict(net.state_dict(), strict=True)
    return net.to(dev).eval(), ref.eval()


def test_full_image_non_window_multiple_vs_oracle():
    net, ref = _pair()
    g = torch.Generator().manual_seed(2)
    x = torch.rand(1, 3, 37, 45, generator=g)
    with torch.no_grad():
        e = net(x.to(dev))
        r = ref(x)
    assert e.shape == r.shape == (1, 3, 74, 90)
    assert rel(e, r) < 1e-5


def test_tiled_inference_vs_oracle():
    net, ref = _pair()
    g = torch.Generator().manual_seed(3)
    x = torch.rand(1, 3, 40, 56, generator=g)
    with torch.no_grad():
        e = utils_model.test_tiled(net, x.to(dev), tile=24, tile_overlap=8, sf=2, window_size=8)
        r = utils_model.test_tiled(ref, x, tile=24, tile_overlap=8, sf=2, window_size=8)
    assert e.shape == r.shape == (1, 3, 80, 112)
    assert rel(e, r) < 1e-5


def test_x8_self_ensemble_vs_oracle():
    net, ref = _pair()
    g = torch.Generator().manual_seed(4)
    x = torch.rand(1, 3, 24, 32, generator=g)
    with torch.no_grad():
        e = utils_model.test_mode(net, x.to(dev), mode=3, sf=2, modulo=1)
        r = utils_model.test_mode(ref, x, mode=3, sf=2, modulo=1)
    assert rel(e, r) < 1e-5
