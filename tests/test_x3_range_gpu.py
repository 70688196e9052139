"""The fp32x3 engine's range guard (VERDICT r5 "What's weak" #1): every split-fp16 operand class has a fixed
power-of-2 window (activations 2^4, data gradients 2^(log2(numel / loss weight) + 4), weights 2^12).  A value
that leaves fp16's range turns the step's gradients non-finite; kair_range_check flags it on the device, the
Adam kernel drops the flagged step, and FusedTrainer.check_range lowers the exponents (engine.x3_backoff) and
re-runs the step on the same batch.  These tests drive the guard deliberately and hold the fp32 bars against
the CPU oracle trainer (the reference's ModelPlain.optimize_parameters, model_plain.py:270-318), or see it raise.

  * activations near 1e4 (input patches scaled x 1e4: the conv_first operand and the long-skip tail reach
    ~1e4, 16 x 1e4 > 65504 at the default exponent);
  * a loss weight of 1e3 (G_lossfn_weight): the gradient exponent follows the loss weight, so no event;
  * gradients 2^12 above their window (the gradient exponent forced up): the guard backs off;
  * NaN data: the guard gives up and raises instead of training on."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from conftest import state_rel_excluding_kbias  # noqa: E402
from kair_amd import _hip as H  # noqa: E402
from kair_amd.engine.trainer import FusedTrainer  # noqa: E402
from kair_amd.models.network_swinir import SwinIR  # noqa: E402
from oracle import swinir as osw  # noqa: E402
from oracle.train import OracleTrainer  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_range_check_kernel_and_adam_skip():
    n = 4099   # a ragged tail past the float4 body
    g = torch.randn(n, device=dev)
    p = torch.randn(n, device=dev) * 0.1
    loss = torch.ones(1, device=dev)
    flag = torch.full((1,), 77, dtype=torch.int32, device=dev)
    H.range_check(g, p, loss, 16.0, flag)
    assert int(flag) == 0   # zeroed by the launch, nothing found
    for i in (5, n - 1):    # body and tail
        g2 = g.clone()
        g2[i] = float("inf")
        H.range_check(g2, p, loss, 16.0, flag)
        assert int(flag) == 1
        g2[i] = float("nan")
        H.range_check(g2, p, None, 16.0, flag)
        assert int(flag) == 1
        p2 = p.clone()
        p2[i] = -16.5
        H.range_check(g, p2, loss, 16.0, flag)
        assert int(flag) == 4
    H.range_check(g, p, torch.full((1,), float("nan"), device=dev), 16.0, flag)
    assert int(flag) == 2
    # a flagged step updates nothing (parameters, moments, EMA); a clean one does
    m, v, e = torch.zeros(n, device=dev), torch.zeros(n, device=dev), p.clone()
    lr_t = torch.tensor([1e-3, 1.0], device=dev)
    p0 = p.clone()
    flag.fill_(1)
    H.adam_ema(p, g, m, v, e, n, lr_t, 0.9, 0.999, 1e-8, 0.0, 0.999, skip=flag)
    assert torch.equal(p, p0) and not m.any() and not v.any() and torch.equal(e, p0)
    flag.zero_()
    H.adam_ema(p, g, m, v, e, n, lr_t, 0.9, 0.999, 1e-8, 0.0, 0.999, skip=flag)
    assert not torch.equal(p, p0) and m.any()


def _pair(ups="pixelshuffle", sc=2, img_range=1.0, seed=21):
    torch.manual_seed(seed)
    mk = lambda: SwinIR(upscale=sc, in_chans=3, img_size=16, window_size=8, img_range=img_range, depths=[2, 2],
                        embed_dim=60, num_heads=[6, 6], mlp_ratio=2, upsampler=ups, resi_connection="1conv",
                        drop_path_rate=0.0, compute_dtype="fp32x3")
    net, ema = mk(), mk()
    ema.load_state_dict(net.state_dict())
    mko = lambda: osw.SwinIR(sc, 3, 16, 8, img_range, [2, 2], 60, [6, 6], 2, ups, "1conv")
    ref, ref_e = mko(), mko()
    ref.load_state_dict(net.state_dict(), strict=True)
    ref_e.load_state_dict(net.state_dict(), strict=True)
    return net.to(dev).train(), ema.to(dev).eval(), ref, ref_e


def _train(net, ema, ref, ref_e, scale=1.0, loss_weight=1.0, steps=4, use_graph=True, setup=None, sc=2):
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999, use_graph=use_graph, loss_weight=loss_weight)
    if setup:
        setup(tr.engine)
    otr = OracleTrainer(ref, ref_e, lr=2e-4, E_decay=0.999, loss_weight=loss_weight)
    g = torch.Generator().manual_seed(22)
    losses, olosses = [], []
    for _ in range(steps):   # 2 eager warm-up steps, then graph capture + replay
        L = torch.rand(2, 3, 16, 16, generator=g) * scale
        Hh = torch.rand(2, 3, 16 * sc, 16 * sc, generator=g) * scale
        losses.append(tr.step(L.to(dev), Hh.to(dev)))
        tr.check_range()
        losses[-1] = losses[-1].item()
        olosses.append(otr.optimize_parameters(L, Hh)[1])
    return tr, losses, olosses


def _assert_matches(net, ema, ref, ref_e, losses, olosses, tol=1e-4, steps=4, lr=2e-4, btol=2e-3):
    """Losses and the trained G / EMA states vs the oracle trainer: weights at `tol` (relative L2 per tensor);
    1-D parameters (biases, LayerNorm affine, initialised at 0 / 1: after a few steps they ARE Adam's m / sqrt(v)
    updates, which normalise each element's gradient, so a near-zero gradient element moves by up to lr on
    summation-order noise) at `btol`; the key part of each qkv bias (zero gradient in exact arithmetic) within
    2 lr per step (conftest.state_rel_excluding_kbias)."""
    for a, b in zip(losses, olosses):
        assert abs(a - b) < tol * abs(b), (losses, olosses)
    for mine, theirs in ((net, ref), (ema, ref_e)):
        sd = theirs.state_dict()
        r, kmax = state_rel_excluding_kbias(mine.state_dict(), sd, 60)
        worst = max((v, k) for k, v in r.items() if sd[k].dim() > 1)
        assert worst[0] < tol, worst
        worst = max((v, k) for k, v in r.items() if sd[k].dim() <= 1)
        assert worst[0] < btol, worst
        assert kmax <= 2 * lr * steps, kmax


@pytest.mark.parametrize("use_graph", [True, False])
def test_guard_activations_near_1e4(use_graph):
    """Input patches x 1e4: conv_first's split operand (and the tail's long skip) at ~1e4, 2^4 x 1e4 > 65504.
    The first step is flagged, the exponents drop, the step is re-run; the trajectory holds the fp32 bars."""
    net, ema, ref, ref_e = _pair()
    tr, losses, olosses = _train(net, ema, ref, ref_e, scale=1e4, use_graph=use_graph)
    assert tr.range_events, "the guard never fired"
    assert tr.range_events[0][0] == 1   # flagged at the first step, which was re-run
    assert tr.engine.X3_AEXP < 4 and tr.engine.x3_gexp_off == 4   # only the activation class backed off
    _assert_matches(net, ema, ref, ref_e, losses, olosses)


def test_guard_forced_gradient_exponent():
    """Data gradients 2^12 above their window (the gradient exponent forced up by 12): the backward overflows,
    the guard backs off and the re-run steps hold the fp32 bars."""
    net, ema, ref, ref_e = _pair(seed=23)

    def force(eng):
        eng.x3_gexp_off += 12
    tr, losses, olosses = _train(net, ema, ref, ref_e, setup=force)
    assert tr.range_events and tr.range_events[0][1] & 1, tr.range_events
    assert tr.engine.X3_AEXP == 4   # only the gradient class backed off
    _assert_matches(net, ema, ref, ref_e, losses, olosses)


def test_loss_weight_1e3_no_event():
    """G_lossfn_weight 1e3 scales every data gradient 1e3 x: the gradient exponent follows the loss weight
    (engine._x3_grad_exp), so the window holds with no guard event, at the fp32 bars."""
    net, ema, ref, ref_e = _pair(seed=24)
    tr, losses, olosses = _train(net, ema, ref, ref_e, loss_weight=1e3)
    assert not tr.range_events, tr.range_events
    _assert_matches(net, ema, ref, ref_e, losses, olosses)


def test_img_range_255_trains_at_fp32_bars():
    """img_range 255 (options/swinir/train_swinir_car_jpeg.json's scale, here on the classical head): the
    residual stream and the tail carry 255-scaled values; the trajectory holds the fp32 bars (guard events, if
    any, are re-run steps)."""
    net, ema, ref, ref_e = _pair(img_range=255.0, seed=25)
    tr, losses, olosses = _train(net, ema, ref, ref_e)
    _assert_matches(net, ema, ref, ref_e, losses, olosses)


def test_guard_raises_on_nan_data():
    """Non-finite data is not a range problem: after X3_BACKOFF_MAX re-runs the guard raises."""
    net, ema, _, _ = _pair(seed=26)
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999, use_graph=False)
    L = torch.rand(2, 3, 16, 16, device=dev)
    L[0, 0, 3, 3] = float("nan")
    Hh = torch.rand(2, 3, 32, 32, device=dev)
    p0 = tr.flat_p.clone()
    with pytest.raises(RuntimeError, match="range guard"):
        tr.step(L, Hh)
        tr.check_range()
    assert torch.equal(tr.flat_p, p0)   # no flagged step updated the parameters


def test_autograd_forward_guard():
    """The eager / autograd path (SwinIR.forward without the trainer): a non-finite forward is re-run with the
    exponents lowered; output and gradients vs the oracle at the fp32 bars."""
    net, _, ref, _ = _pair(seed=27)
    g = torch.Generator().manual_seed(28)
    L = torch.rand(2, 3, 16, 16, generator=g) * 1e4
    Hh = torch.rand(2, 3, 32, 32, generator=g) * 1e4
    E = net(L.to(dev))
    assert net.engine().x3_backoffs >= 1
    Er = ref(L)
    assert rel(E, Er) < 1e-5
    torch.nn.functional.l1_loss(E, Hh.to(dev)).backward()
    torch.nn.functional.l1_loss(Er, Hh).backward()
    gref = dict(ref.named_parameters())
    worst = max((rel(p.grad, gref[k].grad), k) for k, p in net.named_parameters())
    assert worst[0] < 1e-3, worst
