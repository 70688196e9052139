"""Fused MLP-half diagnostics: per-parameter gradient error vs the fp32 engine (fused vs unfused
bf16) and 25-step loss trajectories with the fused MLP on / off."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import build_net  # noqa: E402
from kair_amd.engine.swinir_engine import SwinIREngine  # noqa: E402
from kair_amd.engine.trainer import FusedTrainer  # noqa: E402
from kair_amd.utils import utils_image as U  # noqa: E402

dev = torch.device("cuda")


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def grads(dtype, fused_mlp, sd, x, D, gE):
    n = build_net(dtype, 0.1).to(dev).train()
    n.load_state_dict(sd)
    e = SwinIREngine(n, dtype, fused_mlp=fused_mlp)
    e.forward(x, D)
    params = list(n.parameters())
    flat = torch.zeros(sum(p.numel() for p in params), device=dev)
    gd, off = {}, 0
    for p in params:
        gd[p] = flat[off:off + p.numel()].view_as(p)
        off += p.numel()
    e.backward_from_grad(gE, gd)
    return {k: gd[p].clone() for (k, _), p in zip(n.named_parameters(), params)}, e.cur["E"].clone()


def main():
    torch.manual_seed(0)
    sd = build_net("bf16", 0.1).state_dict()
    g = torch.Generator().manual_seed(3)
    B = 4
    x = torch.rand(B, 3, 48, 48, generator=g).to(dev)
    nb = 36
    D = ((torch.rand(nb, 2, B, generator=g) < 0.9).float() / 0.9).to(dev)
    gE = torch.randn(B, 3, 192, 192, generator=g).to(dev)
    gr, Er = grads("fp32", False, sd, x, D, gE)
    gf, Ef = grads("bf16", True, sd, x, D, gE)
    gu, Eu = grads("bf16", False, sd, x, D, gE)
    print("E rel fused", rel(Ef, Er), "unfused", rel(Eu, Er))
    worst = sorted(((rel(gf[k], gr[k]) - rel(gu[k], gr[k]), k, rel(gf[k], gr[k]), rel(gu[k], gr[k])) for k in gr), reverse=True)
    for w in worst[:12]:
        print("%-60s fused %.4g unfused %.4g" % (w[1], w[2], w[3]))
    for fm in (True, False, True, False):
        from kair_amd.engine.swinir_engine import SwinIREngine
        net = build_net("bf16", 0.1).to(dev).train()
        net._engine = SwinIREngine(net, "bf16", fused_mlp=fm)
        ema = build_net("bf16", 0.1).to(dev).eval()
        ema.load_state_dict(net.state_dict())
        tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999)
        L, Hh = U.synth_sr_batch(32, 48, 4, seed=1000, device=dev)
        ls = [float(tr.step(L, Hh)) for _ in range(30)]
        print("fused_mlp", fm, "loss", [round(v, 4) for v in ls[::5]], round(ls[-1], 5))


if __name__ == "__main__":
    main()
