"""Where the split-bf16 engine's gradient error sits: one step of the trajectory golden's small SwinIR (embed 60,
tests/golden/train_trajectory.npz init + step-1 batch) on the fp32 and the fp32x3 engines against the CPU oracle
in float64; per parameter tensor the relative L2 error of each engine and, for the worst tensors, the elements
with the largest error next to their gradient magnitude (Adam's eps = 1e-8 regime amplifies the absolute error
of gradients near 1e-8).

    python tools/x3_grad_diag.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import load_golden, sub_state  # noqa: E402
from kair_amd.models.network_swinir import SwinIR  # noqa: E402
from oracle import swinir as osw  # noqa: E402


def main():
    dev = torch.device("cuda")
    z = load_golden("train_trajectory")
    L, Hh = torch.from_numpy(z["step1.L"]), torch.from_numpy(z["step1.H"])
    ref = osw.SwinIR(4, 3, 16, 8, 1.0, [2, 2], 60, [6, 6], 2, "pixelshuffle").double()
    ref.load_state_dict({k: v.double() for k, v in sub_state(z, "init.").items()}, strict=True)
    torch.nn.functional.l1_loss(ref(L.double()), Hh.double()).backward()
    gref = {k: p.grad for k, p in ref.named_parameters()}
    grads = {}
    for dt in ("fp32", "fp32x3"):
        net = SwinIR(upscale=4, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2, 2], embed_dim=60,
                     num_heads=[6, 6], mlp_ratio=2, upsampler="pixelshuffle", drop_path_rate=0.0, compute_dtype=dt)
        net.load_state_dict(sub_state(z, "init."), strict=True)
        net = net.to(dev).train()
        torch.nn.functional.l1_loss(net(L.to(dev)), Hh.to(dev)).backward()
        grads[dt] = {k: p.grad.double().cpu() for k, p in net.named_parameters()}
    rows = []
    for k, g in gref.items():
        e = {dt: ((grads[dt][k] - g).norm() / g.norm()).item() for dt in grads}
        rows.append((e["fp32x3"], e["fp32"], k))
    rows.sort(reverse=True)
    print("%-60s %10s %10s" % ("parameter", "fp32x3", "fp32"))
    for ex, ef, k in rows[:25]:
        print("%-60s %10.2e %10.2e" % (k, ex, ef))
    for _, _, k in rows[:4]:
        g = gref[k].flatten()
        d = (grads["fp32x3"][k].flatten() - g).abs()
        d32 = (grads["fp32"][k].flatten() - g).abs()
        idx = d.argsort(descending=True)[:6]
        print(k, "| |g| rms %.3e" % g.pow(2).mean().sqrt())
        for i in idx.tolist():
            print("   [%d] g %.4e  err x3 %.2e  err fp32 %.2e" % (i, g[i], d[i], d32[i]))


if __name__ == "__main__":
    main()
