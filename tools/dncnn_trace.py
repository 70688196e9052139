"""Layer-by-layer precision trace of the fp32 DnCNN engine against a float64 run of the oracle on the
same weights and patch (VERDICT r2 "What's weak" 1 / ADVICE r2): forward activations, dL/da and
dL/dz at every BatchNorm layer, dgamma / dbeta, conv weight gradients -- where does the error grow?

    python tools/dncnn_trace.py [--depth 17] [--batch 4]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kair_amd import _hip as H  # noqa: E402
from oracle import convnets as ocv  # noqa: E402


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def nhwc(t):   # [B, C, H, W] -> [B*H*W, C]
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=17)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    from kair_amd.models.network_dncnn import DnCNN
    dev = torch.device("cuda")
    torch.manual_seed(1)
    net = DnCNN(1, 1, 64, a.depth, "BR", compute_dtype="fp32")
    ref = ocv.DnCNN(1, 1, 64, a.depth, "BR").train()
    ref.load_state_dict(net.state_dict(), strict=True)
    ref32 = ocv.DnCNN(1, 1, 64, a.depth, "BR").train()
    ref32.load_state_dict(net.state_dict(), strict=True)
    ref = ref.double()
    g = torch.Generator().manual_seed(2)
    x = torch.rand(a.batch, 1, 40, 40, generator=g) + 25.0 / 255 * torch.randn(a.batch, 1, 40, 40, generator=g)
    Hh = torch.rand(a.batch, 1, 40, 40, generator=torch.Generator().manual_seed(7))

    def run_ref(model, dt):
        outs = []
        y = x.to(dt)
        for m in model.model:
            y = m(y)
            y.retain_grad()
            outs.append((m, y))
        E = x.to(dt) - y
        torch.nn.functional.l1_loss(E, Hh.to(dt)).backward()
        return outs
    o64 = run_ref(ref, torch.float64)
    o32 = run_ref(ref32, torch.float32)

    # engine forward, then the backward of DnCNNEngine.backward with captures
    net = net.to(dev).train()
    eng = net.engine()
    E = eng.forward(x.to(dev))
    grads = {p: torch.zeros_like(p) for p in net.parameters()}
    P = eng.cur
    H.l1_loss(P["E"], Hh.to(dev), P["loss"], P["dEf"], 16, 1.0, P["B"], eng.out_ch, P["H"], P["W"], P["loss_ws"])
    cap = {}
    orig_bn_bwd = H.bn_bwd

    def bn_bwd(z, ldz, act_, lda, G, ldg, dz, lddz, M, C, *rest):
        li = len([k for k in cap if k[0] == "G"])
        cap[("G", li)] = G[:M].clone()
        orig_bn_bwd(z, ldz, act_, lda, G, ldg, dz, lddz, M, C, *rest)
        cap[("dz", li)] = dz[:M].clone()
    H.bn_bwd = bn_bwd
    try:
        eng.backward(grads, P)
    finally:
        H.bn_bwd = orig_bn_bwd
    torch.cuda.synchronize()

    # pair engine layers with oracle modules: conv (bn relu) ... ; BN layers in backward order
    bn_mods = [(i, m) for i, (m, _) in enumerate(o64) if isinstance(m, torch.nn.BatchNorm2d)]
    print(f"depth {a.depth}, batch {a.batch}: output rel {rel(E.cpu(), x - o64[-1][1].detach()):.2e}")
    print(f"{'BN layer':>9} {'a fwd':>9} {'(ref32)':>9} {'dL/da':>9} {'(ref32)':>9} {'dL/dz':>9} {'(ref32)':>9} {'dgamma':>9} {'(ref32)':>9}"
          f" {'dbeta':>9} {'(ref32)':>9} {'conv dW':>9} {'(ref32)':>9}")
    ours = dict(net.named_parameters())
    p64 = dict(ref.named_parameters())
    p32 = dict(ref32.named_parameters())
    nb = len(bn_mods)
    for j, (i, bn) in enumerate(reversed(bn_mods)):   # backward order
        li_bn = nb - 1 - j                # BN index in forward order
        relu64 = o64[i + 1][1]            # post-ReLU output (grad = dL/da)
        relu32 = o32[i + 1][1]
        z64, z32 = o64[i - 1][1], o32[i - 1][1]   # conv output = BN input
        eng_li = li_bn + 1                # engine layer index (layer 0 has no BN)
        a_fwd = rel(P["a"][eng_li].cpu(), nhwc(relu64.detach()))
        dA = rel(cap[("G", j)].cpu(), nhwc(relu64.grad))
        dA32 = rel(nhwc(relu32.grad), nhwc(relu64.grad))
        dZ = rel(cap[("dz", j)].cpu(), nhwc(z64.grad))
        dZ32 = rel(nhwc(z32.grad), nhwc(z64.grad))
        name = [k for k, v in ref.named_modules() if v is bn][0]
        conv_name = [k for k, v in ref.named_modules() if v is o64[i - 1][0]][0]
        dg = rel(ours[name + ".weight"].grad if ours[name + ".weight"].grad is not None else grads[ours[name + ".weight"]],
                 p64[name + ".weight"].grad)
        dg = rel(grads[ours[name + ".weight"]], p64[name + ".weight"].grad)
        dg32 = rel(p32[name + ".weight"].grad, p64[name + ".weight"].grad)
        db = rel(grads[ours[name + ".bias"]], p64[name + ".bias"].grad)
        db32 = rel(p32[name + ".bias"].grad, p64[name + ".bias"].grad)
        dw = rel(grads[ours[conv_name + ".weight"]], p64[conv_name + ".weight"].grad)
        dw32 = rel(p32[conv_name + ".weight"].grad, p64[conv_name + ".weight"].grad)
        a_fwd32 = rel(nhwc(relu32.detach()), nhwc(relu64.detach()))
        print(f"{li_bn:9d} {a_fwd:9.1e} ({a_fwd32:7.1e}) {dA:9.1e} {dA32:9.1e} {dZ:9.1e} {dZ32:9.1e} {dg:9.1e} {dg32:9.1e} {db:9.1e} "
              f"{db32:9.1e} {dw:9.1e} {dw32:9.1e}")
    isolate_bn(o64, o32, -1)
    isolate_bn(o64, o32, 0)
    # the last BN layer's backward on the ENGINE's forward z (fp32, with its forward error) through torch fp32:
    # does the forward error alone produce the engine's dz error (ReLU-gate flips)?
    i = bn_mods[-1][0]
    z64 = o64[i - 1][1].detach()
    B_, C_, H_, W_ = z64.shape
    z_eng = P["z"][nb].cpu().view(B_, H_, W_, C_).permute(0, 3, 1, 2).contiguous()
    g64 = o64[i + 1][1].grad.detach()
    bn = bn_mods[-1][1]

    def bwd(z, dt):
        z = z.to(dt).clone().requires_grad_(True)
        a = torch.relu(torch.nn.functional.batch_norm(z, None, None, bn.weight.detach().to(dt), bn.bias.detach().to(dt),
                                                       True, 0.1, 1e-4))
        a.backward(g64.to(dt))
        return a.detach(), z.grad
    a_r, dz_r = bwd(z64, torch.float64)
    a_e, dz_e = bwd(z_eng, torch.float32)
    a_t, dz_t = bwd(o32[i - 1][1].detach(), torch.float32)
    print(f"last BN, torch fp32 backward on: engine z -> dz rel {rel(dz_e, dz_r):.1e} (z rel {rel(z_eng, z64):.1e}, "
          f"gate flips {int(((a_e > 0) != (a_r > 0)).sum())}); torch32 z -> dz rel {rel(dz_t, dz_r):.1e} "
          f"(z rel {rel(o32[i - 1][1], z64):.1e}, flips {int(((a_t > 0) != (a_r > 0)).sum())}) of {a_r.numel()}")


def isolate_bn(o64, o32, net_bn_idx=-1):
    """The BatchNorm + ReLU backward of one layer in isolation: the SAME fp32 inputs (the float64 run's
    z and dL/da rounded to fp32) through kair_bn_fwd / kair_bn_bwd and through torch fp32 (CPU) autograd,
    both against float64."""
    dev = torch.device("cuda")
    bns = [i for i, (m, _) in enumerate(o64) if isinstance(m, torch.nn.BatchNorm2d)]
    i = bns[net_bn_idx]
    bn = o64[i][0]
    z64 = o64[i - 1][1].detach()
    g64 = o64[i + 1][1].grad.detach()
    C = z64.shape[1]
    z32 = z64.float()
    g32 = g64.float()
    gam, bet = bn.weight.detach(), bn.bias.detach()

    def f(z, g, gam, bet, dt):
        z = z.to(dt).clone().requires_grad_(True)
        gm, bt = gam.to(dt).clone().requires_grad_(True), bet.to(dt).clone().requires_grad_(True)
        a = torch.relu(torch.nn.functional.batch_norm(z, None, None, gm, bt, True, 0.1, 1e-4))
        a.backward(g.to(dt))
        return a.detach(), z.grad, gm.grad, bt.grad
    a_r, dz_r, dg_r, db_r = f(z64, g64, gam, bet, torch.float64)
    a_t, dz_t, dg_t, db_t = f(z32, g32, gam, bet, torch.float32)
    M = z32.numel() // C
    zr = nhwc(z32).contiguous().to(dev)
    gr = nhwc(g32).contiguous().to(dev)
    a_k = torch.empty(M, C, device=dev)
    mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
    ws = torch.empty(H.bn_ws(C), device=dev)
    gmd, btd = gam.float().to(dev), bet.float().to(dev)
    H.bn_fwd(zr, C, a_k, C, M, C, gmd, btd, None, None, 0.9, 1e-4, True, mean, rstd, 1, 0.0, ws)
    dz_k = torch.empty(M, C, device=dev)
    dgk, dbk = torch.empty(C, device=dev), torch.empty(C, device=dev)
    H.bn_bwd(zr, C, a_k, C, gr, C, dz_k, C, M, C, gmd, mean, rstd, 1, 0.0, dgk, dbk, False, ws)
    torch.cuda.synchronize()
    print(f"isolated BN+ReLU layer {net_bn_idx}: a  kair {rel(a_k.cpu(), nhwc(a_r)):.1e}  torch32 {rel(nhwc(a_t), nhwc(a_r)):.1e}")
    print(f"    dz  kair {rel(dz_k.cpu(), nhwc(dz_r)):.1e}  torch32 {rel(nhwc(dz_t), nhwc(dz_r)):.1e}")
    print(f"    dgamma kair {rel(dgk.cpu(), dg_r):.1e} torch32 {rel(dg_t, dg_r):.1e}; dbeta kair {rel(dbk.cpu(), db_r):.1e} "
          f"torch32 {rel(db_t, db_r):.1e}")
    # how much of dz is cancellation: |dz| vs |g gamma rstd|
    print(f"    |dz| / |gamma rstd g| = {(dz_r.norm() / (g64 * (gam.double() / (z64.var((0, 2, 3)) + 1e-4).sqrt()).view(1, -1, 1, 1)).norm()).item():.3e}")
    mean_k, mean_r = mean.cpu().double(), z64.mean((0, 2, 3))
    print(f"    batch mean kair rel {rel(mean_k, mean_r):.1e}; rstd kair rel "
          f"{rel(rstd.cpu(), 1 / (z64.var((0, 2, 3), unbiased=False) + 1e-4).sqrt()):.1e}")


if __name__ == "__main__":
    main()
