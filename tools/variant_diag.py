"""bf16 vs fp32 gradient error of small SwinIR variants against the CPU oracle (diagnostic)."""
import torch
from kair_amd.models.network_swinir import SwinIR
from oracle import swinir as osw

dev = torch.device("cuda")


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


for rng in (1.0, 255.0):
    for rc in ("1conv", "3conv"):
        for ups, sc in ((None, 1), ("pixelshuffledirect", 2)):
            torch.manual_seed(40)
            kw = dict(upscale=sc, in_chans=3, img_range=rng, upsampler=ups, resi_connection=rc)
            ref = osw.SwinIR(sc, 3, 16, 8, rng, [2], 60, [6], 2, ups, rc)
            g = torch.Generator().manual_seed(1)
            L, Hh = torch.rand(2, 3, 16, 16, generator=g), torch.rand(2, 3, 16 * sc, 16 * sc, generator=g)
            Er = ref(L)
            torch.nn.functional.l1_loss(Er, Hh).backward()
            gr = dict(ref.named_parameters())
            for dt in ("fp32", "bf16"):
                net = SwinIR(img_size=16, window_size=8, depths=[2], embed_dim=60, num_heads=[6], mlp_ratio=2,
                             drop_path_rate=0.0, compute_dtype=dt, **kw)
                net.load_state_dict(ref.state_dict(), strict=True)
                net = net.to(dev).train()
                E = net(L.to(dev))
                torch.nn.functional.l1_loss(E, Hh.to(dev)).backward()
                errs = sorted((rel(p.grad, gr[k].grad), k) for k, p in net.named_parameters())
                print(f"range {rng:5.0f} {rc} {str(ups):20s} {dt}: E {rel(E, Er):.2e} grad median {errs[len(errs)//2][0]:.2e} "
                      f"worst {errs[-1][0]:.2e} {errs[-1][1]}", flush=True)
