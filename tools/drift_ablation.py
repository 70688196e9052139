"""Which bf16 rounding sites of the forward move the evaluation PSNR?  (VERDICT r3 "next" #1)

Trains the bench recipe (bf16 engine, GPU patch synthesis, B = 32, drop_path 0.1, Adam + EMA) and at
every checkpoint evaluates the bench's 8 held-out patches through the CPU oracle's module tree run on
the GPU in fp32 (TF32 off), once exactly and once per variant with selected tensors rounded to bf16
(RNE, as the kernels' conversions).  Prints the PSNR deltas of each variant against the exact run,
next to the real bf16 engine's, so the emulation's fidelity ("all" ~ engine) is visible.

    python tools/drift_ablation.py [steps] [every]
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import swinir as osw  # noqa: E402

SITES = ("xin", "wlin_qkv", "wlin_proj", "wlin_fc1", "wlin_fc2", "ln1", "qkv", "P", "O", "ln2", "h", "conv_rstb",
         "tail_fb", "tail_a0", "tail_u1", "tail_u2")
INTERNAL = ("ln1", "qkv", "P", "O", "ln2", "h")   # bf16 operands inside the fused block kernels
WLIN = ("wlin_qkv", "wlin_proj", "wlin_fc1", "wlin_fc2")
VARIANTS = ([(s, (s,)) for s in SITES] + [("all", SITES), ("internal", INTERNAL), ("internal+wlin", INTERNAL + WLIN)] +
            [(f"internal+{w}", INTERNAL + (w,)) for w in WLIN] + [("internal+wlin_attn", INTERNAL + WLIN[:2]),
                                                                 ("internal+wlin_mlp", INTERNAL + WLIN[2:])])
ON = set()


def r(name, t):
    return t.to(torch.bfloat16).to(t.dtype) if name in ON else t


def lin(name, mod, x):
    w = r("wlin_" + name, mod.weight)
    return F.linear(x, w, mod.bias)


def attn_forward(self, x, mask=None):
    Bn, N, C = x.shape
    hd = C // self.heads
    qkv = r("qkv", lin("qkv", self.qkv, x))
    q, k, v = qkv.view(Bn, N, 3, self.heads, hd).permute(2, 0, 3, 1, 4)
    s = (q * self.scale) @ k.transpose(-2, -1)
    bias = self.relative_position_bias_table[self.relative_position_index.view(-1)]
    s = s + bias.view(N, N, self.heads).permute(2, 0, 1).unsqueeze(0)
    if mask is not None:
        nW = mask.shape[0]
        s = (s.view(Bn // nW, nW, self.heads, N, N) + mask[None, :, None]).view(Bn, self.heads, N, N)
    p = r("P", torch.softmax(s, dim=-1))
    o = r("O", (p @ v).transpose(1, 2).reshape(Bn, N, C))
    return lin("proj", self.proj, o)


def mlp_forward(self, x):
    return lin("fc2", self.fc2, r("h", F.gelu(lin("fc1", self.fc1, x))))


def block_forward(self, x, size, keep=None):
    H, W = size
    B, L, C = x.shape
    h = r("ln1", self.norm1(x)).view(B, H, W, C)
    if self.shift:
        h = torch.roll(h, (-self.shift, -self.shift), (1, 2))
    mask = None if self.shift == 0 else (self.attn_mask if tuple(size) == self.res else
                                         osw.shift_region_mask(H, W, self.ws, self.shift).to(x.device))
    a = osw.from_windows(self.attn(osw.to_windows(h, self.ws), mask), self.ws, B, H, W)
    if self.shift:
        a = torch.roll(a, (self.shift, self.shift), (1, 2))
    x = x + a.reshape(B, L, C)
    return x + self.mlp(r("ln2", self.norm2(x)))


osw.WindowAttention.forward = attn_forward
osw.Mlp.forward = mlp_forward
osw.SwinTransformerBlock.forward = block_forward


def hook(site):
    def pre(mod, args):
        return (r(site, args[0]),)
    return pre


def build_ref(sd, dev):
    net = osw.SwinIR(4, 3, 48, 8, 1.0, [6] * 6, 180, [6] * 6, 2, "pixelshuffle")
    net.load_state_dict(sd, strict=True)
    net = net.to(dev).eval()
    net.conv_first.register_forward_pre_hook(hook("xin"))
    for layer in net.layers:
        layer.conv.register_forward_pre_hook(hook("conv_rstb"))
    net.conv_after_body.register_forward_pre_hook(hook("conv_rstb"))
    net.conv_before_upsample[0].register_forward_pre_hook(hook("tail_fb"))
    net.upsample[0].register_forward_pre_hook(hook("tail_a0"))
    net.upsample[2].register_forward_pre_hook(hook("tail_u1"))
    net.conv_last.register_forward_pre_hook(hook("tail_u2"))
    return net


def metrics(E, Er, Hh):
    from kair_amd.utils import utils_image as U
    n = E.shape[0]
    pf = [U.psnr_float(E[i:i + 1], Hh[i:i + 1]) - U.psnr_float(Er[i:i + 1], Hh[i:i + 1]) for i in range(n)]
    pu = [U.calculate_psnr(U.tensor2uint(E[i]), U.tensor2uint(Hh[i]), border=4) -
          U.calculate_psnr(U.tensor2uint(Er[i]), U.tensor2uint(Hh[i]), border=4) for i in range(n)]
    return {"d8": abs(sum(pf) / n), "u8": abs(sum(pu) / n), "dmax": max(map(abs, pf)), "umax": max(map(abs, pu)),
            "rms_err": float((E - Er).pow(2).mean().sqrt())}


def main():
    from kair_amd.engine.trainer import FusedTrainer
    from kair_amd.data.gpu_synth import PatchSynth, synthetic_pool
    from kair_amd.utils import utils_image as U
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 160
    every = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dev = torch.device("cuda", 0)
    net = bench.build_net("bf16", 0.1).to(dev).train()
    ema = bench.build_net("bf16", 0.1).to(dev).eval()
    ema.load_state_dict(net.state_dict())
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999)
    pool = synthetic_pool(64, 3, 256, 256, seed=99, device=dev)
    synth = PatchSynth(pool, task="sr", scale=4, H_size=192, seed=1000, rank=0, world=1)
    L, Hh = U.synth_sr_batch(8, 48, 4, seed=77)
    for s in range(1, steps + 1):
        tr.step(*synth.next(32))
        if s % every:
            continue
        torch.cuda.synchronize()
        sd = {k: v.detach().float().clone() for k, v in net.state_dict().items()}
        ref = build_ref(sd, dev)
        net.eval()
        with torch.no_grad():
            Eb = net(L.to(dev)).float().cpu()
            ON.clear()
            Er = ref(L.to(dev)).float().cpu()
            rows = {"engine_bf16": metrics(Eb, Er, Hh)}
            from kair_amd.engine.swinir_engine import SwinIREngine
            for name, kw in (("engine_bf16_no_split_act", dict(split_act=False)),
                             ("engine_bf16_split_linear", dict(split_linear=True))):
                n2 = bench.build_net("bf16", 0.0).to(dev).eval()
                n2.load_state_dict(sd, strict=True)
                n2._engine = SwinIREngine(n2, "bf16", **kw)
                rows[name] = metrics(n2(L.to(dev)).float().cpu(), Er, Hh)
                del n2
            for name, v in VARIANTS:
                ON.clear()
                ON.update(v)
                rows[name] = metrics(ref(L.to(dev)).float().cpu(), Er, Hh)
        net.train()
        ON.clear()
        del ref
        for k, m in rows.items():
            print(json.dumps({"step": s, "variant": k, **{a: float("%.3g" % b) for a, b in m.items()}}), flush=True)


if __name__ == "__main__":
    main()
