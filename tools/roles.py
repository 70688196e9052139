"""Every libkair launch of one SwinIR classical x4 training step, by call site, with its kernel duration
(bench.time_roles: dispatch-packet timestamps of every launch, as rocprofv3 --kernel-trace reports them;
serial by default: the side-stream work in place).

    python tools/roles.py [B] [--in-step] [--dtype bf16|fp32|fp32x3]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from kair_amd.engine.trainer import FusedTrainer  # noqa: E402
from kair_amd.utils.utils_image import synth_sr_batch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 32
    dev = torch.device("cuda", 0)
    dt = sys.argv[sys.argv.index("--dtype") + 1] if "--dtype" in sys.argv else "bf16"
    net = bench.build_net(dt, 0.1).to(dev).train()
    ema = bench.build_net(dt, 0.1).to(dev).eval()
    ema.load_state_dict(net.state_dict())
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999)
    L, Hh = synth_sr_batch(B, 48, 4, seed=1000, device=dev)
    for _ in range(3):
        tr.step(L, Hh)
    torch.cuda.synchronize()
    roles, kernels = bench.time_roles(tr, serial="--in-step" not in sys.argv)
    tot = sum(v["ms_total"] for v in kernels.values())
    print(f"B = {B}: {tot:.3f} ms of kernel time over {sum(v['launches'] for v in kernels.values())} launches")
    for k, v in sorted(roles.items(), key=lambda kv: -kv[1]["ms_total"]):
        gbs = f"{v['bytes'] / (v['ms'] * 1e-3) / 1e9:7.0f} GB/s" if v.get("bytes") else " " * 12
        print(f"{v['ms_total']:8.3f} ms {v['launches']:4d}x {1e3 * v['ms']:8.1f} us {gbs}  {v['kernel'][:40]:40s} {k}")
    print("per kernel:")
    for v in sorted(kernels.values(), key=lambda v: -v["ms_total"]):
        print(f"{v['ms_total']:8.3f} ms {v['launches']:4d}x {1e3 * v['ms']:8.1f} us  {v['kernel']}")


if __name__ == "__main__":
    main()
