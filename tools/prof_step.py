"""The bench's training step alone, for rocprofv3 PMC passes: B patches (default 32), GPU patch synthesis,
graph-replayed steps; no evaluation, no other configs, so every dispatch is a full-batch one.

    python tools/prof_step.py [B] [steps] [dtype: fp32x3 (default, the bench headline) | bf16 | fp32]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from kair_amd.data.gpu_synth import PatchSynth, synthetic_pool  # noqa: E402
from kair_amd.engine.trainer import FusedTrainer  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dtype = sys.argv[3] if len(sys.argv) > 3 else "fp32x3"
    dev = torch.device("cuda", 0)
    net = bench.build_net(dtype, 0.1).to(dev).train()
    ema = bench.build_net(dtype, 0.1).to(dev).eval()
    ema.load_state_dict(net.state_dict())
    tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999)
    pool = synthetic_pool(64, 3, 256, 256, seed=99, device=dev)
    synth = PatchSynth(pool, task="sr", scale=4, H_size=192, seed=1000, rank=0, world=1)
    for _ in range(steps):
        tr.step(*synth.next(B))
    torch.cuda.synchronize()
    print("done", B, steps)


if __name__ == "__main__":
    main()
