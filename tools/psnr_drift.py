"""bench.py's PSNR parity (an engine vs the fp32 engine vs CPU oracle, 8 held-out patches) along one
bench training trajectory, every 20 steps: how the engine's delta depends on the trained state.
    python tools/psnr_drift.py [steps] [--dtype bf16|fp32x3]"""
import sys
import torch
sys.path.insert(0, "/root/repo")
import bench
from kair_amd.engine.trainer import FusedTrainer
from kair_amd.data.gpu_synth import PatchSynth, synthetic_pool

dev = torch.device("cuda", 0)
steps = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 160
dt = sys.argv[sys.argv.index("--dtype") + 1] if "--dtype" in sys.argv else "bf16"
net = bench.build_net(dt, 0.1).to(dev).train()
ema = bench.build_net(dt, 0.1).to(dev).eval()
ema.load_state_dict(net.state_dict())
tr = FusedTrainer(net, ema, lr=2e-4, E_decay=0.999)
pool = synthetic_pool(64, 3, 256, 256, seed=99, device=dev)
synth = PatchSynth(pool, task="sr", scale=4, H_size=192, seed=1000, rank=0, world=1)
for s in range(1, steps + 1):
    tr.step(*synth.next(32))
    if s % 20 == 0:
        torch.cuda.synchronize()
        p = bench.psnr_parity(net, dev, dt)
        print("step %4d  oracle %.5f  fp32 d %.1e  %s d %.2e (uint8 %.2e, max img %.2e / %.2e)" % (
            s, p["cpu_oracle_db"], p["fp32_delta_db"], dt, p["headline_delta_db"], p["uint8_headline_delta_db"],
            p["headline_max_single_image_delta_db"], p["uint8_headline_max_single_image_delta_db"]), flush=True)
