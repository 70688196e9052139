"""The N > 1 trainer path end to end on the one GPU: two ranks (gloo, world size 2, spawned before
they touch the GPU) run FusedTrainer with segmented HIP graphs and the per-bucket async all-reduce
(trainer.py _replay) on 2-patch shards; losses, parameters and EMA must equal a single-process
FusedTrainer on the 4-patch batch (DropPath off).  fp32 engine, so the only difference is the
order of the fp32 gradient sums (rank partial sums vs one batch sum): agreement to ~1e-6 relative."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

STEPS = 3
B = 4


def _net(dtype):
    from kair_amd.models.network_swinir import SwinIR
    torch.manual_seed(5)
    return SwinIR(upscale=2, in_chans=3, img_size=16, window_size=8, img_range=1.0, depths=[2, 2], embed_dim=60,
                  num_heads=[6, 6], mlp_ratio=2, upsampler="pixelshuffle", drop_path_rate=0.0, compute_dtype=dtype)


def _data():
    g = torch.Generator().manual_seed(17)
    return torch.rand(B, 3, 16, 16, generator=g), torch.rand(B, 3, 32, 32, generator=g)


def _run(rank, world, port, out_dir):
    import torch.distributed as dist
    from kair_amd.engine.trainer import FusedTrainer
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        net, ema = _net("fp32"), _net("fp32")
        ema.load_state_dict(net.state_dict())
        net, ema = net.to(dev).train(), ema.to(dev).eval()
        tr = FusedTrainer(net, ema, lr=1e-3, E_decay=0.9, use_graph=True, bucket_mb=0.01)
        L, Hh = _data()
        per = B // world
        L, Hh = L[rank * per:(rank + 1) * per].to(dev), Hh[rank * per:(rank + 1) * per].to(dev)
        losses = [float(tr.step(L, Hh)) for _ in range(STEPS + 2)]   # 2 warm-up steps, then graph replays
        torch.save({"losses": losses, "p": tr.flat_p.cpu(), "e": tr.flat_e.cpu(),
                    "segmented": tr.graph is not None and tr.graph[1] is not None,
                    "buckets": len(tr.buckets or [])}, os.path.join(out_dir, f"r{rank}_w{world}.pt"))
    finally:
        if world > 1:
            dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_fused_trainer_world2_matches_single_process():
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _port()
        procs = [ctx.Process(target=_run, args=(r, 2, port, d)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=180)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        single = ctx.Process(target=_run, args=(0, 1, 0, d))
        single.start()
        single.join(timeout=180)
        assert single.exitcode == 0
        r0, r1, s = (torch.load(os.path.join(d, f), weights_only=True) for f in ("r0_w2.pt", "r1_w2.pt", "r0_w1.pt"))
    assert r0["segmented"] and r0["buckets"] > 1   # the overlapped per-bucket all-reduce path ran
    # the ranks stay in lockstep
    assert torch.equal(r0["p"], r1["p"]) and torch.equal(r0["e"], r1["e"])
    # the mean of the 2-patch shard losses is the 4-patch L1 mean
    for a, b, c in zip(r0["losses"], r1["losses"], s["losses"]):
        assert abs(0.5 * (a + b) - c) < 1e-5 * max(1.0, abs(c)), (a, b, c)
    rel = lambda x, y: ((x - y).norm() / y.norm()).item()
    assert rel(r0["p"], s["p"]) < 1e-4, rel(r0["p"], s["p"])
    assert rel(r0["e"], s["e"]) < 1e-4, rel(r0["e"], s["e"])
