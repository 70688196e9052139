"""Determinism / resume diagnostics for tests/test_checkpoint_gpu.py."""
import os
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_checkpoint_gpu as T  # noqa: E402


def sd(m):
    return torch.cat([v.detach().float().cpu().reshape(-1) for v in m.netG.state_dict().values()])


def main():
    with tempfile.TemporaryDirectory() as d:
        a, _ = T._model(os.path.join(d, "a"), False)
        T._train(a, 0, 6)
        b, _ = T._model(os.path.join(d, "b"), False)
        T._train(b, 0, 6)
        pa, pb = sd(a), sd(b)
        print("same run twice: equal", torch.equal(pa, pb), "max abs", (pa - pb).abs().max().item())
        # eager (no graph) vs graph
        os.environ["KAIR_NO_GRAPH"] = "1"
        for use_graph in (False,):
            c, _ = T._model(os.path.join(d, "c"), False)
            c.trainer.use_graph = use_graph
            T._train(c, 0, 6)
            pc = sd(c)
            print("graph vs eager: equal", torch.equal(pa, pc), "max abs", (pa - pc).abs().max().item())
        # resume
        e, _ = T._model(os.path.join(d, "e"), False)
        T._train(e, 0, 3, save_every=3)
        f, st = T._model(os.path.join(d, "e"), True)
        print("resume start", st, "t", f.trainer.t, "lr", f.G_optimizer.param_groups[0]["lr"])
        pe3 = sd(e)
        pf3 = sd(f)
        print("after load equal", torch.equal(pe3, pf3))
        print("m equal", torch.equal(e.trainer.m.cpu(), f.trainer.m.cpu()), "v equal", torch.equal(e.trainer.v.cpu(), f.trainer.v.cpu()))
        print("E equal", torch.equal(e.trainer.flat_e.cpu(), f.trainer.flat_e.cpu()))
        T._train(f, 3, 6)
        pf = sd(f)
        print("resume vs full: equal", torch.equal(pa, pf), "max abs", (pa - pf).abs().max().item())


if __name__ == "__main__":
    main()
