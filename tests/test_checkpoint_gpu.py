"""Checkpoint interop: save -> find_last_checkpoint -> resume reproduces the
uninterrupted trajectory bit for bit, through define_Model / ModelPlain / the fused trainer, the
reference's file names ('{iter}_G.pth', '_E', '_optimizerG', '_schedulerG', model_plain.py:138-176)
and its resume recipe (main_train_psnr.py:70-90: pretrained_* paths from find_last_checkpoint,
G_optimizer_reuse).  DropPath off: the reference does not checkpoint RNG state either."""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from kair_amd.models.select_model import define_Model  # noqa: E402
from kair_amd.utils import utils_option as option  # noqa: E402

OPT = {
    "task": "ckpt", "model": "plain", "gpu_ids": [0], "scale": 2, "n_channels": 3,
    "path": {"root": None, "pretrained_netG": None, "pretrained_netE": None},
    "netG": {"net_type": "swinir", "upscale": 2, "in_chans": 3, "img_size": 16, "window_size": 8, "img_range": 1.0,
             "depths": [2, 2], "embed_dim": 60, "num_heads": [6, 6], "mlp_ratio": 2, "upsampler": "pixelshuffle",
             "resi_connection": "1conv", "init_type": "default",
             "drop_path_rate": 0.0},
    "train": {"G_lossfn_type": "l1", "G_lossfn_weight": 1.0, "E_decay": 0.999, "G_optimizer_type": "adam",
              "G_optimizer_lr": 2e-4, "G_optimizer_wd": 0, "G_optimizer_clipgrad": None, "G_optimizer_reuse": True,
              "G_scheduler_type": "MultiStepLR", "G_scheduler_milestones": [3, 5], "G_scheduler_gamma": 0.5,
              "G_param_strict": True, "E_param_strict": True, "checkpoint_save": 3},
}


def _batch(step):
    g = torch.Generator().manual_seed(100 + step)
    return {"L": torch.rand(2, 3, 16, 16, generator=g), "H": torch.rand(2, 3, 32, 32, generator=g)}


def _model(tmp, resume):
    d = json.loads(json.dumps(OPT))
    d["path"]["root"] = str(tmp)
    os.makedirs(str(tmp), exist_ok=True)
    path = os.path.join(str(tmp), "opt.json")
    with open(path, "w") as f:
        json.dump(d, f)
    opt = option.parse(path, is_train=True)
    start = 0
    if resume:
        md = opt["path"]["models"]
        start, opt["path"]["pretrained_netG"] = option.find_last_checkpoint(md, net_type="G")
        _, opt["path"]["pretrained_netE"] = option.find_last_checkpoint(md, net_type="E")
        _, opt["path"]["pretrained_optimizerG"] = option.find_last_checkpoint(md, net_type="optimizerG")
        _, opt["path"]["pretrained_schedulerG"] = option.find_last_checkpoint(md, net_type="schedulerG")
    opt = option.dict_to_nonedict(opt)
    torch.manual_seed(0)
    m = define_Model(opt)
    m.init_train()
    return m, start


def _train(m, start, stop, save_every=None):
    for step in range(start + 1, stop + 1):
        m.update_learning_rate(step)
        m.feed_data(_batch(step))
        m.optimize_parameters(step)
        if save_every and step % save_every == 0:
            m.save(step)


def test_save_find_resume_bitwise(tmp_path):
    a, _ = _model(tmp_path / "run", resume=False)
    assert a.trainer is not None   # the fused, graph-captured trainer
    _train(a, 0, 6, save_every=3)
    full_G = {k: v.detach().cpu().clone() for k, v in a.netG.state_dict().items()}
    full_E = {k: v.detach().cpu().clone() for k, v in a.netE.state_dict().items()}
    lr_a = a.G_optimizer.param_groups[0]["lr"]
    files = sorted(os.listdir(a.save_dir))
    assert {"6_G.pth", "6_E.pth", "6_optimizerG.pth", "6_schedulerG.pth"} <= set(files), files
    # the reference prunes BEFORE saving and keeps the newest existing file: previous + new remain
    assert sorted(f for f in files if f.endswith("_G.pth")) == ["3_G.pth", "6_G.pth"], files
    # resume from iteration 3: keep only the iteration-3 files, as if the run had stopped there
    for f in files:
        os.remove(os.path.join(a.save_dir, f))
    del a
    b, _ = _model(tmp_path / "run3", resume=False)
    _train(b, 0, 3, save_every=3)
    del b
    c, start = _model(tmp_path / "run3", resume=True)
    assert start == 3
    assert c.trainer.t == 3
    _train(c, 3, 6)
    assert c.G_optimizer.param_groups[0]["lr"] == lr_a
    for k, v in c.netG.state_dict().items():
        assert torch.equal(v.detach().cpu(), full_G[k]), k
    for k, v in c.netE.state_dict().items():
        assert torch.equal(v.detach().cpu(), full_E[k]), k
