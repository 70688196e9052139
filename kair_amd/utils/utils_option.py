"""Option-JSON surface (mirror of /root/reference/utils/utils_option.py).

parse() keeps the reference semantics (utils_option.py:24-210): '//' comments stripped line by
line, defaults filled, scale / n_channels broadcast into every dataset, paths derived, DDP flags
defaulted, max_iter / percentage milestones derived.  Differences, all relaxations of reference
failures recorded in SURVEY.md §0 "Gotchas":
  * 'speed' / 'normalization' are broadcast only when present (the fork reads them
    unconditionally, so every stock options/*.json raised KeyError: 'speed');
  * gpu_ids may be null/absent (no CUDA_VISIBLE_DEVICES rewrite then);
  * CUDA_VISIBLE_DEVICES is never rewritten after a HIP context exists.
"""
import glob
import json
import math
import os
import re
from collections import OrderedDict
from datetime import datetime


def get_timestamp():
    return datetime.now().strftime("_%y%m%d_%H%M%S")


def _strip_comments(path):
    with open(path, "r") as f:
        return "".join(line.split("//")[0] + "\n" for line in f)


def parse(opt_path, is_train=True):
    opt = json.loads(_strip_comments(opt_path), object_pairs_hook=OrderedDict)
    opt["opt_path"] = opt_path
    opt["is_train"] = is_train
    opt.setdefault("merge_bn", False)
    if "merge_bn_startpoint" not in opt:
        opt["merge_bn_startpoint"] = -1
    opt.setdefault("scale", 1)
    # datasets
    for phase, ds in opt.get("datasets", {}).items():
        ds["phase"] = phase.split("_")[0]
        ds["scale"] = opt["scale"]
        ds["n_channels"] = opt.get("n_channels", 3)
        for key in ("speed", "normalization"):
            if key in opt:
                ds[key] = opt[key]
        for key in ("dataroot_H", "dataroot_L"):
            if ds.get(key) is not None:
                ds[key] = os.path.expanduser(ds[key])
    # paths
    opt.setdefault("path", OrderedDict())
    for key, p in list(opt["path"].items()):
        if p and isinstance(p, str):
            opt["path"][key] = os.path.expanduser(p)
    root = opt["path"].get("root", ".")
    task = os.path.join(root, opt.get("task", "task"))
    opt["path"]["task"] = task
    opt["path"]["log"] = task
    opt["path"]["options"] = os.path.join(task, "options")
    if is_train:
        opt["path"]["models"] = os.path.join(task, "models")
        opt["path"]["images"] = os.path.join(task, "images")
    else:
        opt["path"]["images"] = os.path.join(task, "test_images")
    for key in ("pretrained_netG", "pretrained_netE", "pretrained_optimizerG", "pretrained_schedulerG"):
        opt["path"].setdefault(key, None)
    # network
    opt.setdefault("netG", OrderedDict())
    opt["netG"]["scale"] = opt["scale"]
    # devices (the reference exports CUDA_VISIBLE_DEVICES from gpu_ids, utils_option.py:94-96)
    gpu_ids = opt.get("gpu_ids")
    if gpu_ids:
        if "HIP_VISIBLE_DEVICES" not in os.environ and "CUDA_VISIBLE_DEVICES" not in os.environ:
            os.environ["CUDA_VISIBLE_DEVICES"] = ",".join(str(x) for x in gpu_ids)
    opt.setdefault("find_unused_parameters", False)
    opt.setdefault("use_static_graph", False)
    opt.setdefault("dist", False)
    opt["num_gpu"] = len(gpu_ids) if gpu_ids else 0
    # training derived values
    tr = opt.setdefault("train", OrderedDict())
    if is_train:
        if tr.get("max_epoch") is not None:
            ds = opt.get("datasets", {}).get("train", {})
            if all(k in ds for k in ("start_index", "end_index", "dataloader_batch_size")) and ds["dataloader_batch_size"] > 0:
                n = ds["end_index"] - ds["start_index"]
                tr["max_iter"] = math.ceil(n / ds["dataloader_batch_size"]) * tr["max_epoch"]
        if tr.get("G_scheduler_milestones_percent") is not None and tr.get("max_iter") is not None:
            tr["G_scheduler_milestones"] = [int(p * tr["max_iter"]) for p in tr["G_scheduler_milestones_percent"]]
    defaults = {"F_feature_layer": 34, "F_weights": 1.0, "F_lossfn_type": "l1", "F_use_input_norm": True,
                "F_use_range_norm": False, "G_optimizer_type": "adam", "G_optimizer_betas": [0.9, 0.999],
                "G_scheduler_restart_weights": 1, "G_optimizer_wd": 0, "G_optimizer_reuse": False,
                "G_param_strict": True, "E_param_strict": True, "E_decay": 0}
    for k, v in defaults.items():
        tr.setdefault(k, v)
    return opt


def find_last_checkpoint(save_dir, net_type="G", pretrained_path=None):
    """utils_option.py:213-235: newest '{iter}_{net_type}.pth' in save_dir, else the pretrained path."""
    files = glob.glob(os.path.join(save_dir, "*_{}.pth".format(net_type)))
    # numbered files only: the reference indexes re.findall(...)[0] and raises on 'latest_G.pth'
    iters = [int(m.group(1)) for m in (re.fullmatch(r"(\d+)_{}\.pth".format(re.escape(net_type)), os.path.basename(f))
                                        for f in files) if m]
    if iters:
        it = max(iters)
        return it, os.path.join(save_dir, "{}_{}.pth".format(it, net_type))
    return 0, pretrained_path


def save(opt):
    src = opt["opt_path"]
    dst_dir = opt["path"]["options"]
    os.makedirs(dst_dir, exist_ok=True)
    name, ext = os.path.splitext(os.path.basename(src))
    with open(os.path.join(dst_dir, name + get_timestamp() + ext), "w") as f:
        json.dump(opt, f, indent=2)


def dict2str(opt, indent_l=1):
    msg = ""
    for k, v in opt.items():
        if isinstance(v, dict):
            msg += " " * (indent_l * 2) + k + ":[\n" + dict2str(v, indent_l + 1) + " " * (indent_l * 2) + "]\n"
        else:
            msg += " " * (indent_l * 2) + k + ": " + str(v) + "\n"
    return msg


class NoneDict(dict):
    def __missing__(self, key):
        return None


def dict_to_nonedict(opt):
    if isinstance(opt, dict):
        return NoneDict(**{k: dict_to_nonedict(v) for k, v in opt.items()})
    if isinstance(opt, list):
        return [dict_to_nonedict(v) for v in opt]
    return opt
