"""ModelBase — trainer plumbing (mirror of /root/reference/models/model_base.py:14-275).

Kept: network save/load (strict, or non-strict copy-by-position; 'params' key unwrap,
model_base.py:158-216), optimizer / scheduler save & load in torch's own state_dict formats
(221-245), update_E EMA over parameters only (247-252), get_bare_model.
Changed for MI355X: model_to_device does not wrap the fused-engine networks in DDP — their
gradient all-reduce is done by kair_amd.engine.trainer.FusedTrainer on the flat gradient buffer
(RCCL); other modules keep DistributedDataParallel.  The SPECT evaluation helpers
(model_base.py:280-569) are out of scope.
"""
import os

import torch
import torch.nn as nn
from torch.nn.parallel import DataParallel, DistributedDataParallel


class ModelBase:
    def __init__(self, opt):
        self.opt = opt
        self.save_dir = opt["path"]["models"]
        if not torch.cuda.is_available():
            raise RuntimeError("kair_amd trains on the MI355X (HIP device) only; no CPU fallback")
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.is_train = opt["is_train"]
        self.schedulers = []

    # -------------------------------------------------------------- hooks (overridden)
    def init_train(self):
        pass

    def load(self):
        pass

    def save(self, label):
        pass

    def define_loss(self):
        pass

    def define_optimizer(self):
        pass

    def define_scheduler(self):
        pass

    def feed_data(self, data):
        pass

    def optimize_parameters(self, current_step):
        pass

    def current_visuals(self):
        pass

    def current_losses(self):
        pass

    def update_learning_rate(self, n):
        for scheduler in self.schedulers:
            scheduler.step()

    def current_learning_rate(self):
        return self.schedulers[0].get_last_lr()[0]

    def requires_grad(self, model, flag=True):
        for p in model.parameters():
            p.requires_grad = flag

    # -------------------------------------------------------------- devices
    def get_bare_model(self, network):
        if isinstance(network, (DataParallel, DistributedDataParallel)):
            network = network.module
        return network

    def model_to_device(self, network):
        network = network.to(self.device)
        if hasattr(network, "engine") and getattr(network, "fused_trainable", True):
            return network           # fused engine: FusedTrainer owns the gradient all-reduce
        if self.opt.get("dist"):
            return DistributedDataParallel(network, device_ids=[torch.cuda.current_device()],
                                           find_unused_parameters=self.opt.get("find_unused_parameters", False))
        return network

    # -------------------------------------------------------------- info
    def describe_network(self, network):
        network = self.get_bare_model(network)
        return "\nNetworks name: {}\nParams number: {}\nNet structure:\n{}\n".format(
            network.__class__.__name__, sum(p.numel() for p in network.parameters()), str(network))

    def describe_params(self, network):
        network = self.get_bare_model(network)
        msg = "\n | {:^6s} | {:^6s} | {:^6s} | {:^6s} || {:<20s}\n".format("mean", "min", "max", "std", "shape")
        for name, p in network.state_dict().items():
            if "num_batches_tracked" not in name:
                v = p.data.clone().float()
                msg += " | {:>6.3f} | {:>6.3f} | {:>6.3f} | {:>6.3f} | {} || {:s}\n".format(
                    v.mean(), v.min(), v.max(), v.std(), v.shape, name)
        return msg

    # -------------------------------------------------------------- save / load
    def save_network(self, save_dir, network, network_label, iter_label):
        path = os.path.join(save_dir, "{}_{}.pth".format(iter_label, network_label))
        network = self.get_bare_model(network)
        torch.save({k: v.detach().cpu() for k, v in network.state_dict().items()}, path)

    def load_network(self, load_path, network, strict=True, param_key="params"):
        network = self.get_bare_model(network)
        sd = torch.load(load_path, map_location="cpu", weights_only=True)
        if param_key in sd.keys():
            sd = sd[param_key]
        if strict:
            network.load_state_dict(sd, strict=True)
        else:   # copy by position (model_base.py:208-216)
            cur = network.state_dict()
            for (_, v_old), k in zip(sd.items(), list(cur.keys())):
                cur[k] = v_old
            network.load_state_dict(cur, strict=True)

    def save_optimizer(self, save_dir, optimizer, optimizer_label, iter_label):
        torch.save(optimizer.state_dict(), os.path.join(save_dir, "{}_{}.pth".format(iter_label, optimizer_label)))

    def load_optimizer(self, load_path, optimizer):
        optimizer.load_state_dict(torch.load(load_path, map_location="cpu", weights_only=True))

    def save_scheduler(self, save_dir, scheduler, scheduler_label, iter_label):
        torch.save(scheduler.state_dict(), os.path.join(save_dir, "{}_{}.pth".format(iter_label, scheduler_label)))

    def load_scheduler(self, load_path, scheduler):
        scheduler.load_state_dict(torch.load(load_path, map_location="cpu", weights_only=True))

    @torch.no_grad()
    def update_E(self, decay=0.999):
        netG = self.get_bare_model(self.netG)
        g = dict(netG.named_parameters())
        for k, e in self.netE.named_parameters():
            e.data.mul_(decay).add_(g[k].data, alpha=1 - decay)

    # -------------------------------------------------------------- BN merge (DnCNN)
    def merge_bnorm_train(self):
        from ..utils.utils_bnorm import merge_bn, tidy_sequential
        merge_bn(self.netG)
        tidy_sequential(self.netG)
        self.define_optimizer()
        self.define_scheduler()

    def merge_bnorm_test(self):
        from ..utils.utils_bnorm import merge_bn, tidy_sequential
        merge_bn(self.netG)
        tidy_sequential(self.netG)
