"""ModelBase — trainer plumbing (mirror of /root/reference/models/model_base.py:14-275).

Kept: network save/load (strict, or non-strict copy-by-position; 'params' key unwrap,
model_base.py:158-216), optimizer / scheduler save & load in torch's own state_dict formats
(221-245), update_E EMA over parameters only (247-252), get_bare_model.
Changed for MI355X: a network with a HIP step program (`engine`) is not wrapped in DDP here.
When ModelPlain then uses the fused trainer, kair_amd.engine.trainer.FusedTrainer owns the
gradient all-reduce (RCCL, flat buffer); when it falls back to the autograd + torch.optim path
(l2 loss, grad clipping, regularizers, ...) ModelPlain.define_optimizer wraps the network in
DistributedDataParallel then (wrap_ddp), so ranks never train divergent replicas.  With dist on,
rank 0's parameters and buffers are broadcast at construction (the reference's DDP construction
does this, model_base.py:116) before netE is seeded from netG.
The SPECT evaluation helpers (model_base.py:280-569) are out of scope.
"""
import os

import torch
import torch.nn as nn
from torch.nn.parallel import DataParallel, DistributedDataParallel


class ModelBase:
    def __init__(self, opt):
        self.opt = opt
        self.save_dir = opt["path"]["models"]
        # model_base.py:18 -- 'cuda' when gpu_ids is set, else the host.  Only DnCNN (BASELINE
        # config 1) has a host path; the other networks raise on CPU tensors.
        if opt.get("gpu_ids") is not None:
            if not torch.cuda.is_available():
                raise RuntimeError("kair_amd: gpu_ids is set but no HIP device is visible")
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")
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
        if self.opt.get("dist"):
            self.broadcast_from_rank0(network)
        if hasattr(network, "engine") and self.device.type == "cuda":
            return network           # DDP decided in define_optimizer (fused trainer or wrap_ddp)
        if self.opt.get("dist"):
            return self.wrap_ddp(network)
        return network

    def wrap_ddp(self, network):
        """DistributedDataParallel as in model_base.py:113-119 (no-op when already wrapped)."""
        if isinstance(network, (DataParallel, DistributedDataParallel)):
            return network
        ids = [torch.cuda.current_device()] if self.device.type == "cuda" else None
        net = DistributedDataParallel(network, device_ids=ids,
                                      find_unused_parameters=self.opt.get("find_unused_parameters", False))
        if self.opt.get("use_static_graph"):
            net._set_static_graph()
        return net

    @staticmethod
    @torch.no_grad()
    def broadcast_from_rank0(network):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            for t in network.state_dict().values():
                dist.broadcast(t, 0)

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
