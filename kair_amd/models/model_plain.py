"""ModelPlain — pixel-loss trainer (mirror of /root/reference/models/model_plain.py:15-402).

optimize_parameters keeps the reference order (zero_grad -> forward -> w*L1 -> backward -> Adam ->
log G_loss -> EMA update_E) but, for networks with a fused MI355X engine and the 'l1' loss, runs it
as ONE launch-only step captured in a HIP graph (kair_amd.engine.trainer.FusedTrainer): the grads
land in a flat buffer, are all-reduced over RCCL when dist is on, and one kernel applies Adam +
EMA.  The optimizer object is a torch.optim.Optimizer subclass whose state_dict() is torch Adam's
format, so '{iter}_optimizerG.pth' interchanges with the reference; the scheduler is torch's
MultiStepLR stepped before the optimizer step exactly as main_train_psnr.py:176 does.
"""
from collections import OrderedDict

import torch
import torch.nn as nn
from torch.optim import Adam, lr_scheduler

from ..engine.trainer import FusedTrainer
from .model_base import ModelBase
from .select_network import define_G


class FusedAdam(torch.optim.Optimizer):
    """torch-compatible facade over FusedTrainer's flat Adam state (param_groups drive the lr)."""

    def __init__(self, params, trainer, lr, betas, eps, weight_decay):
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None))
        self.trainer = trainer

    def step(self, closure=None):   # the fused step runs inside FusedTrainer.step
        raise RuntimeError("FusedAdam.step is driven by FusedTrainer.step")

    def state_dict(self):
        t = self.trainer
        st, off = {}, 0
        for i, p in enumerate(t.params):
            n = p.numel()
            st[i] = {"step": torch.tensor(float(t.t)),
                     "exp_avg": t.m[off:off + n].view_as(p).detach().cpu().clone(),
                     "exp_avg_sq": t.v[off:off + n].view_as(p).detach().cpu().clone()}
            off += n
        groups = []
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(len(t.params)))
            groups.append(d)
        return {"state": st, "param_groups": groups}

    def load_state_dict(self, sd):
        """torch.optim.Adam state_dict format; validated like torch (group sizes, per-parameter
        shapes, one shared step count) before anything is copied."""
        t = self.trainer
        groups = sd.get("param_groups", [])
        if len(groups) != len(self.param_groups) or sum(len(g["params"]) for g in groups) != len(t.params):
            raise ValueError("loaded state dict contains a parameter group that doesn't match the size of "
                             "optimizer's group")
        ids = [i for g in groups for i in g["params"]]
        state = sd.get("state", {})
        steps = set()
        for i, p in zip(ids, t.params):
            s = state.get(i, state.get(str(i)))
            if s is None:
                continue
            if tuple(s["exp_avg"].shape) != tuple(p.shape) or tuple(s["exp_avg_sq"].shape) != tuple(p.shape):
                raise ValueError(f"optimizer state for parameter {i}: shape {tuple(s['exp_avg'].shape)} != {tuple(p.shape)}")
            steps.add(int(float(s["step"])))
        if len(steps) > 1:
            raise ValueError(f"optimizer state has per-parameter step counts {sorted(steps)}; the fused Adam keeps one")
        off = 0
        for i, p in zip(ids, t.params):
            n = p.numel()
            s = state.get(i, state.get(str(i)))
            if s is not None:
                t.m[off:off + n].copy_(s["exp_avg"].reshape(-1))
                t.v[off:off + n].copy_(s["exp_avg_sq"].reshape(-1))
            else:
                t.m[off:off + n].zero_()
                t.v[off:off + n].zero_()
            off += n
        if steps:
            t.t = steps.pop()
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for k in ("lr", "betas", "eps", "weight_decay", "initial_lr"):
                if k in sg:
                    g[k] = sg[k]


class CharbonnierLoss(nn.Module):
    """models/loss.py:208-218: mean(sqrt((x - y)^2 + eps)) (the autograd path's loss)."""

    def __init__(self, eps=1e-9):
        super().__init__()
        self.eps = eps

    def forward(self, x, y):
        d = x - y
        return torch.mean(torch.sqrt(d * d + self.eps))


class ModelPlain(ModelBase):
    """Train with pixel loss."""

    def __init__(self, opt):
        super().__init__(opt)
        self.opt_train = self.opt["train"]
        self.netG = self.model_to_device(define_G(opt))
        if self.opt_train["E_decay"] > 0:
            self.netE = define_G(opt).to(self.device).eval()
        # amp_enabled selects the bf16 engine in define_G (select_network.compute_dtype_of); the step itself is
        # the same fused trainer at either precision
        self.amp_enabled = bool(self.opt_train.get("amp_enabled", False))
        self.trainer = None
        self.log_dict = OrderedDict()

    # ------------------------------------------------------------------ preparation
    def init_train(self):
        self.load()
        self.netG.train()
        self.define_loss()
        self.define_optimizer()
        self.load_optimizers()
        self.define_scheduler()
        self.load_scheduler_states()
        self.log_dict = OrderedDict()

    def load(self):
        p = self.opt["path"].get("pretrained_netG")
        if p is not None:
            self.load_network(p, self.netG, strict=self.opt_train["G_param_strict"], param_key="params")
        if self.opt_train["E_decay"] > 0:
            pe = self.opt["path"].get("pretrained_netE")
            if pe is not None:
                self.load_network(pe, self.netE, strict=self.opt_train["E_param_strict"], param_key="params_ema")
            else:
                self.update_E(0)
            self.netE.eval()

    def load_optimizers(self):
        p = self.opt["path"].get("pretrained_optimizerG")
        if p is not None and self.opt_train["G_optimizer_reuse"]:
            self.load_optimizer(p, self.G_optimizer)

    def load_scheduler_states(self):
        p = self.opt["path"].get("pretrained_schedulerG")
        if p is not None and self.schedulers:
            self.load_scheduler(p, self.schedulers[0])

    def save(self, iter_label):
        import os
        os.makedirs(self.save_dir, exist_ok=True)
        self._delete_old_checkpoints("G")
        self.save_network(self.save_dir, self.netG, "G", iter_label)
        if self.opt_train["E_decay"] > 0:
            self._delete_old_checkpoints("E")
            self.save_network(self.save_dir, self.netE, "E", iter_label)
        if self.opt_train["G_optimizer_reuse"]:
            self._delete_old_checkpoints("optimizerG")
            self.save_optimizer(self.save_dir, self.G_optimizer, "optimizerG", iter_label)
        if self.schedulers:
            self._delete_old_checkpoints("schedulerG")
            self.save_scheduler(self.save_dir, self.schedulers[0], "schedulerG", iter_label)

    def _delete_old_checkpoints(self, model_type):
        """model_plain.py:149-176 — keep only the newest '{iter}_{type}.pth' (called before saving)."""
        import os
        import re
        if not os.path.isdir(self.save_dir):
            return
        found = []
        for fn in os.listdir(self.save_dir):
            if fn.endswith(f"_{model_type}.pth"):
                m = re.match(r"(\d+)_", fn)
                if m:
                    found.append((int(m.group(1)), fn))
        found.sort(reverse=True)
        for _, fn in found[1:]:
            os.remove(os.path.join(self.save_dir, fn))

    # ------------------------------------------------------------------ loss / optim / sched
    def define_loss(self):
        t = self.opt_train["G_lossfn_type"]
        self.G_lossfn_type = t
        if t == "l1":
            self.G_lossfn = nn.L1Loss()
        elif t == "l2":
            self.G_lossfn = nn.MSELoss()
        elif t == "l2sum":
            self.G_lossfn = nn.MSELoss(reduction="sum")
        elif t == "charbonnier":   # models/loss.py:208-218; the fused trainer runs kair_charbonnier_loss
            self.G_lossfn = CharbonnierLoss(self.opt_train.get("G_charbonnier_eps", 1e-9))
        else:
            raise NotImplementedError("Loss type [{:s}] is not on the kair_amd path.".format(t))
        self.G_lossfn_weight = self.opt_train["G_lossfn_weight"]

    def _fused_ok(self):
        net = self.get_bare_model(self.netG)
        return (hasattr(net, "engine") and self.device.type == "cuda" and all(p.requires_grad for p in net.parameters())
                and self.G_lossfn_type in ("l1", "charbonnier") and not self.opt_train.get("G_optimizer_clipgrad")
                and self.opt_train["G_optimizer_type"] == "adam"
                and not self.opt_train.get("G_regularizer_orthstep") and not self.opt_train.get("G_regularizer_clipstep"))

    def define_optimizer(self):
        params = [p for p in self.netG.parameters() if p.requires_grad]
        tr = self.opt_train
        if self._fused_ok():
            netE = self.netE if tr["E_decay"] > 0 else None
            self.trainer = FusedTrainer(self.get_bare_model(self.netG), netE, lr=tr["G_optimizer_lr"],
                                        betas=tuple(tr["G_optimizer_betas"]), eps=1e-8,
                                        weight_decay=tr["G_optimizer_wd"], E_decay=tr["E_decay"],
                                        loss_weight=self.G_lossfn_weight,
                                        charb_eps=(tr.get("G_charbonnier_eps", 1e-9) if self.G_lossfn_type == "charbonnier"
                                                   else None),
                                        use_graph=tr.get("use_hip_graph", True))
            self.G_optimizer = FusedAdam(self.trainer.params, self.trainer, tr["G_optimizer_lr"],
                                         tr["G_optimizer_betas"], 1e-8, tr["G_optimizer_wd"])
        else:
            if tr["G_optimizer_type"] != "adam":
                raise NotImplementedError
            self.trainer = None
            if self.opt.get("dist"):   # autograd path: DDP owns the all-reduce (model_base.py:113-119)
                self.netG = self.wrap_ddp(self.netG)
            self.G_optimizer = Adam(params, lr=tr["G_optimizer_lr"], betas=tr["G_optimizer_betas"],
                                    weight_decay=tr["G_optimizer_wd"])

    def define_scheduler(self):
        tr = self.opt_train
        if tr["G_scheduler_type"] == "MultiStepLR":
            self.schedulers.append(lr_scheduler.MultiStepLR(self.G_optimizer, tr["G_scheduler_milestones"],
                                                            tr["G_scheduler_gamma"]))
        elif tr["G_scheduler_type"] == "CosineAnnealingWarmRestarts":
            self.schedulers.append(lr_scheduler.CosineAnnealingWarmRestarts(
                self.G_optimizer, tr["G_scheduler_periods"], tr["G_scheduler_restart_weights"], tr["G_scheduler_eta_min"]))
        else:
            raise NotImplementedError

    # ------------------------------------------------------------------ step
    def feed_data(self, data, need_H=True):
        self.L = data["L"].to(self.device, non_blocking=True)
        if need_H:
            self.H = data["H"].to(self.device, non_blocking=True)

    def netG_forward(self):
        self.E = self.netG(self.L)

    def optimize_parameters(self, current_step):
        if self.trainer is not None:
            self.trainer.lr = self.G_optimizer.param_groups[0]["lr"]
            loss = self.trainer.step(self.L, self.H, *self._step_cond())
            self.trainer.check_range()   # fp32x3: settle this step's range flag now (the loss is read below anyway)
            self.E = None  # the fused step keeps E in its plan buffer; test() recomputes
            self.log_dict["G_loss"] = loss.item()
            return
        self.G_optimizer.zero_grad()
        self.netG_forward()
        G_loss = self.G_lossfn_weight * self.G_lossfn(self.E, self.H)
        G_loss.backward()
        clip = self.opt_train.get("G_optimizer_clipgrad") or 0
        if clip > 0:
            torch.nn.utils.clip_grad_norm_(self.netG.parameters(), max_norm=clip, norm_type=2)
        self.G_optimizer.step()
        self.log_dict["G_loss"] = G_loss.item()
        if self.opt_train["E_decay"] > 0:
            self.update_E(self.opt_train["E_decay"])

    def _step_cond(self):
        """Extra forward inputs of the fused step (none for the single-input networks)."""
        return ()

    def test(self):
        self.netG.eval()
        with torch.no_grad():
            self.netG_forward()
        self.netG.train()

    def testx8(self):
        from ..utils.utils_model import test_mode
        self.netG.eval()
        with torch.no_grad():
            self.E = test_mode(self.netG, self.L, mode=3, sf=self.opt["scale"], modulo=1)
        self.netG.train()

    def current_log(self):
        return self.log_dict

    def current_visuals(self, need_H=True):
        out = OrderedDict()
        out["L"] = self.L.detach()[0].float().cpu()
        out["E"] = self.E.detach()[0].float().cpu()
        if need_H:
            out["H"] = self.H.detach()[0].float().cpu()
        return out

    def current_results(self, need_H=True):
        out = OrderedDict()
        out["L"] = self.L.detach().float().cpu()
        out["E"] = self.E.detach().float().cpu()
        if need_H:
            out["H"] = self.H.detach().float().cpu()
        return out

    def print_network(self):
        print(self.describe_network(self.netG))

    def print_params(self):
        print(self.describe_params(self.netG))

    def info_network(self):
        return self.describe_network(self.netG)

    def info_params(self):
        return self.describe_params(self.netG)
