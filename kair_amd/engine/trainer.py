"""Fused training step for the define_G networks on MI355X.

Replaces ModelPlain.optimize_parameters (/root/reference/models/model_plain.py:270-318) +
ModelBase.update_E (model_base.py:247-252) + the DDP reducer (model_base.py:113-119) with:

  forward (engine) -> L1 loss + dL/dE (kernel) -> backward (engine, grads written into ONE flat
  fp32 buffer) -> [RCCL all-reduce of the flat buffer, bucketed, divided by world size]
  -> fused Adam + EMA over the flat parameter / state buffers (one kernel)

Parameters of netG (and netE) become views into flat fp32 buffers, so state_dict()/load_state_dict
and checkpoints are unchanged.  The step is launch-only and is captured into a HIP graph after a
warm-up (torch.cuda.CUDAGraph drives HIP graphs on ROCm); replays only refresh the input batch
and the two Adam scalars.
"""
import math

import torch
import torch.distributed as dist

from .. import _hip as H
from .comm import allreduce_mean_, broadcast_params_


def flatten_params(module, device):
    """Move every parameter of `module` into one contiguous fp32 buffer (params become views)."""
    params = [p for p in module.parameters()]
    n = sum(p.numel() for p in params)
    flat = torch.empty(n, device=device, dtype=torch.float32)
    off = 0
    for p in params:
        k = p.numel()
        flat[off:off + k].copy_(p.data.reshape(-1))
        p.data = flat[off:off + k].view_as(p)
        off += k
    return flat, params


class FusedTrainer:
    def __init__(self, netG, netE=None, lr=2e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, E_decay=0.999,
                 loss_weight=1.0, use_graph=True, process_group=None, bucket_mb=25):
        self.net, self.ema_net = netG, netE
        self.device = next(netG.parameters()).device
        self.engine = netG.engine()
        self.flat_p, self.params = flatten_params(netG, self.device)
        broadcast_params_(self.flat_p, 0, process_group)   # identical start on every rank (DDP init)
        self.flat_g = torch.zeros_like(self.flat_p)
        self.m = torch.zeros_like(self.flat_p)
        self.v = torch.zeros_like(self.flat_p)
        self.flat_e = None
        if netE is not None and E_decay > 0:
            self.flat_e, _ = flatten_params(netE, self.device)
        self.grads, off = {}, 0
        for p in self.params:
            self.grads[p] = self.flat_g[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.lr = lr
        self.betas, self.eps, self.wd = betas, eps, weight_decay
        self.E_decay, self.loss_weight = E_decay, loss_weight
        self.t = 0
        self.scal = torch.zeros(2, device=self.device)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (process_group is not None or
                                                            (dist.is_available() and dist.is_initialized())) else 1
        self.bucket = max(1, int(bucket_mb * 2 ** 20 // 4))
        self.use_graph = use_graph
        self.graph = None
        self.static = None
        self.warm = 0
        self.engine._packed_version = None
        if any(b.dp > 0 for b in self.engine.blocks):
            from .swinir_engine import drop_path_scales
            drop_path_scales(self.engine, 1, self.device)   # materialise the keep-prob table eagerly

    # ------------------------------------------------------------------------------------
    def _allreduce(self):
        if self.world > 1:
            allreduce_mean_(self.flat_g, self.bucket, self.pg, self.world)

    def _fwd_bwd(self, L, Hh):
        eng = self.engine
        drop = None
        if any(b.dp > 0 for b in eng.blocks) and self.net.training:
            from .swinir_engine import drop_path_scales
            drop = drop_path_scales(eng, L.shape[0], L.device)
        eng._packed_version = None           # weights change every step: always repack
        eng.forward(L, drop)
        return eng.backward_from_loss(Hh, self.grads, self.loss_weight)

    def _update(self):
        H.adam_ema(self.flat_p, self.flat_g, self.m, self.v, self.flat_e, self.flat_p.numel(), self.scal,
                   self.betas[0], self.betas[1], self.eps, self.wd, self.E_decay if self.flat_e is not None else 0.0)

    def _body(self, L, Hh):
        loss = self._fwd_bwd(L, Hh)
        self._allreduce()
        self._update()
        return loss

    def _set_scalars(self):
        self.t += 1
        b1, b2 = self.betas
        host = torch.tensor([self.lr / (1 - b1 ** self.t), math.sqrt(1 - b2 ** self.t)], dtype=torch.float32)
        self.scal.copy_(host)   # pageable source: the host buffer is consumed before copy_ returns

    def step(self, L, Hh):
        """One training step on the batch (L, Hh) (device tensors).  Returns the device loss [1]."""
        self._set_scalars()
        if not self.use_graph:
            out = self._body(L, Hh)
            self.engine._packed_version = None
            return out
        if self.static is None or self.static[0].shape != L.shape or self.static[1].shape != Hh.shape:
            self.static = (torch.empty_like(L), torch.empty_like(Hh))
            self.graph = None
            self.warm = 0
        self.static[0].copy_(L)
        self.static[1].copy_(Hh)
        if self.graph is None and self.warm >= 2:
            # world > 1: the RCCL all-reduce stays outside the captured graphs (fwd+bwd graph,
            # eager bucketed all-reduce, update graph); single GPU: one graph for the whole step
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):        # records only; the replay below executes this step
                if self.world > 1:
                    self.loss_out = self._fwd_bwd(*self.static)
                else:
                    self.loss_out = self._body(*self.static)
            g2 = None
            if self.world > 1:
                g2 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g2):
                    self._update()
            torch.cuda.synchronize()
            self.graph = (g, g2)
        if self.graph is not None:
            self.graph[0].replay()
            if self.graph[1] is not None:
                self._allreduce()
                self.graph[1].replay()
            out = self.loss_out
        else:
            self.warm += 1
            out = self._body(*self.static)
        self.engine._packed_version = None   # params were updated in place by the Adam kernel
        return out
