"""Oracle (test infrastructure only): restatement of the reference training step.

ModelPlain.optimize_parameters (/root/reference/models/model_plain.py:270-318, non-AMP branch):
    zero_grad -> E = netG(L) -> loss = w * L1(E, H) (mean) -> backward -> Adam.step -> EMA update
with the driver calling update_learning_rate (MultiStepLR.step) BEFORE the step
(/root/reference/main_train_psnr.py:176, models/model_base.py:69-71) and ModelBase.update_E
(model_base.py:247-252) applying  e = decay*e + (1-decay)*p  over named_parameters only.

Adam is written out explicitly with torch.optim.Adam's single-tensor maths (torch 2.10,
foreach=False, amsgrad=False, weight_decay=0):
    m = b1*m + (1-b1)*g ; v = b2*v + (1-b2)*g*g
    bc1 = 1-b1^t ; bc2 = 1-b2^t ; step = lr/bc1
    p -= step * m / (sqrt(v)/sqrt(bc2) + eps)
"""
import math

import torch
import torch.nn as nn


class OracleTrainer:
    def __init__(self, net, ema_net=None, lr=2e-4, betas=(0.9, 0.999), eps=1e-8, milestones=(), gamma=0.5,
                 E_decay=0.999, loss_weight=1.0, charb_eps=None):
        self.net, self.ema = net, ema_net
        self.lr0, self.betas, self.eps = lr, betas, eps
        self.milestones, self.gamma = sorted(milestones), gamma
        self.E_decay, self.loss_weight = E_decay, loss_weight
        self.charb_eps = charb_eps   # G_lossfn_type 'charbonnier' (model_plain.py:191-192, models/loss.py:208-218)
        self.params = [p for p in net.parameters() if p.requires_grad]
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0
        self.sched_steps = 0
        self.lr = lr
        if ema_net is not None:
            self.update_E(0.0)

    def update_learning_rate(self):
        """MultiStepLR.step(): lr = lr0 * gamma^(#milestones <= last_epoch)."""
        self.sched_steps += 1
        n = sum(1 for m in self.milestones if m <= self.sched_steps)
        self.lr = self.lr0 * (self.gamma ** n)

    @torch.no_grad()
    def update_E(self, decay):
        gp = dict(self.net.named_parameters())
        for k, e in self.ema.named_parameters():
            e.mul_(decay).add_(gp[k], alpha=1 - decay)

    def optimize_parameters(self, L, H, forward=None):
        for p in self.params:
            p.grad = None
        E = (forward or self.net)(L)
        if self.charb_eps is None:
            loss = self.loss_weight * nn.functional.l1_loss(E, H)
        else:
            d = E - H
            loss = self.loss_weight * torch.mean(torch.sqrt(d * d + self.charb_eps))
        loss.backward()
        self._adam()
        if self.ema is not None and self.E_decay > 0:
            self.update_E(self.E_decay)
        return E.detach(), loss.item()

    @torch.no_grad()
    def _adam(self):
        b1, b2 = self.betas
        self.t += 1
        bc1 = 1 - b1 ** self.t
        bc2 = 1 - b2 ** self.t
        step = self.lr / bc1
        bc2_sqrt = math.sqrt(bc2)
        for p, m, v in zip(self.params, self.m, self.v):
            g = p.grad
            m.lerp_(g, 1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v.sqrt() / bc2_sqrt).add_(self.eps)
            p.addcdiv_(m, denom, value=-step)
