"""Fused training step for the define_G networks on MI355X.

Replaces ModelPlain.optimize_parameters (/root/reference/models/model_plain.py:270-318) +
ModelBase.update_E (model_base.py:247-252) + the DDP reducer (model_base.py:113-119) with:

  forward (engine) -> L1 loss + dL/dE (kernel) -> backward (engine, grads written into ONE flat
  fp32 buffer) -> [RCCL all-reduce of the flat buffer, bucketed, divided by world size]
  -> fused Adam + EMA over the flat parameter / state buffers (one kernel)

Parameters of netG (and netE) become views into flat fp32 buffers, so state_dict()/load_state_dict
and checkpoints are unchanged.  The step is launch-only and is captured into HIP graphs after a
warm-up (torch.cuda.CUDAGraph drives HIP graphs on ROCm); replays only refresh the input batch
and the two Adam scalars.

Data parallel (world > 1): the fwd+bwd capture is cut into one graph per gradient segment of the
engine (engine.grad_segments(): for SwinIR the reconstruction tail, then each RSTB, last to first).
After replaying segment k the host issues the RCCL all-reduce of bucket k (async, on RCCL's own
stream, ordered after the replay by an event) and goes on replaying segment k+1, so every bucket
but the last overlaps the remaining backward.  The update graph (mean scale + Adam + EMA) waits
for all buckets.  RCCL is never captured inside a graph.
"""
import math

import torch
import torch.distributed as dist

from .. import _hip as H
from .comm import allreduce_mean_, allreduce_sum_, broadcast_params_


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


def segment_buckets(params, segs):
    """Flat-buffer ranges [(lo, hi)] (params laid out in `params` order) of the gradient segments
    `segs` (parameter lists in backward order), or None when a segment is not contiguous or the
    segments do not tile the buffer."""
    pos, off = {}, 0
    for p in params:
        pos[p] = (off, off + p.numel())
        off += p.numel()
    out = []
    for plist in segs:
        if not plist:
            return None
        lo, hi = min(pos[p][0] for p in plist), max(pos[p][1] for p in plist)
        if hi - lo != sum(p.numel() for p in plist):
            return None
        out.append((lo, hi))
    cover = sorted(out)
    if cover[0][0] != 0 or cover[-1][1] != off or any(a[1] != b[0] for a, b in zip(cover, cover[1:])):
        return None
    return out


class FusedTrainer:
    def __init__(self, netG, netE=None, lr=2e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, E_decay=0.999,
                 loss_weight=1.0, use_graph=True, process_group=None, bucket_mb=25, segment_graphs=None, charb_eps=None,
                 stream_priority=0):
        self.net, self.ema_net = netG, netE
        self.stream_priority = stream_priority   # torch priority of the capture stream (0: default)
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
        # None: L1 (G_lossfn_type 'l1'); a float: the Charbonnier loss with that eps ('charbonnier')
        self.charb_eps = charb_eps
        self.t = 0
        self.scal = torch.zeros(2, device=self.device)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (process_group is not None or
                                                            (dist.is_available() and dist.is_initialized())) else 1
        self.bucket = max(1, int(bucket_mb * 2 ** 20 // 4))
        self.use_graph = use_graph
        # one graph per gradient segment: on for world > 1 (overlapped all-reduce); forcible on one GPU
        self.segment_graphs = (self.world > 1) if segment_graphs is None else bool(segment_graphs)
        self.graph = None
        self.static = None
        self.warm = 0
        self.engine._packed_version = None
        # fp32x3 range guard: the split-fp16 operands have a fixed power-of-2 window per tensor class; a value that
        # leaves it (fp16 overflow) turns the step's gradients non-finite.  Each step ends with kair_range_check over
        # the flat gradients / parameters (+ the loss on one GPU) into a device flag that the Adam kernel reads (a
        # flagged step updates nothing); the host reads the flag one step later (pinned copy + event), lowers the
        # engine's exponents (x3_backoff) and re-runs the flagged step on its own batch before going on.
        self.range_guard = bool(getattr(self.engine, "x3", False))
        self.range_events = []   # (step, flag bits, (activation exp, gradient exp offset) after the back-off)
        if self.range_guard:
            self.rflag = torch.zeros(1, dtype=torch.int32, device=self.device)
            self.rflag_host = torch.zeros(1, dtype=torch.int32).pin_memory()
            self.rflag_evt = torch.cuda.Event()
            self._rflag_pending = False
            # parameters: only non-finite ones are flagged here (a weight outside its pack window, |w| >= 2^(16 -
            # KAIR_X3_WEXP) = 16, overflows its fp16 pack and shows in the gradients like any other operand; the
            # activation / gradient back-off cannot cure it, so the guard raises after X3_BACKOFF_MAX re-runs)
            self.p_limit = 3.0e38
        if any(b.dp > 0 for b in self.engine.blocks):
            from .swinir_engine import drop_path_scales
            drop_path_scales(self.engine, 1, self.device)   # materialise the keep-prob table eagerly

    # ------------------------------------------------------------------------------------
    def _allreduce(self):
        if self.world > 1:
            allreduce_mean_(self.flat_g, self.bucket, self.pg, self.world)

    def _fwd_bwd(self, L, Hh, *cond):
        """cond: the network's extra forward inputs (USRNet: k, sf, sigma; model_plain4.py:22-23)."""
        eng = self.engine
        drop = None
        if any(b.dp > 0 for b in eng.blocks) and self.net.training:
            from .swinir_engine import drop_path_scales
            drop = drop_path_scales(eng, L.shape[0], L.device)
        eng._packed_version = None           # weights change every step: always repack
        if cond:
            eng.forward(L, *cond)
        else:
            eng.forward(L, drop)
        return eng.backward_from_loss(Hh, self.grads, self.loss_weight, charb_eps=self.charb_eps)

    def _update(self, loss=None):
        skip = None
        if self.range_guard:
            # (world > 1: gradients and parameters only -- identical on every rank after the all-reduce -- so every
            # rank drops and re-runs the same steps; a rank's own loss would not be)
            H.range_check(self.flat_g, self.flat_p, loss if self.world == 1 else None, self.p_limit, self.rflag)
            skip = self.rflag
        H.adam_ema(self.flat_p, self.flat_g, self.m, self.v, self.flat_e, self.flat_p.numel(), self.scal,
                   self.betas[0], self.betas[1], self.eps, self.wd, self.E_decay if self.flat_e is not None else 0.0,
                   skip=skip)

    def _body(self, L, Hh, *cond):
        loss = self._fwd_bwd(L, Hh, *cond)
        self._allreduce()
        self._update(loss)
        return loss

    # ---- fp32x3 range guard -----------------------------------------------------------------
    def _post_step(self):
        if self.range_guard:
            self.rflag_host.copy_(self.rflag, non_blocking=True)
            self.rflag_evt.record()
            self._rflag_pending = True

    def check_range(self):
        """Read the range flag of the last step (waits for it) and, if the step was flagged, back the exponents off
        and re-run it on the same batch -- repeatedly, until it is clean or the engine gives up (RuntimeError).
        step() calls this for the previous step; call it once after the last step of a run."""
        while self.range_guard and self._rflag_pending:
            self.rflag_evt.synchronize()
            self._rflag_pending = False
            bits = int(self.rflag_host[0])
            if bits == 0:
                return
            if bits & 4:
                raise RuntimeError(f"fp32x3 range guard: a parameter is not finite at step {self.t}")
            # one GPU: a non-finite loss means the forward overflowed (activation exponent), a finite loss with
            # non-finite gradients the backward (gradient exponent); several ranks see only the all-reduced
            # gradients (the same bits everywhere), so both exponents drop
            fwd = bool(bits & 2) or self.world > 1
            bwd = not (bits & 2) or self.world > 1
            exps = self.engine.x3_backoff(act=fwd, grad=bwd)
            self.range_events.append((self.t, bits, exps))
            # re-run step t (its Adam scalars are still in self.scal, its batch in the static / last inputs)
            if not self.use_graph or self.graph is None:
                self._body(*self._last_args)
            else:
                self._capture()
                self._replay()
            self.engine._packed_version = None
            self._post_step()

    def _set_scalars(self):
        self.t += 1
        b1, b2 = self.betas
        host = torch.tensor([self.lr / (1 - b1 ** self.t), math.sqrt(1 - b2 ** self.t)], dtype=torch.float32)
        self.scal.copy_(host)   # pageable source: the host buffer is consumed before copy_ returns

    def segment_buckets(self):
        segs = getattr(self.engine, "grad_segments", None)
        return segment_buckets(self.params, segs()) if segs is not None else None

    def _capture(self):
        """Record the step: [fwd+bwd] (+ [update] when world > 1 or segmented), or one graph per
        gradient segment when segment_graphs is on."""
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        buckets = self.segment_buckets() if self.segment_graphs else None
        graphs, gu = [], None
        cs = torch.cuda.Stream(priority=self.stream_priority)
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            if self.world == 1 and not buckets:
                g = torch.cuda.CUDAGraph()
                g.capture_begin(pool=pool)
                self.loss_out = self._body(*self.static)
                g.capture_end()
                graphs.append(g)
            else:
                cur = {"g": torch.cuda.CUDAGraph()}
                cur["g"].capture_begin(pool=pool)

                def cut():
                    cur["g"].capture_end()
                    graphs.append(cur["g"])
                    cur["g"] = torch.cuda.CUDAGraph()
                    cur["g"].capture_begin(pool=pool)

                self.engine.seg_hook = cut if buckets else None
                try:
                    self.loss_out = self._fwd_bwd(*self.static)
                finally:
                    self.engine.seg_hook = None
                cur["g"].capture_end()
                graphs.append(cur["g"])
                gu = torch.cuda.CUDAGraph()
                gu.capture_begin(pool=pool)
                if self.world > 1:
                    self.flat_g.mul_(1.0 / self.world)
                self._update(self.loss_out)
                gu.capture_end()
        torch.cuda.current_stream().wait_stream(cs)
        torch.cuda.synchronize()
        if buckets is not None and len(buckets) != len(graphs):
            raise RuntimeError(f"segmented capture: {len(graphs)} graphs for {len(buckets)} gradient buckets")
        self.buckets = buckets
        self.graph = (graphs, gu)

    def _replay(self):
        graphs, gu = self.graph
        if gu is None:
            graphs[0].replay()
            return
        works = []
        for k, g in enumerate(graphs):
            g.replay()
            if self.world > 1 and self.buckets:
                lo, hi = self.buckets[k]
                works.append(dist.all_reduce(self.flat_g[lo:hi], op=dist.ReduceOp.SUM, group=self.pg, async_op=True))
        if self.world > 1 and not self.buckets:
            allreduce_sum_(self.flat_g, self.bucket, self.pg)
        for w in works:
            w.wait()   # the current stream waits for RCCL's stream (no host block)
        gu.replay()

    def step(self, L, Hh, *cond):
        """One training step on the batch (L, Hh) (device tensors); cond: the network's extra forward
        inputs (USRNet: k [B,1,kh,kw], sf int, sigma [B,1,1,1]).  Returns the device loss [1].
        The graph is re-recorded when any input's shape or a non-tensor input (sf) changes.
        fp32x3: first settles the previous step's range flag (check_range), which may re-run that step."""
        self.check_range()
        self._set_scalars()
        if not self.use_graph:
            self._last_args = (L, Hh) + tuple(cond)
            out = self._body(L, Hh, *cond)
            self.engine._packed_version = None
            self._post_step()
            return out
        args = (L, Hh) + tuple(cond)
        key = tuple(a.shape if torch.is_tensor(a) else ("const", a) for a in args)
        if self.static is None or self._static_key != key:
            self.static = tuple(torch.empty_like(a) if torch.is_tensor(a) else a for a in args)
            self._static_key = key
            self.graph = None
            self.warm = 0
        for dst, src in zip(self.static, args):
            if torch.is_tensor(src):
                dst.copy_(src)
        if self.graph is None and self.warm >= 2:
            self._capture()                  # records only; the replay below executes this step
        self._last_args = self.static
        if self.graph is not None:
            self._replay()
            out = self.loss_out
        else:
            self.warm += 1
            out = self._body(*self.static)
        self.engine._packed_version = None   # params were updated in place by the Adam kernel
        self._post_step()
        return out
