"""Per-shape HBM buffer sets ("plans") of the step programs, and who may use them when.

A step program (swinir_engine, dncnn/rrdbnet/usrnet engines) runs over preallocated buffers keyed by
the input shape.  Three kinds of users exist:

* the fused trainer (FusedTrainer) runs forward + backward back to back and captures them in a HIP
  graph: it always gets the ``primary`` plan of its shape, so the captured pointers stay valid; no
  lease ever hands that plan out (a graph replay would overwrite a leased node's activations);
* an autograd node (SwinIRFunction / ConvNetFunction / USRNetFunction) keeps the forward's saved
  activations until its backward: it ``lease``s a training plan, and a second forward of the same
  shape before that backward gets another plan instead of overwriting the first one's activations
  (gradient accumulation, two losses on two forwards).  The lease ends at backward, or when the
  autograd graph is freed without one;
* no-grad forwards (eval, ModelPlain.test on full images of many sizes) use ``infer`` plans, built
  by the engine without backward buffers and kept in a small LRU so memory stays bounded.
"""
from collections import OrderedDict


class Lease:
    """Holds a training plan for one autograd node; released explicitly or when garbage collected."""

    def __init__(self, plan):
        self.plan = plan
        plan["_lease"] = self

    def release(self):
        if self.plan is not None and self.plan.get("_lease") is self:
            self.plan["_lease"] = None
        self.plan = None

    def __del__(self):
        self.release()


class PlanPool:
    def __init__(self, build, max_infer=2):
        self.build = build            # build(key, infer: bool) -> plan dict
        self.primary = {}             # key -> the fused trainer's plan (never leased)
        self.leased = {}              # key -> [plan, ...] for autograd nodes
        self.infer = OrderedDict()    # key -> plan (LRU)
        self.max_infer = max_infer

    def get(self, key, mode="primary"):
        if mode == "infer":
            P = self.infer.pop(key, None)
            if P is None:
                P = self.build(key, True)
            self.infer[key] = P
            while len(self.infer) > self.max_infer:
                self.infer.popitem(last=False)
            return P
        if mode == "primary":
            if key not in self.primary:
                self.primary[key] = self.build(key, False)
            return self.primary[key]
        if mode != "lease":
            raise ValueError(mode)
        slots = self.leased.setdefault(key, [])
        for P in slots:
            if P.get("_lease") is None:
                return P
        P = self.build(key, False)
        slots.append(P)
        return P

    def n_train(self, key):
        return (key in self.primary) + len(self.leased.get(key, []))

    def clear(self):
        self.primary.clear()
        self.leased.clear()
        self.infer.clear()


class plan_mode:
    """Context manager: the engine's next plan() calls use `mode` (see PlanPool.get)."""

    def __init__(self, engine, mode):
        self.engine, self.mode = engine, mode

    def __enter__(self):
        self.prev = getattr(self.engine, "plan_mode", "primary")
        self.engine.plan_mode = self.mode
        return self

    def __exit__(self, *exc):
        self.engine.plan_mode = self.prev
        return False


def autograd_mode(params):
    """'lease' when the forward records an autograd graph (grad enabled and some parameter trains),
    'infer' otherwise."""
    import torch
    if torch.is_grad_enabled() and any(p.requires_grad for p in params):
        return "lease"
    return "infer"
