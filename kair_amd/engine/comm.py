"""Gradient exchange for data-parallel training (replaces the DDP reducer, model_base.py:113-119).

The fused trainer keeps every gradient in ONE flat fp32 buffer laid out in parameter order, so the
exchange is a bucketed all-reduce over contiguous slices of it: RCCL ("nccl" backend) over xGMI on
the MI355X node, gloo on CPU for the tests.  Buckets are issued from the END of the buffer (the
last layers' grads are final first in backward, as the DDP reducer orders them) and the mean is
taken with one scale of the whole buffer afterwards.
"""
import torch
import torch.distributed as dist


def bucket_bounds(numel, bucket_elems):
    """[(lo, hi)] slices of a flat buffer of `numel`, <= bucket_elems each, last slice first."""
    if bucket_elems <= 0:
        raise ValueError("bucket_elems must be positive")
    out = []
    hi = numel
    while hi > 0:
        lo = max(0, hi - bucket_elems)
        out.append((lo, hi))
        hi = lo
    return out


def allreduce_mean_(flat, bucket_elems, group=None, world=None):
    """In-place mean over ranks of the flat gradient buffer (sum by buckets, then one scale)."""
    world = world or dist.get_world_size(group)
    if world == 1:
        return flat
    for lo, hi in bucket_bounds(flat.numel(), bucket_elems):
        dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, group=group)
    flat.mul_(1.0 / world)
    return flat


def allreduce_sum_(flat, bucket_elems, group=None):
    """In-place sum over ranks, bucketed from the end (the mean scale is applied by the caller)."""
    for lo, hi in bucket_bounds(flat.numel(), bucket_elems):
        dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, group=group)
    return flat


def broadcast_params_(flat, src=0, group=None):
    """Make every rank start from rank `src`'s parameters (DDP's construction-time broadcast)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat, src=src, group=group)
    return flat
