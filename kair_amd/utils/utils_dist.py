"""Process-group helpers (mirror of /root/reference/utils/utils_dist.py:13-59).

init_dist('pytorch') reads RANK / LOCAL_RANK / WORLD_SIZE (torchrun), binds the rank to its GPU and
joins the 'nccl' backend, which is RCCL on PyTorch-ROCm (over xGMI inside a node).  The
reference's unused collective helpers (reduce_sum, gather_grad, all_gather, reduce_loss_dict;
utils_dist.py:118-200, never called) are not reproduced.
"""
import os

import torch
import torch.distributed as dist


def init_dist(launcher="pytorch", backend="nccl", **kwargs):
    if launcher != "pytorch":
        raise ValueError(f"launcher {launcher!r}: only 'pytorch' (torchrun) is supported on the MI355X path")
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank % max(1, torch.cuda.device_count())))
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local), **kwargs)
    else:
        dist.init_process_group(backend, **kwargs)


def get_dist_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1
