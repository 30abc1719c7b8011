"""torch.distributed helpers used by the scoring path (reference: straggler/dist_utils.py:21-116).

gloo keeps tensors on the CPU; any other backend ("nccl" = RCCL on ROCm) gets tensors on
the current HIP device.  World size 1 (or no process group) turns every collective into a
local no-op, as in the reference.
"""
from typing import Optional

import torch

from ..common.device_utils import get_current_device


def _initialized() -> bool:
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def get_world_size(group=None) -> int:
    return torch.distributed.get_world_size(group) if _initialized() else 1


def get_rank(group=None) -> int:
    return torch.distributed.get_rank(group) if _initialized() else 0


def get_device_for_backend(group=None) -> torch.device:
    if _initialized() and torch.distributed.get_backend(group) != torch.distributed.Backend.GLOO:
        return get_current_device()
    return torch.device("cpu")


def all_gather_object(obj, group=None):
    ws = get_world_size(group)
    objs = [None] * ws
    if ws > 1:
        torch.distributed.all_gather_object(objs, obj, group)
    else:
        objs[0] = obj
    return objs


def all_reduce(tensor, op=torch.distributed.ReduceOp.SUM,
               group: Optional[torch.distributed.ProcessGroup] = None, async_op: bool = False):
    if get_world_size(group) > 1:
        torch.distributed.all_reduce(tensor=tensor, op=op, group=group, async_op=async_op)


def gather_on_rank0(tensor, group: Optional[torch.distributed.ProcessGroup] = None):
    """List of every rank's tensor on rank 0 (on the input's device); None elsewhere."""
    ws = get_world_size(group)
    if ws <= 1:
        return [tensor]
    rank = get_rank(group)
    src_dev = tensor.device
    t = tensor.to(get_device_for_backend(group))
    out = [torch.empty_like(t) for _ in range(ws)] if rank == 0 else None
    torch.distributed.gather(tensor=t, gather_list=out, dst=0, group=group)
    if rank == 0:
        out = [x.to(src_dev) for x in out]
    return out


def is_all_true(flag: bool, group: Optional[torch.distributed.ProcessGroup] = None) -> bool:
    if get_world_size(group) <= 1:
        return flag
    t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float32,
                     device=get_device_for_backend(group))
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN, group=group)
    return bool(t.item() > 0)
