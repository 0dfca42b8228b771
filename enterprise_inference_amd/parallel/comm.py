"""Tensor-parallel collectives.

all_reduce picks, per call:
  * the custom xGMI one-shot / two-shot kernel (parallel/custom_allreduce.py)
    for decode-sized messages, when it is registered for this group, else
  * RCCL ``all_reduce`` (ring/tree over xGMI) for large prefill buffers.
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from . import state

_CUSTOM_AR = None   # set by custom_allreduce.init_custom_allreduce()


def set_custom_allreduce(ar) -> None:
    global _CUSTOM_AR
    _CUSTOM_AR = ar


def get_custom_allreduce():
    return _CUSTOM_AR


def all_reduce(x: torch.Tensor) -> torch.Tensor:
    if state.tp_size() == 1:
        return x
    ar = _CUSTOM_AR
    if ar is not None and ar.should_use(x):
        return ar.all_reduce(x)
    dist.all_reduce(x, group=state.tp_group())
    return x


def all_reduce_async(x: torch.Tensor):
    """RCCL all-reduce on the collective's own stream; returns the Work (wait() orders the
    caller's stream after it) or None at TP=1."""
    if state.tp_size() == 1:
        return None
    return dist.all_reduce(x, group=state.tp_group(), async_op=True)


def all_reduce_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor,
                           eps: float):
    """(rmsnorm(residual + allreduce(x)) * w, residual) with residual updated in place.

    Decode-sized messages run the fused xGMI kernel (one launch, no HBM round trip of the
    reduced tensor); otherwise RCCL all-reduce followed by the fused add+RMSNorm kernel."""
    from ..ops import norm
    ar = _CUSTOM_AR
    if state.tp_size() > 1 and ar is not None and ar.can_fuse_norm(x) and \
            residual.is_contiguous() and residual.dtype == x.dtype:
        return ar.add_rmsnorm(x, residual, weight, eps), residual
    return norm.fused_add_rms_norm(all_reduce(x), residual, weight, eps)


def all_gather(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    ws = state.tp_size()
    if ws == 1:
        return x
    dim = dim % x.dim()
    flat = torch.empty(ws * x.numel(), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(flat, x.contiguous().view(-1), group=state.tp_group())
    out = flat.view((ws,) + tuple(x.shape)).movedim(0, dim)
    shape = list(x.shape)
    shape[dim] *= ws
    return out.reshape(shape)


def gather_to_driver(x: torch.Tensor, dim: int = -1) -> Optional[torch.Tensor]:
    """Vocab-parallel logits -> full logits (all ranks receive; C4)."""
    return all_gather(x, dim)


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None):
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=state.tp_group())
    return out


def broadcast_object(obj, src: int = 0):
    if state.tp_size() == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=state.tp_ranks()[src], group=state.tp_cpu_group())
    return lst[0]


def barrier() -> None:
    if dist.is_initialized():
        dist.barrier()
