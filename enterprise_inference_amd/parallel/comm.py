"""Tensor-parallel collectives.

all_reduce picks, per call:
  * the custom xGMI one-shot / two-shot kernel (parallel/custom_allreduce.py)
    for decode-sized messages, when it is registered for this group, else
  * RCCL ``all_reduce`` (ring/tree over xGMI) for large prefill buffers.

With a gloo group (the CPU path, or the one-GPU TP rehearsal ``EIA_TP_SHARE_DEVICE`` where
every rank shares cuda:0 and RCCL cannot run) device tensors are staged through host memory:
the same collective sequence, numerically identical sums, no HIP-graph capture.
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


def _staged(x: torch.Tensor) -> bool:
    return x.is_cuda and state.host_staged()


def all_reduce(x: torch.Tensor, group=None) -> torch.Tensor:
    if state.tp_size() == 1 and group is None:
        return x
    group = group if group is not None else state.tp_group()
    if _staged(x):
        h = x.detach().cpu()
        dist.all_reduce(h, group=group)
        x.copy_(h)
        return x
    ar = _CUSTOM_AR
    if ar is not None and ar.should_use(x):
        return ar.all_reduce(x)
    dist.all_reduce(x, group=group)
    return x


def all_reduce_async(x: torch.Tensor):
    """RCCL all-reduce on the collective's own stream; returns the Work (wait() orders the
    caller's stream after it) or None when the reduction already completed (TP=1, gloo)."""
    if state.tp_size() == 1:
        return None
    if _staged(x):
        all_reduce(x)
        return None
    return dist.all_reduce(x, group=state.tp_group(), async_op=True)


def all_reduce_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor,
                           eps: float):
    """(rmsnorm(residual + allreduce(x)) * w, residual) with residual updated in place.

    Decode-sized messages run the fused xGMI kernel (one launch, no HBM round trip of the
    reduced tensor); otherwise RCCL all-reduce followed by the fused add+RMSNorm kernel.
    ``x`` may be the row-parallel GEMM's split-K slabs (``gemm.SplitK``): the fused kernel sums
    them while staging, so the GEMM's own reduce launch disappears."""
    from ..ops import norm
    ar = _CUSTOM_AR
    if state.tp_size() > 1 and ar is not None and ar.can_fuse_norm(x) and \
            residual.is_contiguous() and residual.dtype == torch.bfloat16:
        return ar.add_rmsnorm(x, residual, weight, eps), residual
    if hasattr(x, "materialize"):          # split-K slabs the custom kernel cannot take
        x = x.materialize()
    return norm.fused_add_rms_norm(all_reduce(x), residual, weight, eps)


def _gather_flat(x: torch.Tensor, ws: int, group) -> torch.Tensor:
    """[ws * numel] of every rank's x in rank order."""
    if _staged(x) or (not x.is_cuda and dist.get_backend(group) == "gloo"):
        parts = [torch.empty(x.numel(), dtype=x.dtype) for _ in range(ws)]
        dist.all_gather(parts, x.detach().contiguous().view(-1).cpu(), group=group)
        return torch.cat(parts).to(x.device)
    flat = torch.empty(ws * x.numel(), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(flat, x.contiguous().view(-1), group=group)
    return flat


def all_gather(x: torch.Tensor, dim: int = -1, group=None) -> torch.Tensor:
    ws = state.tp_size() if group is None else dist.get_world_size(group)
    if ws == 1:
        return x
    group = group if group is not None else state.tp_group()
    dim = dim % x.dim()
    flat = _gather_flat(x, ws, group)
    out = flat.view((ws,) + tuple(x.shape)).movedim(0, dim)
    shape = list(x.shape)
    shape[dim] *= ws
    return out.reshape(shape)


def gather_to_driver(x: torch.Tensor, dim: int = -1) -> Optional[torch.Tensor]:
    """Vocab-parallel logits -> full logits (all ranks receive; C4)."""
    return all_gather(x, dim)


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None,
                      group=None):
    group = group if group is not None else state.tp_group()
    if _staged(inp):
        h_out = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h_out, inp.detach().contiguous().cpu(), out_splits, in_splits,
                               group=group)
        out.copy_(h_out)
        return out
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
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
