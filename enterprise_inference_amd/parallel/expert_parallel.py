"""Expert parallelism with all-to-all token dispatch / combine.

Two EP forms exist in this framework:

* ``allreduce`` (default, reference core/helm-charts/vllm/gaudi3-values.yaml:492
  ``--enable-expert-parallel``): attention is tensor-parallel, so every rank already holds
  every token; rank r runs its experts [e_lo, e_hi) on the tokens routed there and the
  layer's (fused) all-reduce sums the ranks' partial outputs.
* ``all_to_all`` (this module): each rank owns a disjoint slice of the tokens (a
  data-parallel attention deployment, or -- inside the TP engine -- a 1/W slice of the
  replicated batch).  The (token, slot) pairs are sorted by owning rank and exchanged with
  ``all_to_all_single`` (RCCL over xGMI on MI355X: every peer is one hop, so the exchange is
  bounded by the per-link rate, not a ring), the owner runs its local experts on the rows it
  received (the same device-side grouped GEMMs as the single-GPU path, weight 1 per row),
  the results travel back by the inverse exchange and each rank applies its routing weights
  locally.  Traffic per rank: 2 * (T/W) * k * H * (W-1)/W rows each way instead of the
  all-reduce's 2 * T * H * (W-1)/W; with the TP engine an all-gather of the W token slices
  restores the replicated activations (``moe_all_to_all_replicated``).

The counts exchange is the one host synchronisation of a dispatch (split sizes must be
known to the collective); it is a W-element all_to_all.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

from . import comm


def _exchange_counts(send_counts: torch.Tensor, group) -> torch.Tensor:
    recv = torch.empty_like(send_counts)
    comm.all_to_all_single(recv, send_counts, group=group)
    return recv


def moe_all_to_all(x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor,
                   w13_local: torch.Tensor, w2_local: torch.Tensor, e_lo: int, e_per: int,
                   group=None, act: str = "silu",
                   world: Optional[int] = None) -> torch.Tensor:
    """Token-sharded MoE layer.  x [T_r, H] are THIS rank's tokens, topk_ids GLOBAL expert
    ids; this rank owns experts [e_lo, e_lo + e_per) (w13_local [e_per, 2I, H], w2_local
    [e_per, H, I]); expert e lives on rank e // e_per.  Returns [T_r, H]."""
    from ..ops import moe as moe_ops

    group = group if group is not None else dist.group.WORLD
    W = world or dist.get_world_size(group)
    T, H = x.shape
    k = topk_ids.shape[1]
    ids = topk_ids.reshape(-1).long()
    owner = torch.div(ids, e_per, rounding_mode="floor")
    order = torch.argsort(owner, stable=True)
    send_counts = torch.bincount(owner, minlength=W).to(torch.int64)
    recv_counts = _exchange_counts(send_counts, group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    tok = torch.div(order, k, rounding_mode="floor")
    send_x = x.index_select(0, tok)
    send_e = ids.index_select(0, order).to(torch.int32)
    R = sum(rc)
    recv_x = x.new_empty((R, H))
    recv_e = torch.empty(R, dtype=torch.int32, device=x.device)
    comm.all_to_all_single(recv_x, send_x, rc, sc, group=group)
    comm.all_to_all_single(recv_e, send_e, rc, sc, group=group)
    if R:
        ones = torch.ones(R, 1, dtype=torch.float32, device=x.device)
        y = moe_ops.fused_moe(recv_x, w13_local, w2_local, ones, recv_e[:, None],
                              (e_lo, e_lo + e_per), act)
    else:
        y = x.new_empty((0, H))
    back = x.new_empty((len(order), H))
    comm.all_to_all_single(back, y.contiguous(), sc, rc, group=group)
    w_sorted = topk_w.reshape(-1).index_select(0, order).float()
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    out.index_add_(0, tok, back.float() * w_sorted[:, None])
    return out.to(x.dtype)


def token_slice(T: int, rank: int, world: int) -> Tuple[int, int]:
    per = -(-T // world)
    lo = min(T, rank * per)
    return lo, min(T, lo + per)


def moe_all_to_all_replicated(x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor,
                              w13_local: torch.Tensor, w2_local: torch.Tensor, e_lo: int,
                              e_per: int, group=None, act: str = "silu") -> torch.Tensor:
    """All-to-all EP inside a tensor-parallel engine (tokens replicated on every rank): rank
    r dispatches its 1/W slice of the tokens, then an all-gather rebuilds [T, H] -- the MoE
    output is complete on every rank (no trailing all-reduce)."""
    group = group if group is not None else dist.group.WORLD
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    T, H = x.shape
    lo, hi = token_slice(T, r, W)
    part = moe_all_to_all(x[lo:hi], topk_w[lo:hi], topk_ids[lo:hi], w13_local, w2_local,
                          e_lo, e_per, group, act, W)
    per = -(-T // W)
    mine = x.new_zeros((per, H))
    mine[:hi - lo] = part
    buf = comm.all_gather(mine, 0, group=group)          # [per * W, H]
    return buf[:T]
