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

Two exchange forms:

* exact (prefill-sized batches): the W-element counts all_to_all is read back to the host
  (split sizes must be known to the collective) and only real rows travel;
* padded (decode batches, graph-capturable; ``moe_all_to_all(..., capacity=C)``): every rank
  sends a fixed [W, C] block of rows, C = the worst case (all of a rank's T_r * k (token,
  slot) pairs routed to one peer), padding rows carry expert id -1 (skipped by the owner's
  align kernel, they come back as zeros).  The layout -- each pair's slot in its peer's
  block -- is computed on the device (one-hot prefix count over the owners), so nothing is
  read back and the whole MoE layer captures into the decode HIP graph.  W x the rows of the
  exact form, which at decode (T <= a few hundred) is a few MB per layer, the size the
  all-reduce form moves anyway; prefill keeps the exact form.
"""

from __future__ import annotations

from typing import Optional, Tuple

import os

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import comm

# token count (global, before the 1/W slicing) up to which the TP engine uses the padded,
# graph-capturable exchange; decode batches are <= max_num_seqs.  EIA_EP_A2A_PADDED_MAX_TOKENS
PADDED_MAX_TOKENS = int(os.environ.get("EIA_EP_A2A_PADDED_MAX_TOKENS", "512"))


def dispatch_layout(topk_ids: torch.Tensor, e_per: int, world: int, capacity: int):
    """Device-side slot of every (token, slot) pair in the padded [world * capacity] send
    buffer: pairs keep their order within each owner's block.  Returns (global expert ids
    [n] int64, destination rows [n] int64)."""
    ids = topk_ids.reshape(-1).long()
    owner = torch.div(ids, e_per, rounding_mode="floor")
    onehot = F.one_hot(owner, world)                       # [n, W]
    pos = (onehot.cumsum(0) * onehot).sum(1) - 1           # rank among same-owner pairs
    return ids, owner * capacity + pos


def _moe_all_to_all_padded(x, topk_w, topk_ids, w13_local, w2_local, e_lo, e_per, group, act,
                           W: int, capacity: int) -> torch.Tensor:
    from ..ops import moe as moe_ops

    T, H = x.shape
    k = topk_ids.shape[1]
    n = T * k
    if n > capacity:
        raise ValueError(f"{T} tokens x top-{k} exceed the padded all-to-all capacity "
                         f"{capacity}")
    ids, dest = dispatch_layout(topk_ids, e_per, W, capacity)
    tok = torch.div(torch.arange(n, device=x.device), k, rounding_mode="floor")
    send_x = x.new_zeros((W * capacity, H))
    send_x.index_copy_(0, dest, x.index_select(0, tok))
    send_e = torch.full((W * capacity,), -1, dtype=torch.int32, device=x.device)
    send_e.index_copy_(0, dest, ids.to(torch.int32))
    recv_x = torch.empty_like(send_x)
    recv_e = torch.empty_like(send_e)
    comm.all_to_all_single(recv_x, send_x, group=group)
    comm.all_to_all_single(recv_e, send_e, group=group)
    ones = torch.ones(W * capacity, 1, dtype=torch.float32, device=x.device)
    # W * capacity rows over e_per experts can exceed the MFMA regime's rows per expert
    # (Mixtral TP8: e_per 1) -- the padded form must stay on the device-side kernels
    y = moe_ops.fused_moe(recv_x, w13_local, w2_local, ones, recv_e[:, None],
                          (e_lo, e_lo + e_per), act, capturable=True)
    back = torch.empty_like(send_x)
    comm.all_to_all_single(back, y.contiguous(), group=group)
    pairs = back.index_select(0, dest).float() * topk_w.reshape(-1, 1).float()
    return pairs.view(T, k, H).sum(1).to(x.dtype)


def _exchange_counts(send_counts: torch.Tensor, group) -> torch.Tensor:
    recv = torch.empty_like(send_counts)
    comm.all_to_all_single(recv, send_counts, group=group)
    return recv


def moe_all_to_all(x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor,
                   w13_local: torch.Tensor, w2_local: torch.Tensor, e_lo: int, e_per: int,
                   group=None, act: str = "silu",
                   world: Optional[int] = None, capacity: Optional[int] = None) -> torch.Tensor:
    """Token-sharded MoE layer.  x [T_r, H] are THIS rank's tokens, topk_ids GLOBAL expert
    ids; this rank owns experts [e_lo, e_lo + e_per) (w13_local [e_per, 2I, H], w2_local
    [e_per, H, I]); expert e lives on rank e // e_per.  Returns [T_r, H].  ``capacity``
    (the same on every rank, >= T_r * k) selects the padded, host-sync-free exchange."""
    from ..ops import moe as moe_ops

    group = group if group is not None else dist.group.WORLD
    W = world or dist.get_world_size(group)
    if capacity is not None:
        return _moe_all_to_all_padded(x, topk_w, topk_ids, w13_local, w2_local, e_lo, e_per,
                                      group, act, W, capacity)
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
    output is complete on every rank (no trailing all-reduce).  Batches up to
    PADDED_MAX_TOKENS (every decode step) take the padded exchange with capacity
    ceil(T / W) * k, known to every rank from T alone: no host synchronisation, so the decode
    graph captures the layer."""
    group = group if group is not None else dist.group.WORLD
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    T, H = x.shape
    lo, hi = token_slice(T, r, W)
    per = -(-T // W)
    cap = per * topk_ids.shape[1] if T <= PADDED_MAX_TOKENS else None
    part = moe_all_to_all(x[lo:hi], topk_w[lo:hi], topk_ids[lo:hi], w13_local, w2_local,
                          e_lo, e_per, group, act, W, capacity=cap)
    mine = x.new_zeros((per, H))
    mine[:hi - lo] = part
    buf = comm.all_gather(mine, 0, group=group)          # [per * W, H]
    return buf[:T]
