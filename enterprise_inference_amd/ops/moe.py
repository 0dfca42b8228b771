"""Fused MoE (K9) -> csrc/kernels/moe.hip + the grouped skinny GEMM (gemm_skinny.hip).

Decode-sized batches (tokens per expert <= 128 on average) run entirely in HIP:
top-k routing, on-device expert alignment, grouped gate_up GEMM with the SwiGLU
epilogue, grouped down GEMM, weighted combine.  Prefill-sized batches run one
hipBLASLt GEMM pair per expert on the gathered rows (MFMA-bound there).

Expert parallelism (``--enable-expert-parallel``, core/helm-charts/vllm/gaudi3-values.yaml:492):
rank r owns experts [e_lo, e_hi); tokens routed elsewhere contribute zero locally
and the caller's all-reduce sums the ranks' partial outputs.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import reference as ref
from ._dispatch import check, lib, ptr, stream, use_hip

SCORING = {"softmax": 0, "sigmoid": 1}


def topk_route(logits: torch.Tensor, k: int, renormalize: bool = True,
               scoring: str = "softmax") -> Tuple[torch.Tensor, torch.Tensor]:
    """Router logits [T, E] -> (weights fp32 [T, k], expert ids int32 [T, k])."""
    T, E = logits.shape
    if not use_hip(logits):
        if scoring == "sigmoid":
            v, ids = torch.topk(logits.float(), k, dim=-1)
            return torch.sigmoid(v), ids.to(torch.int32)
        return ref.topk_softmax(logits, k, renormalize)
    lg = logits.contiguous()
    w = torch.empty(T, k, dtype=torch.float32, device=logits.device)
    ids = torch.empty(T, k, dtype=torch.int32, device=logits.device)
    check(lib().eia_moe_topk(ptr(lg), 1 if lg.dtype == torch.bfloat16 else 0, T, E, k,
                             1 if renormalize else 0, SCORING[scoring], ptr(w), ptr(ids),
                             stream(lg)), "moe_topk")
    return w, ids


def _grouped_ok(x, w13, w2) -> bool:
    return (x.dtype == torch.bfloat16 and x.shape[1] % 256 == 0 and w2.shape[2] % 256 == 0
            and (w13.shape[1] // 2) % 32 == 0 and w2.shape[1] % 64 == 0)


def fused_moe(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
              topk_ids: torch.Tensor, expert_range: Optional[Tuple[int, int]] = None,
              act: str = "silu") -> torch.Tensor:
    """x [T, H]; w13 [E_local, 2I, H] ([gate; up] rows); w2 [E_local, H, I] -> [T, H]."""
    T, H = x.shape
    El = w13.shape[0]
    e_lo, e_hi = expert_range or (0, El)
    k = topk_ids.shape[1]
    if not use_hip(x):
        ids = topk_ids.long() - e_lo
        keep = (ids >= 0) & (ids < El)
        tw = torch.where(keep, topk_w, torch.zeros_like(topk_w))
        return ref.fused_moe(x, w13, w2, tw, ids.clamp(0, El - 1).to(torch.int32), act)
    avg = T * k / max(1, El)
    if act == "silu" and avg <= 96 and _grouped_ok(x, w13, w2):
        return _fused_moe_grouped(x, w13, w2, topk_w, topk_ids, e_lo, e_hi)
    return _fused_moe_per_expert(x, w13, w2, topk_w, topk_ids, e_lo, act)


def _fused_moe_grouped(x, w13, w2, topk_w, topk_ids, e_lo, e_hi):
    T, H = x.shape
    El, I2, _ = w13.shape
    I = I2 // 2
    k = topk_ids.shape[1]
    n = T * k
    dev = x.device
    E_total = max(e_hi, int(El + e_lo))
    offs = torch.empty(El + 1, dtype=torch.int32, device=dev)
    row_idx = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    inv = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    st = stream(x)
    check(lib().eia_moe_align(ptr(topk_ids), n, E_total, e_lo, e_hi, ptr(offs), ptr(row_idx),
                              ptr(inv), k, st), "moe_align")
    mt = max(1, min(8, -(-int(1.5 * n / El + 1) // 16)))
    h1 = torch.empty(max(1, n), I, dtype=x.dtype, device=dev)
    check(lib().eia_moe_gemm(ptr(x), x.stride(0), ptr(w13), w13.stride(1), None, ptr(h1),
                             h1.stride(0), I2, H, El, ptr(offs), ptr(row_idx), mt, 2,
                             3 if (I % 64 == 0) else 1, st), "moe_gemm_gate_up")
    h2 = torch.empty(max(1, n), H, dtype=x.dtype, device=dev)
    check(lib().eia_moe_gemm(ptr(h1), h1.stride(0), ptr(w2), w2.stride(1), None, ptr(h2),
                             h2.stride(0), H, I, El, ptr(offs), None, mt, 0,
                             2 if H % 128 == 0 else 0, st), "moe_gemm_down")
    out = torch.empty(T, H, dtype=x.dtype, device=dev)
    check(lib().eia_moe_combine(ptr(h2), h2.stride(0), ptr(topk_w), ptr(inv), T, k, H, ptr(out),
                                out.stride(0), st), "moe_combine")
    return out


def _fused_moe_per_expert(x, w13, w2, topk_w, topk_ids, e_lo, act):
    """Prefill path: gather each expert's rows, two hipBLASLt GEMMs, weighted scatter-add."""
    from . import activation

    T, H = x.shape
    El = w13.shape[0]
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    ids = topk_ids.long() - e_lo
    for e in range(El):
        tok, slot = (ids == e).nonzero(as_tuple=True)
        if tok.numel() == 0:
            continue
        h = activation.act_and_mul(F.linear(x.index_select(0, tok), w13[e]), act)
        y = F.linear(h, w2[e])
        out.index_add_(0, tok, y.float() * topk_w[tok, slot, None])
    return out.to(x.dtype)
