"""Fused MoE (K9) -> csrc/kernels/moe.hip + the grouped skinny GEMM (gemm_skinny.hip).

Both regimes run entirely on the device with no host synchronisation: top-k routing,
on-device expert alignment (offsets + sorted token list), grouped gate_up GEMM with the
SwiGLU epilogue, grouped down GEMM, weighted combine.  Decode-sized batches (<= 96 rows per
expert on average) use the weight-streaming grouped skinny GEMM (gemm_skinny.hip); prefill-
sized batches use the MFMA grouped GEMM (moe_gemm.hip), whose grid is an upper bound that
each workgroup maps to (expert, M tile) from the device-side offsets (graph-capturable).  Past
128 rows per expert hipBLASLt's tiles are faster (Mixtral-8x7B, profiles/moe_bench_r2.log:
512 / 2048 / 8192 tokens = 0.98 / 1.89 / 5.19 ms against 1.08 / 2.42 / 8.13 ms for the
grouped MFMA kernel), so that regime reads the E+1 offsets back once per layer and runs one
GEMM pair per expert on contiguous slices of the sorted rows (the old path synchronised once
per expert through nonzero() and scattered with fp32 index_add: 1.43 ms at 65 tokens,
profiles/moe_bench_r2.log first run).

Expert parallelism (``--enable-expert-parallel``, core/helm-charts/vllm/gaudi3-values.yaml:492):
rank r owns experts [e_lo, e_hi); tokens routed elsewhere contribute zero locally
and the caller's all-reduce sums the ranks' partial outputs.
"""

from __future__ import annotations

import os

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import reference as ref
from ._dispatch import check, lib, ptr, stream, use_hip

SCORING = {"softmax": 0, "sigmoid": 1}


# grouped skinny GEMM configurations (csrc/kernels/gemm_skinny.hip cfg bits: NT-1 | (WAVES/2-1)<<1);
# -1 = the shape rule in moe_cfgs.  Overrides for tuning runs.  (3-stage weight pipelines were
# measured neutral at Mixtral decode and are not built for the grouped kernel:
# profiles/moe_s3_ab_r4.log.)
UP_CFG = int(os.environ.get("EIA_MOE_UP_CFG", "-1"))
DOWN_CFG = int(os.environ.get("EIA_MOE_DOWN_CFG", "-1"))


def moe_cfgs(I: int, H: int, up: int = -1, down: int = -1) -> Tuple[int, int]:
    """(gate_up cfg, down cfg) of the grouped expert GEMMs: 4-wave workgroups where the shape
    divides (two 16-row tiles per wave for the SwiGLU pairs), else 2-wave; overrides kept to
    the four grouped forms (cfg 0-3)."""
    u = up & 3 if up >= 0 else (3 if I % 64 == 0 else 1)
    d = down & 3 if down >= 0 else (2 if H % 128 == 0 else 0)
    return u, d
# K split of the decode-sized down projection (K = I): fp32 slabs summed by the combine.
# Mixtral-8x7B at 65 users: TPOT 20.33 -> 19.52 ms at 2 (19.60 at 4), engine 2991 -> 3105 tok/s
# (profiles/moe_down_sk_r4.log): more workgroups keep more weight bytes in flight.  With the
# staggered K walk on, 4 edges out 2: TPOT 19.26 vs 19.32 ms in two pairs (moe_sk_ab2_r4.log).
DOWN_SK = int(os.environ.get("EIA_MOE_DOWN_SK", "4"))

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


def route(x: torch.Tensor, router_w: torch.Tensor, k: int, renormalize: bool = True,
          scoring: str = "softmax") -> Tuple[torch.Tensor, torch.Tensor]:
    """Router GEMM + top-k.  On the GPU one kernel computes the E logits per token (bf16
    rounded, like the Linear it replaces) and selects (moe.hip route_kernel)."""
    T, H = x.shape
    E = router_w.shape[0]
    if (use_hip(x) and x.dtype == torch.bfloat16 and router_w.dtype == torch.bfloat16
            and E <= 64 and H % 8 == 0 and x.stride(1) == 1 and x.stride(0) % 8 == 0
            and router_w.is_contiguous()):
        w = torch.empty(T, k, dtype=torch.float32, device=x.device)
        ids = torch.empty(T, k, dtype=torch.int32, device=x.device)
        check(lib().eia_moe_route(ptr(x), x.stride(0), ptr(router_w), H, T, E, k,
                                  1 if renormalize else 0, SCORING[scoring], ptr(w), ptr(ids),
                                  stream(x)), "moe_route")
        return w, ids
    return topk_route(F.linear(x, router_w), k, renormalize, scoring)


def _grouped_ok(x, w13, w2) -> bool:
    return (x.dtype == torch.bfloat16 and x.shape[1] % 256 == 0 and w2.shape[2] % 256 == 0
            and (w13.shape[1] // 2) % 32 == 0 and w2.shape[1] % 64 == 0)


# Decode-step fusions of the norms around the MoE block (moe.hip splitk_norm_route_kernel,
# moe_combine_norm_kernel): the O projection's split-K add + RMSNorm also computes the router
# logits and top-k, and the experts' combine is left to the next add + RMSNorm.
FUSED_NORMS = os.environ.get("EIA_MOE_FUSED_NORMS", "1") != "0"


class MoECombine:
    """A decode MoE block's output left as the down projection's fp32 split-K slabs plus the
    routing: the consumer's add + RMSNorm combines them (``combine_add_rmsnorm``, one launch
    instead of combine + norm); anything else calls ``materialize``."""

    __slots__ = ("part", "sk", "rows", "topk_w", "inv", "T", "k", "H")

    def __init__(self, part, sk, rows, topk_w, inv, T, k, H):
        self.part, self.sk, self.rows = part, sk, rows
        self.topk_w, self.inv, self.T, self.k, self.H = topk_w, inv, T, k, H

    @property
    def shape(self):
        return (self.T, self.H)

    def materialize(self) -> torch.Tensor:
        out = torch.empty(self.T, self.H, dtype=torch.bfloat16, device=self.part.device)
        check(lib().eia_moe_combine_sk(ptr(self.part), self.sk, self.rows, ptr(self.topk_w),
                                       ptr(self.inv), self.T, self.k, self.H, ptr(out),
                                       out.stride(0), stream(out)), "moe_combine_sk")
        return out


def combine_add_rmsnorm(c: MoECombine, residual: torch.Tensor, weight: torch.Tensor,
                        eps: float):
    """residual += combine(c); returns (rmsnorm(residual) * weight, residual)."""
    out = torch.empty(c.T, c.H, dtype=torch.bfloat16, device=residual.device)
    check(lib().eia_moe_combine_norm(ptr(c.part), c.sk, c.rows, ptr(c.topk_w), ptr(c.inv), c.T,
                                     c.k, c.H, ptr(residual), ptr(weight), float(eps), ptr(out),
                                     out.stride(0), stream(out)), "moe_combine_norm")
    return out, residual


def splitk_norm_route_ok(s, residual, router_w: torch.Tensor, k: int) -> bool:
    from .gemm import SplitK
    return (FUSED_NORMS and isinstance(s, SplitK) and s.bias is None and s.part.is_cuda
            and residual is not None and residual.is_contiguous()
            and residual.dtype == torch.bfloat16 and router_w.dtype == torch.bfloat16
            and router_w.is_contiguous() and router_w.shape[0] <= 16 and k <= router_w.shape[0]
            and s.N % 4 == 0 and s.N <= 8192 and router_w.shape[1] == s.N)


def splitk_norm_route(s, residual: torch.Tensor, weight: torch.Tensor, eps: float,
                      router_w: torch.Tensor, k: int, renormalize: bool = True,
                      scoring: str = "softmax", row_len: Optional[torch.Tensor] = None):
    """residual += reduce(s); x = rmsnorm(residual) * weight; route(x) -- one launch.
    ``row_len`` (int32 [T], nullable): rows whose entry is 0 -- a decode graph's batch-bucket
    padding -- route to no expert (id = E, weight 0).
    Returns (x, residual, (topk weights fp32 [T, k], expert ids int32 [T, k]))."""
    if row_len is not None:
        assert row_len.dtype == torch.int32 and row_len.is_cuda and row_len.numel() >= s.M
    out = torch.empty(s.M, s.N, dtype=torch.bfloat16, device=residual.device)
    w = torch.empty(s.M, k, dtype=torch.float32, device=residual.device)
    ids = torch.empty(s.M, k, dtype=torch.int32, device=residual.device)
    check(lib().eia_moe_splitk_norm_route(ptr(s.part), s.sk, s.M, s.N, ptr(residual),
                                          ptr(weight), float(eps), ptr(out), out.stride(0),
                                          ptr(router_w), router_w.shape[0], k,
                                          1 if renormalize else 0, SCORING[scoring], ptr(w),
                                          ptr(ids), ptr(row_len), stream(out)),
          "moe_splitk_norm_route")
    return out, residual, (w, ids)


def fused_moe(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
              topk_ids: torch.Tensor, expert_range: Optional[Tuple[int, int]] = None,
              act: str = "silu", defer_combine: bool = False, capturable: bool = False):
    """x [T, H]; w13 [E_local, 2I, H] ([gate; up] rows); w2 [E_local, H, I] -> [T, H].
    ``defer_combine``: the decode path may return a ``MoECombine`` for the next add + norm.
    ``capturable`` (implied while a HIP graph is being captured): only the device-side grouped
    forms, whatever the rows per expert -- the sorted-row and per-expert regimes read expert
    offsets back to the host, which a graph cannot contain."""
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
    capturable = capturable or torch.cuda.is_current_stream_capturing()
    if act == "silu" and avg <= 96 and _grouped_ok(x, w13, w2):
        return _fused_moe_grouped(x, w13, w2, topk_w, topk_ids, e_lo, e_hi,
                                  defer_combine=defer_combine)
    if act == "silu" and _mfma_ok(x, w13, w2) and (avg <= MFMA_MAX_ROWS or capturable):
        return _fused_moe_grouped(x, w13, w2, topk_w, topk_ids, e_lo, e_hi, mfma=True)
    if capturable:
        if act == "silu" and _grouped_ok(x, w13, w2):
            return _fused_moe_grouped(x, w13, w2, topk_w, topk_ids, e_lo, e_hi)
        raise RuntimeError(
            f"fused_moe: no host-sync-free form for act={act} H={H} I={w13.shape[1] // 2} "
            "(grouped kernels need SiLU, H % 128 == 0, I % 64 == 0); run this MoE eagerly")
    if _grouped_ok(x, w13, w2):
        return _fused_moe_sorted_blas(x, w13, w2, topk_w, topk_ids, e_lo, e_hi, act)
    return _fused_moe_per_expert(x, w13, w2, topk_w, topk_ids, e_lo, act)


MFMA_MAX_ROWS = 128      # rows per expert above which the per-expert hipBLASLt GEMMs win


def _mfma_ok(x, w13, w2) -> bool:
    H, I = x.shape[1], w13.shape[1] // 2
    return (x.dtype == torch.bfloat16 and H % 128 == 0 and I % 64 == 0
            and w13.is_contiguous() and w2.is_contiguous() and x.stride(1) == 1)


def _fused_moe_grouped(x, w13, w2, topk_w, topk_ids, e_lo, e_hi, mfma: bool = False,
                       defer_combine: bool = False):
    T, H = x.shape
    El, I2, _ = w13.shape
    I = I2 // 2
    k = topk_ids.shape[1]
    n = T * k
    dev = x.device
    st = stream(x)
    offs, row_idx, inv = _align(topk_ids, El, e_lo, e_hi, n, dev, st)
    h1 = torch.empty(max(1, n), I, dtype=x.dtype, device=dev)
    h2 = torch.empty(max(1, n), H, dtype=x.dtype, device=dev)
    if mfma:
        check(lib().eia_moe_grouped_gemm(ptr(x), x.stride(0), ptr(row_idx), ptr(w13), I2, H, El,
                                         ptr(offs), n, 1, ptr(h1), h1.stride(0), st),
              "moe_grouped_gemm_gate_up")
        check(lib().eia_moe_grouped_gemm(ptr(h1), h1.stride(0), None, ptr(w2), H, I, El,
                                         ptr(offs), n, 0, ptr(h2), h2.stride(0), st),
              "moe_grouped_gemm_down")
    else:
        mt = max(1, min(8, -(-int(1.5 * n / El + 1) // 16)))
        up_cfg, down_cfg = moe_cfgs(I, H, UP_CFG, DOWN_CFG)
        w_up = w13
        packed = getattr(w13, "_eia_wg", None)
        if packed and up_cfg in (1, 3) and (2 if up_cfg == 1 else 4, True) in packed:
            # workgroup-packed expert gate_up (ops/gemm.py attach_wg_packed): one sequential
            # weight stream per workgroup
            w_up = packed[(2 if up_cfg == 1 else 4, True)]
            up_cfg |= 1024
        check(lib().eia_moe_gemm(ptr(x), x.stride(0), ptr(w_up), w13.stride(1), None, ptr(h1),
                                 h1.stride(0), I2, H, El, ptr(offs), ptr(row_idx), mt, 2,
                                 up_cfg, st), "moe_gemm_gate_up")
        w_down = w2
        if packed_down := getattr(w2, "_eia_wg", None):
            wp = packed_down.get((4 if down_cfg == 2 else 2, False, 1)) if down_cfg in (0, 2) \
                else None
            if wp is not None:       # workgroup-packed expert down (one tile per wave)
                w_down = wp
                down_cfg |= 1024
        if DOWN_SK > 1 and I % (DOWN_SK * 256) == 0:
            part = torch.empty(DOWN_SK, max(1, n), H, dtype=torch.float32, device=dev)
            check(lib().eia_moe_gemm_sk(ptr(h1), h1.stride(0), ptr(w_down), w2.stride(1),
                                        ptr(part), max(1, n), H, I, El, ptr(offs), None, mt,
                                        DOWN_SK, down_cfg, st), "moe_gemm_down_sk")
            if (defer_combine and FUSED_NORMS and k <= 2 and H % 4 == 0 and H <= 8192
                    and DOWN_SK in (1, 2, 4) and x.dtype == torch.bfloat16):
                return MoECombine(part, DOWN_SK, max(1, n), topk_w, inv, T, k, H)
            out = torch.empty(T, H, dtype=x.dtype, device=dev)
            check(lib().eia_moe_combine_sk(ptr(part), DOWN_SK, max(1, n), ptr(topk_w), ptr(inv),
                                           T, k, H, ptr(out), out.stride(0), st), "moe_combine_sk")
            return out
        check(lib().eia_moe_gemm(ptr(h1), h1.stride(0), ptr(w_down), w2.stride(1), None, ptr(h2),
                                 h2.stride(0), H, I, El, ptr(offs), None, mt, 0,
                                 down_cfg, st), "moe_gemm_down")
    out = torch.empty(T, H, dtype=x.dtype, device=dev)
    check(lib().eia_moe_combine(ptr(h2), h2.stride(0), ptr(topk_w), ptr(inv), T, k, H, ptr(out),
                                out.stride(0), st), "moe_combine")
    return out


def _align(topk_ids, El, e_lo, e_hi, n, dev, st):
    E_total = max(e_hi, int(El + e_lo))
    offs = torch.empty(El + 1, dtype=torch.int32, device=dev)
    # with expert parallelism the align kernel scatters only the local rows and zeroes the rest
    row_idx = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    inv = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    check(lib().eia_moe_align(ptr(topk_ids), n, E_total, e_lo, e_hi, ptr(offs), ptr(row_idx),
                              ptr(inv), topk_ids.shape[1], st), "moe_align")
    return offs, row_idx, inv


def _fused_moe_sorted_blas(x, w13, w2, topk_w, topk_ids, e_lo, e_hi, act):
    """Long-prompt regime: device-side alignment, ONE read-back of the expert offsets, one
    hipBLASLt GEMM pair per expert on contiguous slices of the gathered rows, HIP combine."""
    from . import activation

    T, H = x.shape
    El = w13.shape[0]
    k = topk_ids.shape[1]
    n = T * k
    dev = x.device
    st = stream(x)
    offs, row_idx, inv = _align(topk_ids, El, e_lo, e_hi, n, dev, st)
    bounds = offs.tolist()                     # the one host synchronisation of this layer
    # expert parallelism: only the first bounds[El] sorted rows belong to local experts (the
    # rest of row_idx is never written by the align kernel)
    xs = x.index_select(0, row_idx[:bounds[El]].long())
    h2 = torch.empty(max(1, n), H, dtype=x.dtype, device=dev)
    for e in range(El):
        a, b = bounds[e], bounds[e + 1]
        if a == b:
            continue
        h = activation.act_and_mul(F.linear(xs[a:b], w13[e]), act)
        torch.matmul(h, w2[e].t(), out=h2[a:b])
    out = torch.empty(T, H, dtype=x.dtype, device=dev)
    check(lib().eia_moe_combine(ptr(h2), h2.stride(0), ptr(topk_w), ptr(inv), T, k, H, ptr(out),
                                out.stride(0), st), "moe_combine")
    return out


def _fused_moe_per_expert(x, w13, w2, topk_w, topk_ids, e_lo, act):
    """Fallback for shapes / activations the grouped kernels do not cover (non-SiLU experts,
    H % 128 or I % 64 != 0): per-expert hipBLASLt GEMMs on the gathered rows."""
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
