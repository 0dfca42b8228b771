"""Fused RoPE + paged-KV write (K4 + K3) -> csrc/kernels/rope_cache.hip."""

from __future__ import annotations

from typing import Optional

import torch

from . import reference as ref
from ._dispatch import check, lib, ptr, require, stream, use_hip


class RotaryCache:
    """Per-model cos/sin table [max_pos, head_dim] fp32 (cos | sin halves)."""

    def __init__(self, head_dim: int, max_pos: int, theta: float, scaling: Optional[dict],
                 device: torch.device, is_neox: bool = True):
        self.head_dim = head_dim
        self.is_neox = is_neox
        self.cos_sin = ref.rope_cos_sin_cache(max_pos, head_dim, theta, scaling).to(device)


def rope_qkv_cache(qkv, positions: Optional[torch.Tensor],
                   rotary: Optional[RotaryCache], slot_mapping: torch.Tensor,
                   k_cache: torch.Tensor, v_cache: torch.Tensor, num_heads: int,
                   num_kv_heads: int, head_dim: int, bias: Optional[torch.Tensor] = None,
                   q_norm_w: Optional[torch.Tensor] = None, k_norm_w: Optional[torch.Tensor] = None,
                   norm_eps: float = 1e-6) -> torch.Tensor:
    """qkv [T, (Hq+2Hkv)*D] -> q [T, Hq, D]; k/v scattered into the paged cache.

    ``qkv`` may be a ``gemm.SplitK`` (fp32 split-K partials of the QKV projection): the kernel
    then sums the slabs itself (no separate reduce launch)."""
    from .gemm import SplitK
    cos_sin = None if rotary is None else rotary.cos_sin
    part = None
    if isinstance(qkv, SplitK):
        if qkv.bias is not None:
            require(bias is None, "rope_qkv_cache: bias given twice")
        if use_hip(qkv.part, k_cache):
            part = qkv
            bias = qkv.bias if qkv.bias is not None else bias   # added by the kernel
        else:
            qkv = qkv.materialize()                             # includes the bias
    if part is None and not (use_hip(qkv, k_cache) and qkv.dtype == torch.bfloat16):
        return ref.rope_qkv_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache,
                                  num_heads, num_kv_heads, head_dim, bias, q_norm_w, k_norm_w,
                                  norm_eps, rotary is None or rotary.is_neox)
    T = qkv.shape[0]
    if part is None:
        require(qkv.stride(-1) == 1 and qkv.shape[1] == (num_heads + 2 * num_kv_heads) * head_dim,
                "rope_qkv_cache: qkv shape")
    else:
        require(qkv.N == (num_heads + 2 * num_kv_heads) * head_dim and qkv.part.is_contiguous(),
                "rope_qkv_cache: split-K qkv shape")
    require(slot_mapping.dtype == torch.int32 and slot_mapping.numel() >= T, "slot_mapping int32[T]")
    if positions is not None:
        require(positions.dtype == torch.int32, "positions must be int32")
    require(k_cache.shape[1] == num_kv_heads and k_cache.shape[3] == head_dim, "k_cache layout")
    require(v_cache.shape[2] == head_dim, "v_cache layout")
    dev = qkv.part.device if part is not None else qkv.device
    q = torch.empty((T, num_heads, head_dim), dtype=torch.bfloat16, device=dev)
    check(lib().eia_rope_qkv_cache(
        None if part is not None else ptr(qkv), 0 if part is not None else qkv.stride(0),
        ptr(part.part) if part is not None else None, part.sk if part is not None else 0,
        ptr(positions), ptr(cos_sin), ptr(slot_mapping), ptr(k_cache),
        ptr(v_cache), ptr(q), ptr(bias), ptr(q_norm_w), ptr(k_norm_w), float(norm_eps), T,
        num_heads, num_kv_heads, head_dim, k_cache.shape[2],
        1 if (rotary is None or rotary.is_neox) else 0, stream(q)), "rope_qkv_cache")
    return q
