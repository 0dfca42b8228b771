"""RMSNorm / LayerNorm ops (K5, K5b) -> csrc/kernels/norm.hip on the GPU."""

from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import reference as ref
from ._dispatch import check, lib, ptr, require, stream, use_hip


def _rows(x: torch.Tensor) -> torch.Tensor:
    return x.reshape(-1, x.shape[-1])


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not (use_hip(x) and x.dtype == torch.bfloat16):
        r = ref.rms_norm(x, weight, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    x2 = _rows(x)
    require(x2.stride(-1) == 1, "rms_norm: last dim must be contiguous")
    o = torch.empty(x.shape, dtype=x.dtype, device=x.device) if out is None else out
    o2 = _rows(o)
    T, H = x2.shape
    check(lib().eia_rms_norm(ptr(o2), ptr(x2), None, ptr(weight), float(eps), T, H,
                             x2.stride(0), o2.stride(0), stream(x)), "rms_norm")
    return o


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor,
                       eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """residual <- x + residual (in place); returns (rms_norm(residual), residual)."""
    if not (use_hip(x, residual) and x.dtype == torch.bfloat16):
        out, r = ref.fused_add_rms_norm(x, residual, weight, eps)
        residual.copy_(r)
        return out, residual
    x2, r2 = _rows(x), _rows(residual)
    require(r2.is_contiguous() and x2.stride(-1) == 1, "fused_add_rms_norm: layout")
    T, H = x2.shape
    o = torch.empty_like(r2)
    check(lib().eia_rms_norm(ptr(o), ptr(x2), ptr(r2), ptr(weight), float(eps), T, H,
                             x2.stride(0), o.stride(0), stream(x)), "fused_add_rms_norm")
    return o.view(residual.shape), residual


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], eps: float,
               residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """LayerNorm; with ``residual`` computes residual <- x + residual first (in place)."""
    if not (use_hip(x) and x.dtype == torch.bfloat16):
        if residual is not None:
            out, r = ref.fused_add_layer_norm(x, residual, weight, bias, eps)
            residual.copy_(r)
            return out
        return ref.layer_norm(x, weight, bias, eps)
    x2 = _rows(x).contiguous()
    T, H = x2.shape
    o = torch.empty_like(x2)
    r2 = None if residual is None else _rows(residual)
    check(lib().eia_layer_norm(ptr(o), ptr(x2), ptr(r2), ptr(weight), ptr(bias), float(eps), T, H,
                               stream(x)), "layer_norm")
    return o.view(x.shape)
