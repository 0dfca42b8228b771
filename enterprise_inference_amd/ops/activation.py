"""Gated activations (K7 epilogue form) -> csrc/kernels/activation.hip."""

from __future__ import annotations

import torch

from . import reference as ref
from ._dispatch import check, lib, ptr, stream, use_hip

_KIND = {"silu": 0, "swiglu": 0, "gelu_tanh": 1, "gelu_pytorch_tanh": 1, "gelu_new": 1,
         "gelu": 2, "gelu_erf": 2}


def act_and_mul(x: torch.Tensor, act: str = "silu") -> torch.Tensor:
    kind = _KIND[act]
    if not (use_hip(x) and x.dtype == torch.bfloat16):
        return ref.silu_and_mul(x) if kind == 0 else ref.gelu_and_mul(x) if kind == 1 else (
            (torch.nn.functional.gelu(x[..., :x.shape[-1] // 2].float()) *
             x[..., x.shape[-1] // 2:].float()).to(x.dtype))
    x2 = x.reshape(-1, x.shape[-1])
    T, F2 = x2.shape
    F = F2 // 2
    out = torch.empty((T, F), dtype=x.dtype, device=x.device)
    check(lib().eia_act_and_mul(ptr(out), ptr(x2), T, F, x2.stride(0), out.stride(0), kind,
                                stream(x)), "act_and_mul")
    return out.view(*x.shape[:-1], F)


def silu_and_mul(x: torch.Tensor) -> torch.Tensor:
    return act_and_mul(x, "silu")


def activation(x: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return torch.relu(x)
    kind = _KIND[act]
    if not (use_hip(x) and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0):
        if kind == 0:
            return torch.nn.functional.silu(x.float()).to(x.dtype)
        return torch.nn.functional.gelu(x.float(), approximate="tanh" if kind == 1 else "none").to(x.dtype)
    out = torch.empty_like(x)
    check(lib().eia_act(ptr(out), ptr(x), x.numel(), kind, stream(x)), "activation")
    return out
