"""Device dispatch helpers shared by the op wrappers."""

from __future__ import annotations

import os

import torch

from .. import _native

# Debug switch: run the PyTorch reference ops even on the GPU (never the default).
FORCE_TORCH = os.environ.get("EIA_FORCE_TORCH_OPS", "0") == "1"
# Debug switch (SURVEY §5.2 "HIP_LAUNCH_BLOCKING test mode"): synchronise after every native
# kernel launch and surface asynchronous faults at the op that caused them.
SYNC_KERNELS = (os.environ.get("EIA_SYNC_KERNELS", "0") == "1"
                or os.environ.get("HIP_LAUNCH_BLOCKING", "0") == "1"
                or os.environ.get("AMD_SERIALIZE_KERNEL", "0") == "3")


def use_hip(*tensors: torch.Tensor) -> bool:
    """True when the HIP kernels must be used for these tensors."""
    if FORCE_TORCH:
        return False
    return all(t is None or t.is_cuda for t in tensors) and any(
        t is not None and t.is_cuda for t in tensors)


def ptr(t):
    return None if t is None else t.data_ptr()


def stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def lib():
    return _native.kernels()


def check(status: int, name: str) -> None:
    _native.check(status, name)
    if SYNC_KERNELS and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:   # asynchronous fault: name the op that launched it
            raise RuntimeError(f"{name}: device fault after launch: {e}") from e


def require(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)
