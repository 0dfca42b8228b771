"""Loader for the in-tree native libraries.

* ``_lib/libeia_kernels.so`` -- gfx950 HIP kernels with a C ABI, bound here with
  ctypes (argtypes declared once, so a call costs ~1 µs and is capture-safe:
  launches go to the caller's current HIP stream).
* ``_lib/_eia_runtime*.so`` -- pybind11 host runtime (block manager, batch
  builder, shm ring).

Policy: on a machine with a GPU the HIP kernels are REQUIRED -- a missing or
broken library raises instead of silently falling back to PyTorch ops.
"""

from __future__ import annotations

import ctypes
import importlib
import importlib.util
import os
import sys
import threading
from typing import Optional

import torch  # noqa: F401  (must be imported first: it owns the HIP runtime)

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
_KERNELS_SO = os.path.join(_LIB_DIR, "libeia_kernels.so")
_lock = threading.Lock()
_kernels: Optional[ctypes.CDLL] = None
_runtime = None

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float
IP = ctypes.c_void_p  # int* (device)
S = ctypes.c_void_p   # hipStream_t

_SIGNATURES = {
    "eia_rms_norm": [P, P, P, P, F, I, I, L, L, S],
    "eia_layer_norm": [P, P, P, P, P, F, I, I, S],
    "eia_rope_qkv_cache": [P, L, P, I, IP, P, IP, P, P, P, P, P, P, F, I, I, I, I, I, I, S],
    "eia_paged_decode": [P, L, P, P, IP, I, IP, P, L, P, P, P, F, I, I, I, I, I, I, I, I, IP, S],
    "eia_paged_decode_rope": [P, L, P, I, P, P, P, F, IP, P, IP, I, P, P, IP, I, IP, P, L, P, P, P,
                              F, I, I, I, I, I, I, I, I, IP, S],
    "eia_paged_prefill": [P, L, P, L, P, P, IP, I, IP, IP, IP, I, F, I, I, I, I, I, I, I, I, I, S],
    "eia_paged_prefill_fa": [P, L, P, L, P, P, IP, I, IP, IP, IP, I, F, I, I, I, I, I, I, I, S],
    "eia_act_and_mul": [P, P, I, I, L, L, I, S],
    "eia_act": [P, P, L, I, S],
    "eia_sample": [P, L, I, I, P, P, P, P, P, P, S],
    "eia_apply_penalties": [P, L, P, P, P, I, P, P, P, S],
    "eia_sample_split": [P, L, I, I, I, P, P, P, P, P, S],
    "eia_sample_shard": [P, L, I, I, I, I, P, P, P, P, P, P, P, S],
    "eia_radix_hist": [P, L, I, I, P, P, P, P, P, I, P, S],
    "eia_fill_ids": [P, P, P, I, S],
    "eia_moe_topk": [P, I, I, I, I, I, I, P, P, S],
    "eia_moe_align": [P, I, I, I, I, P, P, P, I, S],
    "eia_moe_route": [P, L, P, I, I, I, I, I, I, P, P, S],
    "eia_moe_gemm": [P, L, P, L, P, P, L, I, I, I, P, P, I, I, I, S],
    "eia_moe_combine": [P, L, P, P, I, I, I, P, L, S],
    "eia_moe_gemm_sk": [P, L, P, L, P, I, I, I, I, P, P, I, I, I, S],
    "eia_moe_combine_sk": [P, I, I, P, P, I, I, I, P, L, S],
    "eia_moe_grouped_gemm": [P, L, IP, P, I, I, I, IP, I, I, P, L, S],
    "eia_gemm_skinny": [P, L, P, L, P, P, L, I, I, I, I, I, I, S],
    "eia_splitk_reduce": [P, I, I, I, P, P, L, S],
    "eia_splitk_swiglu": [P, I, I, I, P, L, S],
    "eia_splitk_add_rmsnorm": [P, I, I, I, P, P, F, P, L, S],
    "eia_ar_alloc": [P, L],
    "eia_moe_splitk_norm_route": [P, I, I, I, P, P, F, P, L, P, I, I, I, I, P, P, P, S],
    "eia_moe_combine_norm": [P, I, I, P, P, I, I, I, P, P, F, P, L, S],
    "eia_ar_free": [P],
    "eia_ar_signal_bytes": [],
    "eia_ar_run": [P, P, I, I, P, P, L, L, I, I, S],
    "eia_ar_read_err": [P, P],
    "eia_ar_read_err_async": [P, P, S],
    "eia_ar_set_err": [P, I],
    "eia_ar_add_rmsnorm": [P, P, I, I, P, P, P, P, F, I, I, L, I, I, S],
    "eia_ar_add_rmsnorm_splitk": [P, P, I, I, P, I, P, P, P, F, I, I, L, I, I, S],
}


def kernels_path() -> str:
    return _KERNELS_SO


def gpu_available() -> bool:
    return torch.cuda.is_available()


def _build_kernels() -> None:
    root = os.path.dirname(os.path.dirname(_LIB_DIR))
    spec = importlib.util.spec_from_file_location("eia_build", os.path.join(root, "csrc", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.build_kernels()


def _build_runtime() -> None:
    root = os.path.dirname(os.path.dirname(_LIB_DIR))
    spec = importlib.util.spec_from_file_location("eia_build", os.path.join(root, "csrc", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.build_runtime()


def kernels() -> ctypes.CDLL:
    """Return the HIP kernel library (building it in-tree if it is missing)."""
    global _kernels
    if _kernels is not None:
        return _kernels
    with _lock:
        if _kernels is not None:
            return _kernels
        if not os.path.exists(_KERNELS_SO):
            _build_kernels()
        lib = ctypes.CDLL(_KERNELS_SO, mode=ctypes.RTLD_GLOBAL)
        missing = [n for n in _SIGNATURES if not hasattr(lib, n)]
        if missing:
            # a stale build: fail here, not at the first call of the missing kernel
            raise RuntimeError(f"{_KERNELS_SO} lacks {missing}; rebuild it "
                               "(python -c 'import __graft_entry__ as g; g.build()')")
        for name, argtypes in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        _kernels = lib
        return lib


def runtime():
    """Return the pybind11 host runtime module (auto-built with g++ if missing)."""
    global _runtime
    if _runtime is not None:
        return _runtime
    with _lock:
        if _runtime is not None:
            return _runtime
        if _LIB_DIR not in sys.path:
            sys.path.insert(0, _LIB_DIR)
        try:
            _runtime = importlib.import_module("_eia_runtime")
        except ImportError:
            _build_runtime()
            importlib.invalidate_caches()
            _runtime = importlib.import_module("_eia_runtime")
        return _runtime


def check(status: int, name: str) -> None:
    if status != 0:
        raise RuntimeError(f"{name} failed with status {status}")


def stream_ptr(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def loaded_native_libraries() -> list[str]:
    """Paths of in-tree native libraries mapped into this process (for smoke checks)."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if _LIB_DIR in line:
                    p = line.split()[-1]
                    if p not in out:
                        out.append(p)
    except OSError:
        pass
    return out
