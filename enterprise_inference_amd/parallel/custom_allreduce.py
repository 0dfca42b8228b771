"""Custom xGMI all-reduce (K12) for decode-sized TP messages.

Each rank registers one IPC-shared device buffer (hipIpcGetMemHandle, exchanged
over the gloo group) plus a signal area.  Per call every rank copies its input
into its own buffer, raises a flag, and the kernel in csrc/kernels/allreduce.hip
either
  * one-shot: reads all peers' buffers and sums (1 sync; small messages), or
  * two-shot: reduce-scatter its 1/n slice from all peers, then all-gather the
    reduced slices (2 syncs; every xGMI link carries 2S/n bytes).
Larger messages go to RCCL (parallel/comm.py).  See SURVEY §2.12 for the xGMI
arithmetic behind the crossover.
"""

from __future__ import annotations

import ctypes
import logging
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import _native
from . import comm, state

logger = logging.getLogger(__name__)

_hip = None


def _hiprt():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so.7")
    return _hip


class _IpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def _ipc_get(ptr: int) -> bytes:
    h = _IpcHandle()
    rc = _hiprt().hipIpcGetMemHandle(ctypes.byref(h), ctypes.c_void_p(ptr))
    if rc != 0:
        raise RuntimeError(f"hipIpcGetMemHandle failed ({rc})")
    return bytes(h.reserved)


def _ipc_open(handle: bytes) -> int:
    h = _IpcHandle()
    ctypes.memmove(ctypes.addressof(h), handle, 64)
    p = ctypes.c_void_p()
    rc = _hiprt().hipIpcOpenMemHandle(ctypes.byref(p), h, ctypes.c_uint(1))
    if rc != 0:
        raise RuntimeError(f"hipIpcOpenMemHandle failed ({rc})")
    return p.value


class CustomAllReduce:
    MAX_RANKS = 8
    SIGNAL_BYTES = 64 * 1024

    def __init__(self, max_bytes: int):
        self.rank = state.tp_rank()
        self.world = state.tp_size()
        self.max_bytes = max_bytes
        dev = torch.device("cuda", torch.cuda.current_device())
        # data buffer (+ signal area at the end), zero-initialised
        self.buf = torch.zeros(max_bytes + self.SIGNAL_BYTES, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        my = _ipc_get(self.buf.data_ptr())
        handles: List[Optional[bytes]] = [None] * self.world
        dist.all_gather_object(handles, my, group=state.tp_cpu_group())
        ptrs = []
        for r, h in enumerate(handles):
            ptrs.append(self.buf.data_ptr() if r == self.rank else _ipc_open(h))
        self.peer_ptrs = torch.tensor(ptrs + [0] * (self.MAX_RANKS - self.world), dtype=torch.int64,
                                      device=dev)
        self.epoch = torch.zeros(1, dtype=torch.int32, device=dev)
        self.lib = _native.kernels()
        self.oneshot_max = 512 * 1024

    def should_use(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and n <= self.max_bytes
                and n % 16 == 0)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        n = x.numel()
        fn = self.lib.eia_ar_oneshot if n * 2 <= self.oneshot_max else self.lib.eia_ar_twoshot
        st = torch.cuda.current_stream().cuda_stream
        rc = fn(x.data_ptr(), x.data_ptr(), self.peer_ptrs.data_ptr(), self.epoch.data_ptr(),
                self.rank, self.world, n, self.max_bytes, 0, st)
        _native.check(rc, "custom_allreduce")
        return x


def init_custom_allreduce(max_bytes: int) -> Optional[CustomAllReduce]:
    if state.tp_size() == 1 or not torch.cuda.is_available():
        return None
    if not hasattr(_native.kernels(), "eia_ar_oneshot"):
        return None
    if state.tp_size() > CustomAllReduce.MAX_RANKS:
        return None
    try:
        ar = CustomAllReduce(max_bytes)
    except Exception as e:   # noqa: BLE001 - RCCL remains correct
        logger.warning("custom all-reduce disabled: %s", e)
        return None
    comm.set_custom_allreduce(ar)
    return ar
