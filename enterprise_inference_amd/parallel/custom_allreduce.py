"""Custom xGMI all-reduce (K12) for decode-sized TP messages.

Every rank allocates an UNCACHED signal block and a double-buffered data region
(``eia_ar_alloc`` -> hipExtMallocWithFlags(hipDeviceMallocUncached)), exports them with
hipIpcGetMemHandle, and the handles are exchanged once over the gloo TP group.  Each
call is ONE kernel (csrc/kernels/allreduce.hip): blocks stage their share of the input
into the own buffer, meet the same block of every peer at a flag barrier, then
  * one-shot: sum all W peers' buffers directly (1 sync; small messages), or
  * two-shot: reduce-scatter + all-gather over all links (2 syncs; every xGMI link
    carries 2S/W bytes).
No host-side state changes between calls, so TP decode steps stay HIP-graph capturable.
Messages above ``max_bytes`` go to RCCL (parallel/comm.py).

The one-shot/two-shot crossover defaults to 512 KiB (SURVEY §2.12 xGMI arithmetic:
one-shot moves S per link with one sync, two-shot 2S/W with two).
"""

from __future__ import annotations

import ctypes
import logging
import os
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
        for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
            try:
                _hip = ctypes.CDLL(name)
                break
            except OSError:
                continue
    return _hip


class _IpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def ipc_get(ptr: int) -> bytes:
    h = _IpcHandle()
    rc = _hiprt().hipIpcGetMemHandle(ctypes.byref(h), ctypes.c_void_p(ptr))
    if rc != 0:
        raise RuntimeError(f"hipIpcGetMemHandle failed ({rc})")
    return bytes(h.reserved)


def ipc_open(handle: bytes) -> int:
    h = _IpcHandle()
    ctypes.memmove(ctypes.addressof(h), handle, 64)
    p = ctypes.c_void_p()
    rc = _hiprt().hipIpcOpenMemHandle(ctypes.byref(p), h, ctypes.c_uint(1))
    if rc != 0:
        raise RuntimeError(f"hipIpcOpenMemHandle failed ({rc})")
    return p.value


class CustomAllReduce:
    MAX_RANKS = 8

    def __init__(self, max_bytes: int, group=None, cpu_group=None, rank: Optional[int] = None,
                 world: Optional[int] = None, nblocks: int = 32,
                 oneshot_max: Optional[int] = None):
        self.rank = state.tp_rank() if rank is None else rank
        self.world = state.tp_size() if world is None else world
        self.cpu_group = cpu_group if cpu_group is not None else state.tp_cpu_group()
        self.max_bytes = max_bytes
        self.nblocks = nblocks
        self.oneshot_max = oneshot_max or int(os.environ.get("EIA_AR_ONESHOT_MAX", 512 * 1024))
        self.lib = _native.kernels()
        sig_bytes = self.lib.eia_ar_signal_bytes()
        self._own = []
        sig = self._alloc(sig_bytes)
        data = self._alloc(2 * max_bytes)
        mine = (ipc_get(sig), ipc_get(data))
        handles: List[Optional[tuple]] = [None] * self.world
        dist.all_gather_object(handles, mine, group=self.cpu_group)
        self._opened = []
        sigs, datas = [], []
        err = None
        for r, (hs, hd) in enumerate(handles):
            if r == self.rank:
                sigs.append(sig)
                datas.append(data)
                continue
            try:
                ps, pd = ipc_open(hs), ipc_open(hd)
            except Exception as e:   # noqa: BLE001 - agreed on below, never one-sided
                err = e
                break
            self._opened += [ps, pd]
            sigs.append(ps)
            datas.append(pd)
        # every rank must agree before any of them switches: a rank on RCCL while its peers
        # spin in the custom kernel would hang (or corrupt) the group
        ok = torch.tensor([0 if err else 1], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=self.cpu_group)
        if int(ok.item()) == 0:
            self.close()
            raise RuntimeError(f"custom all-reduce unavailable on some rank ({err!r} here)")
        self._sig_arr = (ctypes.c_void_p * self.world)(*sigs)
        self._data_arr = (ctypes.c_void_p * self.world)(*datas)
        self.own_sig = sig
        dist.barrier(group=self.cpu_group)

    def _alloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        rc = self.lib.eia_ar_alloc(ctypes.byref(p), ctypes.c_long(nbytes))
        if rc != 0:
            raise RuntimeError(f"eia_ar_alloc({nbytes}) failed ({rc})")
        self._own.append(p.value)
        return p.value

    def should_use(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and n <= self.max_bytes
                and x.numel() % 8 == 0)

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                   kind: Optional[int] = None) -> torch.Tensor:
        """In place by default (out = x)."""
        out = x if out is None else out
        n = x.numel()
        if kind is None:
            kind = 0 if n * 2 <= self.oneshot_max else 1
        st = torch.cuda.current_stream().cuda_stream
        rc = self.lib.eia_ar_run(ctypes.cast(self._sig_arr, ctypes.c_void_p),
                                 ctypes.cast(self._data_arr, ctypes.c_void_p), self.rank,
                                 self.world, x.data_ptr(), out.data_ptr(), n, self.max_bytes, kind,
                                 self.nblocks, st)
        _native.check(rc, "custom_allreduce")
        return out

    def can_fuse_norm(self, x: torch.Tensor) -> bool:
        return (self.should_use(x) and x.dim() == 2 and x.shape[1] % 8 == 0
                and x.shape[1] <= 16384)

    def add_rmsnorm(self, x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor,
                    eps: float, twoshot: Optional[bool] = None) -> torch.Tensor:
        """One kernel: all-reduce x over the TP group, residual += sum (in place), returns
        rmsnorm(residual) * weight.  Bit-identical to all_reduce + fused_add_rms_norm."""
        T, H = x.shape
        out = torch.empty_like(x)
        if twoshot is None:
            twoshot = T * H * 2 > self.oneshot_max and T >= self.world
        rc = self.lib.eia_ar_add_rmsnorm(ctypes.cast(self._sig_arr, ctypes.c_void_p),
                                         ctypes.cast(self._data_arr, ctypes.c_void_p), self.rank,
                                         self.world, x.data_ptr(), residual.data_ptr(),
                                         weight.data_ptr(), out.data_ptr(), float(eps), T, H,
                                         self.max_bytes, int(bool(twoshot)), self.nblocks,
                                         torch.cuda.current_stream().cuda_stream)
        _native.check(rc, "custom_allreduce_add_rmsnorm")
        return out

    def raise_on_error(self) -> None:
        """A barrier spin that hit its bound means a peer stalled and this rank summed stale
        buffers: the activations are wrong from then on -- fail instead of serving them."""
        if self.error_flag():
            raise RuntimeError("custom all-reduce barrier timed out (a TP peer stalled); "
                               "results since then are invalid")

    def error_flag(self) -> int:
        v = ctypes.c_int(0)
        _native.check(self.lib.eia_ar_read_err(ctypes.c_void_p(self.own_sig), ctypes.byref(v)),
                      "ar_read_err")
        return v.value

    def read_error_async(self, host_dst: torch.Tensor) -> None:
        """Enqueue a copy of the flag into pinned int32 ``host_dst`` on the current stream."""
        _native.check(self.lib.eia_ar_read_err_async(
            ctypes.c_void_p(self.own_sig), ctypes.c_void_p(host_dst.data_ptr()),
            torch.cuda.current_stream().cuda_stream), "ar_read_err_async")

    def inject_error(self, v: int = 1) -> None:
        """Test hook: set this rank's flag as a timed-out barrier would."""
        _native.check(self.lib.eia_ar_set_err(ctypes.c_void_p(self.own_sig), int(v)),
                      "ar_set_err")

    def close(self) -> None:
        hip = _hiprt()
        if hip is None:
            return
        for p in self._opened:
            hip.hipIpcCloseMemHandle(ctypes.c_void_p(p))
        for p in self._own:
            self.lib.eia_ar_free(ctypes.c_void_p(p))
        self._opened, self._own = [], []


class CustomAllReduceError(RuntimeError):
    """A custom all-reduce barrier timed out: this rank's activations are no longer valid."""


class ErrorPoller:
    """Failure detection for the custom all-reduce.

    A barrier spin that exhausts its bound sets the rank's error flag and the kernel returns
    with stale peer data summed in, so every activation after it is wrong.  The serving loop
    calls ``step()`` once per launched step; every ``every`` steps it enqueues a stream-ordered
    copy of the flag into pinned memory behind an event and, at the next poll, reads the copy
    it enqueued last time (no device-wide synchronisation on the step path).  ``check_now``
    is the synchronous form (after graph capture / warm-up).  Both raise
    ``CustomAllReduceError``; the engine core then reports itself dead (``/health`` -> 500)
    and exits non-zero, so the pod restarts instead of serving garbage."""

    def __init__(self, ar, every: Optional[int] = None):
        self.ar = ar
        self.every = max(1, int(every or os.environ.get("EIA_AR_CHECK_STEPS", 64)))
        self.n = 0
        self._host = torch.zeros(1, dtype=torch.int32, pin_memory=torch.cuda.is_available())
        self._event = None
        self._pending = False

    def _fail(self) -> None:
        raise CustomAllReduceError("custom all-reduce barrier timed out (a TP peer stalled); "
                                   "results since then are invalid")

    def check_now(self) -> None:
        if self.ar.error_flag():
            self._fail()

    def step(self) -> None:
        self.n += 1
        if self.n % self.every:
            return
        if self._pending:
            if self._event is not None:
                self._event.synchronize()    # enqueued `every` steps ago: long complete
            if int(self._host[0]) != 0:
                self._fail()
        self.ar.read_error_async(self._host)
        self._pending = True
        if torch.cuda.is_available():
            self._event = torch.cuda.Event()
            self._event.record()


def init_custom_allreduce(max_bytes: int) -> Optional[CustomAllReduce]:
    if state.tp_size() == 1 or not torch.cuda.is_available():
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
