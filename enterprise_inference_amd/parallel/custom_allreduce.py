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

Before it serves, ``init_custom_allreduce`` checks and sizes the kernel on the real links:
  * self-test: one-shot, two-shot and the fused add+RMSNorm at three sizes each against
    RCCL on the same inputs (integer-valued bf16, so every correct sum is exact and the
    comparison is bit-for-bit); any mismatch on any rank -> every rank falls back to RCCL
    (agreed over the gloo group, never one-sided), with the reason logged and exported as
    ``eia:custom_allreduce_active{reason=...}``;
  * tuning: one-shot, two-shot and RCCL timed at 32 KiB..max_bytes on the current stream;
    the per-size maxima over the ranks set the one-shot/two-shot crossover and the largest
    message the custom kernel takes (above it RCCL wins).  EIA_AR_TUNE=0 keeps the defaults.
"""

from __future__ import annotations

import ctypes
import logging
import os
import time
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
        self.use_max = max_bytes          # largest message routed here (tune() may lower it)
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

    @classmethod
    def local_group(cls, world: int, max_bytes: int, nblocks: int = 16):
        """W 'ranks' inside ONE process on one GPU (each rank's buffers are ordinary in-process
        allocations; each rank must launch on its own stream): the kernel-level rehearsal of
        the cross-GPU protocol used by the GPU tests, minus IPC.  Returns W instances; close
        rank 0's to free every buffer."""
        lib = _native.kernels()
        objs = []
        sigs, datas, own = [], [], []
        for _ in range(world):
            for nb, lst in ((lib.eia_ar_signal_bytes(), sigs), (2 * max_bytes, datas)):
                p = ctypes.c_void_p()
                rc = lib.eia_ar_alloc(ctypes.byref(p), ctypes.c_long(nb))
                if rc != 0:
                    raise RuntimeError(f"eia_ar_alloc({nb}) failed ({rc})")
                lst.append(p.value)
                own.append(p.value)
        for r in range(world):
            o = cls.__new__(cls)
            o.rank, o.world, o.cpu_group = r, world, None
            o.max_bytes = o.use_max = max_bytes
            o.nblocks = nblocks
            o.oneshot_max = int(os.environ.get("EIA_AR_ONESHOT_MAX", 512 * 1024))
            o.lib = lib
            o._own = own if r == 0 else []
            o._opened = []
            o._sig_arr = (ctypes.c_void_p * world)(*sigs)
            o._data_arr = (ctypes.c_void_p * world)(*datas)
            o.own_sig = sigs[r]
            objs.append(o)
        return objs

    def _alloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        rc = self.lib.eia_ar_alloc(ctypes.byref(p), ctypes.c_long(nbytes))
        if rc != 0:
            raise RuntimeError(f"eia_ar_alloc({nbytes}) failed ({rc})")
        self._own.append(p.value)
        return p.value

    def should_use(self, x: torch.Tensor) -> bool:
        n = x.numel() * x.element_size()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and n <= self.use_max
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

    def can_fuse_norm(self, x) -> bool:
        """``x``: the [T, H] bf16 partial sums, or the row-parallel GEMM's split-K slabs
        (``gemm.SplitK``, no bias) -- summed while the kernel stages them."""
        if getattr(x, "part", None) is not None and hasattr(x, "sk"):
            T, H = x.shape
            return (x.bias is None and x.part.is_cuda and x.part.is_contiguous()
                    and T * H * 2 <= self.use_max and H % 8 == 0 and H <= 16384)
        return (self.should_use(x) and x.dim() == 2 and x.shape[1] % 8 == 0
                and x.shape[1] <= 16384)

    def add_rmsnorm(self, x, residual: torch.Tensor, weight: torch.Tensor,
                    eps: float, twoshot: Optional[bool] = None) -> torch.Tensor:
        """One kernel: all-reduce x over the TP group, residual += sum (in place), returns
        rmsnorm(residual) * weight.  Bit-identical to all_reduce + fused_add_rms_norm.  A
        ``gemm.SplitK`` input is reduced over its K slabs in the same kernel (bit-identical to
        materialising it first), so the row-parallel GEMM needs no reduce launch of its own."""
        T, H = x.shape
        out = torch.empty(T, H, dtype=residual.dtype, device=residual.device)
        if twoshot is None:
            twoshot = T * H * 2 > self.oneshot_max and T >= self.world
        st = torch.cuda.current_stream().cuda_stream
        sig = ctypes.cast(self._sig_arr, ctypes.c_void_p)
        data = ctypes.cast(self._data_arr, ctypes.c_void_p)
        if getattr(x, "part", None) is not None and hasattr(x, "sk"):
            rc = self.lib.eia_ar_add_rmsnorm_splitk(
                sig, data, self.rank, self.world, x.part.data_ptr(), x.sk, residual.data_ptr(),
                weight.data_ptr(), out.data_ptr(), float(eps), T, H, self.max_bytes,
                int(bool(twoshot)), self.nblocks, st)
        else:
            rc = self.lib.eia_ar_add_rmsnorm(sig, data, self.rank, self.world, x.data_ptr(),
                                             residual.data_ptr(), weight.data_ptr(),
                                             out.data_ptr(), float(eps), T, H, self.max_bytes,
                                             int(bool(twoshot)), self.nblocks, st)
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


# ----------------------------------------------------------------------------- init checks

STATUS = {"active": False, "reason": "not initialised"}


def selftest_cases(max_bytes: int, oneshot_max: int, hidden: int = 4096):
    """(op, shape, kind) of the init-time self-test: plain all-reduce at a small, a
    crossover-sized and a large message in both forms, and the fused add+RMSNorm at decode
    rows in both forms (only shapes the kernel accepts within ``max_bytes``)."""
    cases = []
    for nbytes in (16 << 10, oneshot_max, min(4 << 20, max_bytes)):
        n = max(8, (nbytes // 2) // 8 * 8)
        if 2 * n <= max_bytes:
            cases += [("ar", (n,), 0), ("ar", (n,), 1)]
    for T in (1, 65, 256):
        if T * hidden * 2 <= max_bytes:
            cases += [("norm", (T, hidden), 0), ("norm", (T, hidden), 1)]
    if 65 * hidden * 2 <= max_bytes:   # the row-parallel GEMM's split-K slabs as the input
        cases += [("norm_sk", (65, hidden), 0), ("norm_sk", (65, hidden), 1)]
    return cases


def selftest_inputs(case, rank: int, device, seed: int = 1234):
    """Integer-valued bf16 inputs in [-4, 4] (rank-dependent), so any correct reduction over
    <= 8 ranks is exact in bf16 and results compare bit-for-bit; the residual and norm weight
    are the same on every rank."""
    op, shape, kind = case
    g = torch.Generator(device="cpu").manual_seed(seed + 7919 * rank + sum(shape) + kind)
    x = torch.randint(-4, 5, shape, generator=g).to(torch.bfloat16)
    if op == "ar":
        return (x.to(device),)
    if op == "norm_sk":      # two integer-valued fp32 slabs whose bf16 sum is x exactly
        a = torch.randint(-2, 3, shape, generator=g).float()
        x = (a + torch.randint(-2, 3, shape, generator=g).float()).to(torch.bfloat16)
        part = torch.stack([a, x.float() - a])
    g2 = torch.Generator(device="cpu").manual_seed(seed + sum(shape))
    res = torch.randint(-8, 9, shape, generator=g2).to(torch.bfloat16)
    w = (1.0 + torch.rand(shape[1], generator=g2)).to(torch.bfloat16)
    if op == "norm_sk":
        from ..ops.gemm import SplitK
        return x.to(device), res.to(device), w.to(device), \
            SplitK(part.to(device), 2, shape[0], shape[1])
    return x.to(device), res.to(device), w.to(device)


def run_self_test(ar, reference, device, cases=None, eps: float = 1e-5) -> Optional[str]:
    """Every case through ``ar`` and through ``reference(x) -> sum over ranks`` (RCCL);
    returns None when all match, else a short description of the first mismatches."""
    from ..ops import norm as norm_ops
    bad = []
    for case in cases if cases is not None else selftest_cases(ar.max_bytes, ar.oneshot_max):
        op, shape, kind = case
        # Every rank runs the SAME collectives in the same order whatever fails locally: a
        # rank that left the loop early would strand its peers in the next case's RCCL
        # reference.  A local failure skips only this rank's custom call (its
        # peers' custom kernel then spins out and sets their error flag, which is checked below).
        try:
            t = selftest_inputs(case, ar.rank, device)
        except Exception as e:   # noqa: BLE001
            bad.append(f"{op} {tuple(shape)} inputs raised {e!r}")
            t = (torch.zeros(shape, dtype=torch.bfloat16, device=device),)
        want = reference(t[0].clone())
        if len(t) == 1 and op != "ar":
            continue
        try:
            if op == "ar":
                got = ar.all_reduce(t[0].clone(), kind=kind)
                ok = torch.equal(got, want)
                err = 0.0 if ok else float((got.float() - want.float()).abs().max())
            else:
                x, res, w = t[:3]
                r_want = res.clone()
                want, r_want = norm_ops.fused_add_rms_norm(want, r_want, w, eps)
                r_got = res.clone()
                src = t[3] if op == "norm_sk" else x.clone()
                got = ar.add_rmsnorm(src, r_got, w, eps, twoshot=bool(kind))
                ok = torch.equal(r_got, r_want) and bool(
                    torch.allclose(got.float(), want.float(), rtol=1e-2, atol=1e-2))
                err = 0.0 if ok else max(float((r_got.float() - r_want.float()).abs().max()),
                                         float((got.float() - want.float()).abs().max()))
        except Exception as e:   # noqa: BLE001 - recorded; the loop goes on in step
            bad.append(f"{op}/{'2shot' if kind else '1shot'} {tuple(shape)} raised {e!r}")
            continue
        if not ok:
            bad.append(f"{op}{'/2shot' if kind else '/1shot'} {tuple(shape)} max|err| {err:.3g}")
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if ar.error_flag():
        bad.append("barrier spin limit hit during the self-test")
    return "; ".join(bad[:4]) if bad else None


def _time_us(fn, iters: int = 20) -> float:
    fn()
    if not torch.cuda.is_available():          # CPU stand-ins in the tests: wall clock
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        return (time.perf_counter() - t0) * 1e6 / iters
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def tune_thresholds(sizes, t_one, t_two, t_rccl, max_bytes: int):
    """(oneshot_max, use_max) from per-size timings (bytes, us; the max over ranks).
    one-shot serves every size up to the last one where it still beats two-shot (from the
    small end, contiguous); the custom kernel takes messages up to the last size where its
    better form beats RCCL."""
    oneshot_max = sizes[0]
    for sz, a, b in zip(sizes, t_one, t_two):
        if a > b:
            break
        oneshot_max = sz
    use_max = 0
    for sz, a, b, r in zip(sizes, t_one, t_two, t_rccl):
        if min(a, b) <= r:
            use_max = sz
        else:
            break
    return oneshot_max, min(use_max, max_bytes)


def run_tuning(ar, rccl_all_reduce, agree_max) -> dict:
    """Time one-shot / two-shot / RCCL per size on this rank; ``agree_max`` reduces the timing
    vector to its element-wise max over the ranks (same decision everywhere)."""
    sizes = [s for s in (32 << 10, 128 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20,
                         16 << 20, 32 << 20) if s <= ar.max_bytes]
    rows = []
    inf = float("inf")

    def timed(fn):
        try:
            return _time_us(fn)
        except Exception:   # noqa: BLE001 - a failing form never wins; RCCL still runs below
            return inf

    for sz in sizes:
        x = torch.ones(sz // 2, dtype=torch.bfloat16, device=getattr(ar, "device", "cuda"))
        rows.append([timed(lambda: ar.all_reduce(x, kind=0)),
                     timed(lambda: ar.all_reduce(x, kind=1)),
                     _time_us(lambda: rccl_all_reduce(x))])
    t = agree_max(torch.tensor(rows, dtype=torch.float64)).tolist()
    one, two, rc = [r[0] for r in t], [r[1] for r in t], [r[2] for r in t]
    oneshot_max, use_max = tune_thresholds(sizes, one, two, rc, ar.max_bytes)
    return {"sizes": sizes, "oneshot_us": one, "twoshot_us": two, "rccl_us": rc,
            "oneshot_max": oneshot_max, "use_max": use_max}


def init_custom_allreduce(max_bytes: int, factory=None, reference=None, agree=None,
                          tune: Optional[bool] = None) -> Optional[CustomAllReduce]:
    """Build the custom all-reduce for this TP group, self-test it against RCCL and size it;
    returns None (RCCL everywhere) when any rank cannot map the peers or any rank's
    self-test mismatches.  ``factory`` / ``reference`` / ``agree`` are injection points for
    the tests (defaults: CustomAllReduce, RCCL on the TP group, MIN/MAX over the gloo group)."""
    global STATUS
    cpu_group = None
    if factory is None:
        if state.tp_size() == 1 or not torch.cuda.is_available():
            return None
        if state.tp_size() > CustomAllReduce.MAX_RANKS:
            STATUS = {"active": False, "reason": "tp_size > 8"}
            return None
        factory = CustomAllReduce
        cpu_group = state.tp_cpu_group()
    if reference is None:
        def reference(x):
            dist.all_reduce(x, group=state.tp_group())
            return x
    if agree is None:
        def agree(t, op):
            dist.all_reduce(t, op=op, group=cpu_group or state.tp_cpu_group())
            return t
    try:
        ar = factory(max_bytes)
    except Exception as e:   # noqa: BLE001 - RCCL remains correct
        logger.warning("custom all-reduce disabled: %s", e)
        STATUS = {"active": False, "reason": "setup failed"}
        return None
    try:
        why = run_self_test(ar, reference, getattr(ar, "device", "cuda"))
    except Exception as e:   # noqa: BLE001 - a crashing self-test is a failed one
        why = f"self-test raised {e!r}"
    ok = agree(torch.tensor([0 if why else 1], dtype=torch.int32), dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        logger.error("custom all-reduce self-test FAILED (%s); every TP rank uses RCCL",
                     why or "on another rank")
        ar.close()
        STATUS = {"active": False, "reason": "self-test mismatch"}
        return None
    info = {}
    tune = (os.environ.get("EIA_AR_TUNE", "1") != "0") if tune is None else tune
    if tune and (torch.cuda.is_available() or factory is not CustomAllReduce):
        info = run_tuning(ar, reference, lambda t: agree(t, dist.ReduceOp.MAX))
        # The timing pass runs the custom kernels again after the self-test's last spin check:
        # a barrier spin that hits its bound here leaves the sticky flag set, and the engine's
        # ErrorPoller would then fail at start-up.  Every rank reads its flag and the ranks
        # agree (MIN of "clean"), so all of them keep the kernel or all go back to RCCL.
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        clean = agree(torch.tensor([0 if ar.error_flag() else 1], dtype=torch.int32),
                      dist.ReduceOp.MIN)
        if int(clean.item()) == 0:
            logger.error("custom all-reduce barrier spin limit hit while tuning; every TP "
                         "rank uses RCCL")
            ar.close()
            STATUS = {"active": False, "reason": "tuning spin timeout", "tuning": info}
            return None
        ar.oneshot_max, ar.use_max = info["oneshot_max"], info["use_max"]
        logger.info("custom all-reduce tuned: one-shot <= %d B, custom <= %d B (RCCL above)",
                    ar.oneshot_max, ar.use_max)
    # decode_epilogue: how a TP decode layer's row-parallel output reaches the next norm --
    # the skinny GEMM's split-K slabs (or its bf16 tile) go straight into ONE kernel that
    # stages them (summing the slabs), all-reduces over xGMI, adds the residual and normalises
    STATUS = {"active": True, "reason": "ok", "oneshot_max": ar.oneshot_max,
              "use_max": ar.use_max, "decode_epilogue": "splitk+allreduce+add+rmsnorm, 1 launch",
              **({"tuning": info} if info else {})}
    comm.set_custom_allreduce(ar)
    return ar
