"""Executors: how a scheduled step reaches the GPU(s).

* ``UniprocExecutor``  -- one ModelRunner in this process (TP=1, or the CPU path).
* ``TPExecutor``       -- tensor parallel, one process per GPU (the reference's
  ``--distributed_executor_backend mp``, core/helm-charts/vllm/xeon-values.yaml:78-79).
  The driver (TP rank 0) owns the scheduler and block manager; per step it
  publishes (plan, staging bytes) through the native shared-memory ring
  (csrc/runtime/shm_ring.cpp) and every rank replays the same plan; the
  collectives inside the model (RCCL / custom xGMI all-reduce) keep them in
  lockstep.  Workers are spawned here, or are already running under torchrun.
"""

from __future__ import annotations

import logging
import multiprocessing as mp
import os
import socket
import time
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import _native
from ..config import EngineConfig
from ..parallel import state as pstate
from .model_runner import ModelRunner, StepOutput

logger = logging.getLogger(__name__)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _agree_num_blocks(nb: int) -> int:
    if len(pstate.replica_ranks()) == 1:
        return nb
    t = torch.tensor([nb], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=pstate.replica_cpu_group())
    return int(t.item())


def describe_distributed(runner: Optional[ModelRunner] = None) -> dict:
    """What THIS rank's process group looks like (the world size RCCL formed, its TP / PP
    coordinates, the collective backend) and the custom all-reduce decision -- gathered over
    the replica at start-up (``gather_dist_info``) so a multi-GPU run describes itself: a
    silent fallback to RCCL then shows up as a reason, not as a slow kernel."""
    from ..parallel import custom_allreduce as car
    info = {"rank": dist.get_rank() if dist.is_initialized() else 0,
            "world_size": dist.get_world_size() if dist.is_initialized() else 1,
            "backend": pstate.backend(), "tp_rank": pstate.tp_rank(),
            "tp_size": pstate.tp_size(), "pp_rank": pstate.pp_rank(),
            "pp_size": pstate.pp_size(), "pid": os.getpid()}
    if runner is not None and runner.is_gpu:
        info["device"] = str(runner.device)
    st = dict(car.STATUS)
    tuning = st.pop("tuning", None)
    info["custom_allreduce"] = st
    if tuning:
        info["custom_allreduce"]["tuning"] = {k: tuning[k] for k in
                                              ("sizes", "oneshot_us", "twoshot_us", "rccl_us")
                                              if k in tuning}
    return info


def gather_dist_info(runner: ModelRunner) -> List[dict]:
    """Every replica rank's ``describe_distributed`` (a gloo all-gather over the replica's
    CPU group; a one-process engine reports itself)."""
    mine = describe_distributed(runner)
    grp = pstate.replica_cpu_group()
    if len(pstate.replica_ranks()) == 1 or grp is None:
        return [mine]
    out = [None] * len(pstate.replica_ranks())
    dist.all_gather_object(out, mine, group=grp)
    return out


def setup_runner(cfg: EngineConfig) -> ModelRunner:
    runner = ModelRunner(cfg)
    ar = None
    if cfg.parallel.tensor_parallel_size > 1 and runner.is_gpu and \
            not cfg.parallel.disable_custom_all_reduce:
        from ..parallel.custom_allreduce import init_custom_allreduce
        ar = init_custom_allreduce(cfg.parallel.custom_allreduce_max_bytes)
    elif cfg.parallel.tensor_parallel_size > 1:
        from ..parallel import custom_allreduce as car
        car.STATUS = {"active": False, "reason": "disabled" if runner.is_gpu and
                      cfg.parallel.disable_custom_all_reduce else "no GPU"}
    runner.dist_info = gather_dist_info(runner)
    nb = runner.determine_num_blocks()
    nb = _agree_num_blocks(nb)
    runner.allocate_kv_cache(nb)
    # K14 swap space on every rank of the replica (each swaps its own KV shard), same count
    from .swap import swap_blocks_for
    runner.allocate_swap(_agree_num_blocks(
        swap_blocks_for(runner.kv_bytes_per_block(), cfg.cache.swap_space_gb)
        if swap_enabled(runner) else 0))
    runner.capture_graphs()
    runner.ar_poller = None
    if ar is not None:
        from ..parallel.custom_allreduce import ErrorPoller
        runner.ar_poller = ErrorPoller(ar)
        runner.ar_poller.check_now()     # profiling run + graph warm-up used the kernel
    return runner


def swap_enabled(runner: ModelRunner) -> bool:
    """Swapping KV into host memory only pays off from a GPU: a CPU engine's KV already lives
    in host RAM (vLLM's CPU backend has no swap space either), so it keeps recompute
    preemption -- EIA_CPU_SWAP=1 turns it on for the CPU tests of the swap machinery."""
    return runner.is_gpu or os.environ.get("EIA_CPU_SWAP", "0") not in ("0", "", "false")


def _init_dist(cfg: EngineConfig) -> None:
    pstate.init_distributed(cfg.parallel.tensor_parallel_size,
                            backend=cfg.parallel.dist_backend,
                            enable_expert_parallel=cfg.parallel.enable_expert_parallel,
                            pp_size=cfg.parallel.pipeline_parallel_size)


class UniprocExecutor:
    # steps can be launched ahead of reading their tokens back (engine overlapped scheduling)
    supports_overlap = True

    def __init__(self, cfg: EngineConfig, runner: Optional[ModelRunner] = None):
        self.runner = runner or setup_runner(cfg)
        self.num_blocks = self.runner.num_blocks

    def dist_info(self) -> List[dict]:
        return getattr(self.runner, "dist_info", None) or [describe_distributed(self.runner)]

    def execute(self, bm, sched) -> StepOutput:
        return self.runner.execute(bm, sched)

    def launch(self, bm, sched, overlap: bool):
        return self.runner.launch(bm, sched, overlap)

    # KV swap (K14): the pool is allocated in setup_runner (swap_enabled)
    def allocate_swap(self, swap_space_gb: float) -> int:
        return getattr(self.runner, "num_cpu_blocks", 0)

    def swap_out(self, gpu_blocks, cpu_blocks) -> None:
        self.runner.swap_out(gpu_blocks, cpu_blocks)

    def encode_images(self, pixel_values):
        """Vision tower + projector on this rank's device (multimodal prompts, TP=1)."""
        enc = getattr(self.runner.model, "encode_images", None)
        if enc is None:
            raise ValueError("this model does not accept image inputs")
        return enc(pixel_values)

    def swap_in(self, cpu_blocks, gpu_blocks) -> None:
        self.runner.swap_in(cpu_blocks, gpu_blocks)

    def copy_blocks(self, pairs) -> None:
        self.runner.copy_blocks(pairs)

    def shutdown(self) -> None:
        pass


def _alive(pid: Optional[int]) -> bool:
    if not pid:
        return True
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def worker_loop(runner: ModelRunner, ring_name: str, driver_pid: Optional[int] = None) -> None:
    """Non-driver TP rank: replay every plan the driver publishes until the empty shutdown
    message arrives (or the driver process is gone -- then the collectives could never
    complete, so the worker exits instead of waiting forever)."""
    ring = _native.runtime().ShmRing(ring_name, False)
    poller = getattr(runner, "ar_poller", None)
    with torch.no_grad():
        while True:
            msg = ring.get(1.0)
            if msg is None:
                if not _alive(driver_pid):
                    logger.error("TP driver %s is gone; worker exiting", driver_pid)
                    return
                continue
            if not msg:
                return
            runner.replay(runner.load_message(msg))
            if poller is not None:
                try:
                    poller.step()
                except RuntimeError:
                    # the driver's monitor sees this exit and takes the replica down with it
                    logger.critical("custom all-reduce error on TP rank %d; worker exiting",
                                    pstate.tp_rank())
                    os._exit(71)


def _spawned_worker(cfg: EngineConfig, rank: int, world: int, port: int, ring_name: str,
                    driver_pid: int) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    if cfg.device == "cuda" and torch.cuda.device_count() > 0:
        if cfg.parallel.share_device:
            torch.cuda.set_device(0)        # one-GPU TP rehearsal: every rank on cuda:0
        else:
            torch.cuda.set_device(rank)
            from ..utils.numa import pin_to_device
            pin_to_device(rank)
    _init_dist(cfg)
    runner = setup_runner(cfg)
    from ..utils.gc_tuning import tune_after_startup
    tune_after_startup()
    worker_loop(runner, ring_name, driver_pid)
    pstate.destroy_distributed()


class TPExecutor:
    """Driver side of tensor (and pipeline) parallelism: one process per rank of the replica.

    Per step the driver publishes ONE message through the native shm ring: a fixed 32-word
    plan header + the staging bytes (ids/positions/slots/block tables + sampling params);
    every rank replays it and samples on its gathered logits, so the next step can be
    launched before this one's tokens reach the host (overlapped scheduling, as TP=1).
    Worker processes are watched: if one dies the driver cannot complete another
    collective, so it fails fast (``os._exit``) and the pod restarts instead of hanging
    until the RCCL timeout."""

    def __init__(self, cfg: EngineConfig, spawn: bool = True):
        tp = cfg.parallel.tensor_parallel_size * cfg.parallel.pipeline_parallel_size
        self.procs = []
        self.ring_name = f"/eia_ring_{os.getpid()}_{id(self) & 0xffff}"
        rt = _native.runtime()
        self.ring = rt.ShmRing(self.ring_name, True, tp - 1, 8, 16 << 20)
        self.supports_overlap = cfg.parallel.pipeline_parallel_size == 1
        self._closed = False
        if spawn and not dist.is_initialized():
            port = _free_port()
            ctx = mp.get_context("spawn")
            for r in range(1, tp):
                p = ctx.Process(target=_spawned_worker,
                                args=(cfg, r, tp, port, self.ring_name, os.getpid()), daemon=True)
                p.start()
                self.procs.append(p)
            keys = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                    "TORCHELASTIC_USE_AGENT_STORE")
            saved = {k: os.environ.get(k) for k in keys}
            os.environ.update(RANK="0", WORLD_SIZE=str(tp), LOCAL_RANK="0",
                              MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            os.environ.pop("TORCHELASTIC_USE_AGENT_STORE", None)   # this rank hosts the store
            if cfg.device == "cuda" and torch.cuda.device_count() > 0:
                torch.cuda.set_device(0)
            try:
                _init_dist(cfg)
            finally:
                # the rendezvous env is only for init: leaving it behind would make a later
                # engine in this process think it is a torchrun-launched rank
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            self._start_monitor()
        self.runner = setup_runner(cfg)
        self.num_blocks = self.runner.num_blocks
        self._swaps = []             # (kind, gpu block, cpu block) until the next plan

    def dist_info(self) -> List[dict]:
        return getattr(self.runner, "dist_info", None) or [describe_distributed(self.runner)]

    # ------------------------------------------------------------------ liveness
    def dead_workers(self):
        return [p for p in self.procs if not p.is_alive()]

    def _start_monitor(self) -> None:
        import threading

        def watch():
            while not self._closed:
                dead = self.dead_workers()
                if dead and not self._closed:
                    logger.critical("TP worker(s) %s died (exit codes %s); aborting the driver",
                                    [p.pid for p in dead], [p.exitcode for p in dead])
                    os._exit(70)
                time.sleep(0.5)

        threading.Thread(target=watch, name="eia-tp-monitor", daemon=True).start()

    def _publish(self, msg: bytes) -> None:
        while not self.ring.put(msg, 1.0):
            dead = self.dead_workers()
            if dead:
                raise RuntimeError(f"TP worker(s) {[p.pid for p in dead]} died")

    # ------------------------------------------------------------------ KV swap (K14)
    # Every rank holds its own KV shard (and PP stage layers), so swaps travel with the
    # step plan and each rank applies them before the step's kernels (ModelRunner.run).
    def allocate_swap(self, swap_space_gb: float) -> int:
        return getattr(self.runner, "num_cpu_blocks", 0)

    def swap_out(self, gpu_blocks, cpu_blocks) -> None:
        self._swaps += [(0, g, c) for g, c in zip(gpu_blocks, cpu_blocks)]

    def swap_in(self, cpu_blocks, gpu_blocks) -> None:
        self._swaps += [(1, g, c) for c, g in zip(cpu_blocks, gpu_blocks)]

    def copy_blocks(self, pairs) -> None:
        self._swaps += [(2, a, b) for a, b in pairs]

    def _take_swaps(self):
        import numpy as np
        if not self._swaps:
            return None
        ops, self._swaps = self._swaps, []
        return np.asarray(ops, dtype=np.int32).reshape(-1)

    # ------------------------------------------------------------------ steps
    def launch(self, bm, sched, overlap: bool):
        r = self.runner
        plan = r.prepare(bm, sched)
        plan.swap = self._take_swaps()
        h = r.launch_plan(plan, sched, overlap,
                          publish=lambda pl: self._publish(r.encode_plan(pl)))
        if r.ar_poller is not None:
            r.ar_poller.step()          # raises CustomAllReduceError -> engine dead, exit
        return h

    def execute(self, bm, sched) -> StepOutput:
        return self.launch(bm, sched, overlap=False).result()

    def shutdown(self) -> None:
        self._closed = True
        try:
            self.ring.put(b"", 5.0)
        except Exception:   # noqa: BLE001
            pass
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        self.procs = []


class FakeExecutor:
    """Test double for host-path benchmarking (``EIA_FAKE_STEP_MS=<ms>``): no model; every step
    sleeps the given time (a stand-in for the GPU) and samples uniform random tokens.  With it
    the API server / engine core / SSE path -- and bench.py's multi-replica fan-out -- run on a
    CPU box at the real step cadence (tests/test_bench_fanout_cpu.py)."""

    supports_overlap = False

    def __init__(self, cfg: EngineConfig, step_ms: float):
        import random as _random
        self.step_s = step_ms / 1000.0
        self.num_blocks = cfg.cache.num_gpu_blocks or 16384
        self.vocab = cfg.model.vocab_size
        self._rng = _random.Random(cfg.seed)
        self._tp = cfg.parallel.tensor_parallel_size

    def dist_info(self) -> List[dict]:
        """The description a real TP replica gives (one record per rank), so the report
        plumbing is testable on the CPU; the fake forms no process group."""
        return [{"rank": r, "world_size": self._tp, "backend": "fake", "tp_rank": r,
                 "tp_size": self._tp, "pp_rank": 0, "pp_size": 1, "pid": os.getpid(),
                 "custom_allreduce": {"active": False, "reason": "fake executor"}}
                for r in range(self._tp)]

    def execute(self, bm, sched) -> StepOutput:
        import time as _time
        n = len(sched.decodes) + sum(1 for p in sched.prefills if p.samples)
        _time.sleep(self.step_s)
        return StepOutput([self._rng.randrange(3, self.vocab) for _ in range(n)], None)

    def copy_blocks(self, pairs) -> None:
        pass

    def shutdown(self) -> None:
        pass


def make_executor(cfg: EngineConfig):
    fake = os.environ.get("EIA_FAKE_STEP_MS")
    if fake:
        return FakeExecutor(cfg, float(fake))
    if cfg.parallel.tensor_parallel_size * cfg.parallel.pipeline_parallel_size > 1:
        if dist.is_initialized():
            # launched under torchrun: this process is TP rank 0 of its group
            return TPExecutor(cfg, spawn=False)
        return TPExecutor(cfg, spawn=True)
    return UniprocExecutor(cfg)
