"""Opt-in profiling and debug hooks.

* ``EIA_TORCH_PROFILER_DIR`` (or vLLM's ``VLLM_TORCH_PROFILER_DIR``): the API server exposes
  ``POST /start_profile`` and ``POST /stop_profile``; between them every engine step runs under
  ``torch.profiler`` (CPU + ROCm kernel activity) and a Chrome trace per session is written to
  the directory (open in Perfetto).  Kernel-level verification on the box uses
  ``scripts/gpu_profile.sh`` (rocprofv3 --kernel-trace --stats).
* ``EIA_CHECK_INVARIANTS=1``: after every engine step the block manager's C++ invariant checker
  (refcounts, free list, no double ownership -- csrc/runtime/kv_manager.cpp) runs and a
  violation raises immediately instead of corrupting KV state silently.
* ``EIA_SYNC_KERNELS=1`` / ``HIP_LAUNCH_BLOCKING=1``: see ops/_dispatch.py.
"""

from __future__ import annotations

import logging
import os
import time
from typing import Optional

logger = logging.getLogger(__name__)


def profiler_dir() -> Optional[str]:
    return os.environ.get("EIA_TORCH_PROFILER_DIR") or os.environ.get("VLLM_TORCH_PROFILER_DIR")


class StepProfiler:
    """torch.profiler session toggled at runtime; wraps engine steps."""

    def __init__(self, out_dir: Optional[str] = None):
        self.out_dir = out_dir or profiler_dir()
        self._prof = None
        self.sessions = 0
        self.last_trace: Optional[str] = None

    @property
    def enabled(self) -> bool:
        return self.out_dir is not None

    @property
    def active(self) -> bool:
        return self._prof is not None

    def start(self) -> None:
        if not self.enabled:
            raise RuntimeError("profiling disabled: set EIA_TORCH_PROFILER_DIR")
        if self._prof is not None:
            return
        import torch
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)   # ROCm activity (roctracer)
        os.makedirs(self.out_dir, exist_ok=True)
        self._prof = torch.profiler.profile(activities=acts, record_shapes=True, with_stack=False)
        self._prof.__enter__()
        logger.info("torch profiler started -> %s", self.out_dir)

    def stop(self) -> Optional[str]:
        if self._prof is None:
            return None
        prof, self._prof = self._prof, None
        prof.__exit__(None, None, None)
        self.sessions += 1
        path = os.path.join(self.out_dir, f"trace_{os.getpid()}_{int(time.time())}_{self.sessions}.json")
        prof.export_chrome_trace(path)
        self.last_trace = path
        logger.info("torch profiler trace written: %s", path)
        return path

    def step(self, fn):
        """Run one engine step (under a record_function range when profiling)."""
        if self._prof is None:
            return fn()
        import torch
        with torch.profiler.record_function("engine_step"):
            return fn()


def invariants_enabled() -> bool:
    return os.environ.get("EIA_CHECK_INVARIANTS", "0") == "1"


def check_engine_invariants(engine) -> None:
    bm = getattr(engine.scheduler, "bm", None)
    if bm is None:
        return
    err = bm.check_invariants()
    if err:
        raise RuntimeError(f"KV block manager invariant violated: {err}")
