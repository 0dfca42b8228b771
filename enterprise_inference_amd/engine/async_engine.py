"""Asyncio front-end over the synchronous ``LLMEngine``.

The engine step loop runs on one background thread (the GPU is driven from a
single host thread; TP workers are separate processes fed by the executor).
Request add / abort calls from the HTTP event loop are queued and applied at
the top of each iteration, and every ``RequestOutput`` is handed back to the
request's asyncio queue with ``call_soon_threadsafe``.

Failure handling:
  * ``healthy`` is False until warmup finished and after the loop dies, so
    ``/health`` turns 503/500 and the kubelet restarts the pod (the reference's
    readiness probe, core/helm-charts/vllm/values.yaml:135-141);
  * a step-time watchdog trips when one iteration exceeds
    ``VLLM_ENGINE_ITERATION_TIMEOUT_S`` (core/helm-charts/vllm/xeon-values.yaml:66);
  * ``EIA_FAULT_INJECT`` (test-only) = ``delay_step:<sec>`` | ``crash_after:<steps>``.
"""

from __future__ import annotations

import asyncio
import concurrent.futures
import logging
import os
import queue
import threading
import time
import weakref
from typing import AsyncIterator, Callable, Dict, Optional

from .llm_engine import LLMEngine, RequestOutput
from .sampling_params import SamplingParams

logger = logging.getLogger(__name__)


class SubmittedStream:
    """Async iterator over one submitted request's outputs.

    ``submit`` hands the request to the engine before anyone iterates, so the release of an
    abandoned request cannot live only in the output generator's ``finally``: a generator
    that never started (the client disconnected while the streaming response was still
    sending its headers, or a later prompt of the same completion failed to submit) has no
    frame and its ``finally`` never runs.  The finaliser here runs when the stream is dropped
    and releases the request if nothing else has (``on_abandon`` must be idempotent)."""

    __slots__ = ("_gen", "_fin", "__weakref__")

    def __init__(self, gen, on_abandon: Callable[[], None]):
        self._gen = gen
        self._fin = weakref.finalize(self, on_abandon)

    def __aiter__(self):
        return self

    async def __anext__(self):
        return await self._gen.__anext__()

    async def aclose(self) -> None:
        await self._gen.aclose()
        self._fin()


class EngineDeadError(RuntimeError):
    pass


class AsyncLLMEngine:
    def __init__(self, engine: LLMEngine, metrics=None, log_requests: bool = True):
        self.engine = engine
        self.tokenizer = engine.tokenizer
        engine.delta_outputs = True        # handlers read deltas; finals carry the full text
        self.metrics = metrics
        self.log_requests = log_requests
        self._cmds: "queue.Queue" = queue.Queue()
        self._streams: Dict[str, asyncio.Queue] = {}
        self._loops: Dict[str, asyncio.AbstractEventLoop] = {}
        self._wake = threading.Event()
        self._stop = False
        self.dead: Optional[BaseException] = None
        self.ready = False
        self.last_step_start: Optional[float] = None
        self.timeout_s = float(os.environ.get("VLLM_ENGINE_ITERATION_TIMEOUT_S",
                                              engine.cfg.engine_iteration_timeout_s))
        self._fault = os.environ.get("EIA_FAULT_INJECT", "")
        self._thread = threading.Thread(target=self._run, name="eia-engine", daemon=True)
        self._thread.start()
        self.ready = True
        if metrics is not None:
            metrics.set_healthy(True)

    # ------------------------------------------------------------------ state
    @property
    def healthy(self) -> bool:
        if self.dead is not None or not self.ready:
            return False
        t = self.last_step_start
        return t is None or (time.time() - t) < self.timeout_s

    def check_health(self) -> None:
        if self.dead is not None:
            raise EngineDeadError(f"engine loop died: {self.dead!r}")
        if not self.healthy:
            raise EngineDeadError("engine step exceeded VLLM_ENGINE_ITERATION_TIMEOUT_S")

    # ------------------------------------------------------------------ API
    async def generate(self, request_id: str, prompt: Optional[str], params: SamplingParams,
                       prompt_token_ids=None, priority: int = 0,
                       multi_modal_data=None) -> AsyncIterator[RequestOutput]:
        async for item in self.submit(request_id, prompt, params, prompt_token_ids, priority,
                                      multi_modal_data):
            yield item

    can_submit = True

    def submit(self, request_id: str, prompt: Optional[str], params: SamplingParams,
               prompt_token_ids=None, priority: int = 0,
               multi_modal_data=None) -> AsyncIterator[RequestOutput]:
        """Queue the request now and return its output iterator (MPEngineClient.submit)."""
        self.check_health()
        q: asyncio.Queue = asyncio.Queue()
        loop = asyncio.get_running_loop()
        self._streams[request_id] = q
        self._loops[request_id] = loop
        self._cmds.put(("add", request_id, prompt, params, prompt_token_ids, time.time(), priority,
                        multi_modal_data))
        self._wake.set()
        return SubmittedStream(self._outputs(request_id, q),
                               lambda: self._release(request_id, abort=True))

    def _release(self, request_id: str, abort: bool) -> None:
        """Drop the request's stream; abort it in the engine if it was still open."""
        if self._streams.pop(request_id, None) is not None and abort:
            self.abort(request_id)
        self._loops.pop(request_id, None)

    async def _outputs(self, request_id: str, q: asyncio.Queue) -> AsyncIterator[RequestOutput]:
        finished = False
        try:
            while True:
                item = await q.get()
                if isinstance(item, BaseException):
                    finished = True
                    raise item
                yield item
                if item.finished:
                    finished = True
                    return
        finally:
            # client disconnected / generator closed early -> abort in the engine
            self._release(request_id, abort=not finished)

    def abort(self, request_id: str) -> None:
        self._cmds.put(("abort", request_id))
        self._wake.set()

    def call_in_engine_thread(self, fn) -> "concurrent.futures.Future":
        """Run ``fn()`` on the engine thread between steps (profiler start/stop, stats)."""
        fut: concurrent.futures.Future = concurrent.futures.Future()
        self._cmds.put(("call", fn, fut))
        self._wake.set()
        return fut

    async def start(self) -> None:
        """Interface parity with ``MPEngineClient`` (the loop thread is already running)."""

    async def wait_ready(self, timeout=None) -> None:
        self.check_health()

    async def run_op(self, op: str):
        """Named engine operation between steps: profile_start/stop, sync, stats."""
        from .core_proc import _run_op
        return await asyncio.wrap_future(self.call_in_engine_thread(lambda: _run_op(self.engine, op)))

    def shutdown(self) -> None:
        self._stop = True
        self._wake.set()
        self._thread.join(timeout=30)
        self.engine.shutdown()

    # ------------------------------------------------------------------ loop
    def _deliver(self, rid: str, item) -> None:
        q, loop = self._streams.get(rid), self._loops.get(rid)
        if q is not None and loop is not None:
            loop.call_soon_threadsafe(q.put_nowait, item)

    def _drain_cmds(self) -> None:
        while True:
            try:
                cmd = self._cmds.get_nowait()
            except queue.Empty:
                return
            if cmd[0] == "add":
                _, rid, prompt, params, ids, arrival, prio, mm = cmd
                try:
                    self.engine.add_request(rid, prompt, params, ids, arrival_time=arrival,
                                            priority=prio, multi_modal_data=mm)
                    if self.log_requests:
                        logger.info("request %s added", rid)
                except Exception as e:   # noqa: BLE001 - validation errors go to the client
                    self._deliver(rid, e)
            elif cmd[0] == "call":
                _, fn, fut = cmd
                try:
                    fut.set_result(fn())
                except Exception as e:   # noqa: BLE001 - returned to the caller
                    fut.set_exception(e)
            else:
                self.engine.abort_request(cmd[1])

    def _run(self) -> None:
        steps = 0
        crash_after = delay = None
        if self._fault.startswith("crash_after:"):
            crash_after = int(self._fault.split(":")[1])
        elif self._fault.startswith("delay_step:"):
            delay = float(self._fault.split(":")[1])
        try:
            while not self._stop:
                self._drain_cmds()
                if not self.engine.has_unfinished_requests():
                    self._wake.wait(0.05)
                    self._wake.clear()
                    continue
                t0 = time.time()
                self.last_step_start = t0
                if delay:
                    time.sleep(delay)
                outs = self.engine.step()
                self.last_step_start = None
                steps += 1
                if crash_after is not None and steps >= crash_after:
                    raise RuntimeError("EIA_FAULT_INJECT crash")
                if self.metrics is not None:
                    self.metrics.observe_step(self.engine, time.time() - t0)
                for o in outs:
                    if o.finished and self.metrics is not None:
                        self.metrics.observe_finished(o)
                    self._deliver(o.request_id, o)
        except BaseException as e:   # noqa: BLE001
            logger.exception("engine loop died")
            self.dead = e
            if self.metrics is not None:
                self.metrics.set_healthy(False)
            err = EngineDeadError(f"engine loop died: {e!r}")
            for rid in list(self._streams):
                self._deliver(rid, err)
