"""Engine-core process: the scheduler + GPU step loop in its own OS process.

Why a process and not a thread: the OpenAI front-end parses requests, tokenises
prompts and frames one SSE chunk per generated token per stream (65 users at
~5 ms/step = 13k chunks/s for the reference's chatbot sizing row,
third_party/IBM/docs/sizing-guide.md:56).  In one process that Python work
holds the GIL the step loop needs to plan and launch the next HIP-graph replay
and the GPU idles -- measured on MI355X: 9.55k tok/s through the endpoint vs
11.56k engine-level, TPOT 5.78 vs 4.92 ms (profiles/serving_r2_base.md).  The
split mirrors what the reference's vLLM container does internally (API server
<-> engine core), re-done here with the runtime's own IPC:

  API process (no GPU)                      engine-core process (owns the GPU(s))
  --------------------                      -------------------------------------
  FastAPI / SSE, tokenizer, chat templates  LLMEngine: scheduler, KV manager,
  MPEngineClient ----- socketpair --------> executor (TP workers are *its*
     add / abort / op     length-prefixed      children), detokeniser, stop checks
  <------ one frame per engine step -------  deltas of every touched request +
     (deltas + metrics snapshot)                the vllm:* metrics snapshot

One frame per step (not per token) keeps IPC at ~200 syscalls/s; the API process
fans the deltas out to per-request asyncio queues on its own loop (no
cross-thread wake-ups).  The core sends full text/token lists only in a
request's final output (``LLMEngine.delta_outputs``).

Failure semantics: the API's ``/health`` is 503 until the core
reports ``ready`` (weights loaded, KV cache sized, HIP graphs captured), 500
once the core died (EOF on the socket / init error) or when a step exceeds
``VLLM_ENGINE_ITERATION_TIMEOUT_S`` while requests are in flight; the core
exits when the API process goes away (EOF), taking its TP workers with it.
"""

from __future__ import annotations

import argparse
import asyncio
import itertools
import logging
import os
import pickle
import select
import socket
import struct
import subprocess
import sys
import time
from typing import Dict, Optional

from .async_engine import EngineDeadError, SubmittedStream
from .llm_engine import CompletionOutput, RequestMetrics, RequestOutput

logger = logging.getLogger(__name__)

_HDR = struct.Struct("<I")


def encode_frame(obj) -> bytes:
    data = pickle.dumps(obj, protocol=5)
    return _HDR.pack(len(data)) + data


class FrameReader:
    """Length-prefixed pickle frames from a blocking socket, read without blocking the step
    loop: ``poll(timeout)`` returns every complete frame that arrived (possibly none)."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf = bytearray()
        self.pending: list = []          # frames read ahead by read_one()

    def poll(self, timeout: Optional[float]) -> list:
        if self.pending:
            out, self.pending = self.pending, []
            return out + self.poll(0)
        r, _, _ = select.select([self.sock], [], [], timeout)
        while r:
            chunk = self.sock.recv(1 << 20)
            if not chunk:
                raise EOFError("peer closed the engine socket")
            self.buf += chunk
            r, _, _ = select.select([self.sock], [], [], 0)
        out = []
        buf = self.buf
        off = 0
        while len(buf) - off >= 4:
            (n,) = _HDR.unpack_from(buf, off)
            if len(buf) - off - 4 < n:
                break
            out.append(pickle.loads(memoryview(buf)[off + 4:off + 4 + n]))
            off += 4 + n
        if off:
            del buf[:off]
        return out

    def read_one(self, timeout: Optional[float] = None):
        t0 = time.time()
        while True:
            frames = self.poll(0.5)
            if frames:
                self.pending = frames[1:]
                return frames[0]
            if timeout is not None and time.time() - t0 > timeout:
                raise TimeoutError("no init frame from the API process")


# --------------------------------------------------------------------------- engine side

def _pack(o: RequestOutput) -> tuple:
    fin = o.finished
    comps = [(c.index, c.new_text, c.new_token_ids, c.new_logprobs, c.finish_reason,
              c.stop_reason) + ((c.text, c.token_ids, c.logprobs, c.cumulative_logprob)
                                if fin else ()) for c in o.outputs]
    m = o.metrics
    met = (m.arrival_time, m.first_scheduled_time, m.first_token_time, m.last_token_time,
           m.finished_time) if fin else None
    return (o.request_id, fin, o.num_cached_tokens, met, comps)


def _run_op(engine, op: str):
    if op == "profile_start":
        return engine.profiler.start()
    if op == "profile_stop":
        return engine.profiler.stop()
    if op == "sync":
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        return True
    if op == "dist":
        return _dist_info(engine)
    if op == "stats":
        st = engine.stats
        return {"num_steps": st.num_steps, "num_generation_tokens": st.num_generation_tokens,
                "num_prompt_tokens": st.num_prompt_tokens, "num_blocks": engine.num_blocks,
                "step_time_s": st.step_time_s,
                "num_overlapped_steps": st.num_overlapped_steps,
                "num_sync_steps": st.num_sync_steps,
                "phase_times": dict(engine.phase_times),
                "loop_times": dict(getattr(engine, "loop_times", {})),
                "dist": _dist_info(engine)}
    raise ValueError(f"unknown engine op {op!r}")


def _dist_info(engine) -> list:
    """Per-rank process-group / custom all-reduce description of this replica (executor)."""
    fn = getattr(getattr(engine, "executor", None), "dist_info", None)
    try:
        return fn() if fn is not None else []
    except Exception as e:   # noqa: BLE001 - a description must never fail the stats op
        return [{"error": repr(e)}]


# Intake coalescing: an idle engine that receives a request keeps reading for as long as more
# requests keep arriving (gaps <= INTAKE_GAP_S, INTAKE_MAX_S in all) before it schedules, so a
# burst of concurrent requests (N users starting together) is prefilled in one step instead of
# a small step for the first few arrivals that everyone else then queues behind.  A lone
# request pays at most one INTAKE_GAP_S.  EIA_INTAKE_GAP_MS=0 disables it.
INTAKE_GAP_S = float(os.environ.get("EIA_INTAKE_GAP_MS", "2")) / 1000.0
INTAKE_MAX_S = float(os.environ.get("EIA_INTAKE_MAX_MS", "20")) / 1000.0


def intake(reader, busy: bool, gap: float = None, cap: float = None) -> list:
    """Frames for this loop iteration: whatever is pending (blocking up to 0.5 s when idle),
    extended by the coalescing window above when the idle engine just received requests."""
    gap = INTAKE_GAP_S if gap is None else gap
    cap = INTAKE_MAX_S if cap is None else cap
    msgs = reader.poll(0 if busy else 0.5)
    if busy or gap <= 0 or not any(m[0] == "add" for m in msgs):
        return msgs
    t_end = time.time() + cap
    while True:
        left = t_end - time.time()
        if left <= 0:
            return msgs
        more = reader.poll(min(gap, left))
        if not more:
            return msgs
        msgs += more


def core_main(fd: int) -> int:
    """Entry point of the engine-core process (``python -m ...core_proc --fd N``)."""
    import signal

    def _term(signum, frame):       # graceful: unwind through engine.shutdown() (TP workers)
        raise SystemExit(0)

    signal.signal(signal.SIGTERM, _term)
    sock = socket.socket(fileno=fd)
    sock.setblocking(True)
    reader = FrameReader(sock)
    kind, cfg, opts = reader.read_one(timeout=300)
    assert kind == "init", kind
    logging.basicConfig(level=os.environ.get("EIA_LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(levelname)s [engine-core] %(name)s: %(message)s")
    from ..metrics import EngineMetrics
    from .llm_engine import LLMEngine

    try:
        if cfg.device == "cuda":
            import torch

            from ..utils.numa import pin_to_device
            if torch.cuda.device_count() > 0:   # step loop + staging next to GPU 0's socket
                pin_to_device(0)
        engine = LLMEngine(cfg)
        engine.delta_outputs = True
    except BaseException as e:   # noqa: BLE001 - reported to the API process, then exit
        logger.exception("engine init failed")
        sock.sendall(encode_frame(("dead", f"engine init failed: {e!r}")))
        return 1
    from ..utils.gc_tuning import tune_after_startup
    tune_after_startup()
    from ..parallel import custom_allreduce as _car
    ready = {"num_blocks": engine.num_blocks, "pid": os.getpid()}
    if cfg.parallel.tensor_parallel_size > 1:
        ready["custom_allreduce"] = {k: v for k, v in _car.STATUS.items() if k != "tuning"}
    sock.sendall(encode_frame(("ready", ready)))
    log_requests = bool(opts.get("log_requests"))
    fault = opts.get("fault", "")
    crash_after = int(fault.split(":")[1]) if fault.startswith("crash_after:") else None
    delay = float(fault.split(":")[1]) if fault.startswith("delay_step:") else None
    steps = 0
    rc = 0
    # host seconds per loop phase (engine.step() has its own breakdown in phase_times): what the
    # core spends outside the step -- request intake and the per-step output frame
    lt = engine.loop_times = {"intake": 0.0, "step": 0.0, "frame": 0.0, "send": 0.0}
    perf = time.perf_counter
    try:
        while True:
            busy = engine.has_unfinished_requests()
            ti = perf()
            msgs = intake(reader, busy)
            if busy:
                lt["intake"] += perf() - ti
            else:
                # an idle engine's burst: how long its requests took to reach the core after the
                # API process received them (first -> last arrival, first arrival -> schedule)
                arr = [m[5] for m in msgs if m[0] == "add"]
                if arr:
                    now = time.time()
                    lt["bursts"] = lt.get("bursts", 0) + 1
                    lt["burst_reqs"] = lt.get("burst_reqs", 0) + len(arr)
                    lt["burst_spread"] = lt.get("burst_spread", 0.0) + (max(arr) - min(arr))
                    lt["burst_wait"] = lt.get("burst_wait", 0.0) + (now - min(arr))
            for msg in msgs:
                k = msg[0]
                if k == "add":
                    _, rid, prompt, params, ids, arrival, prio = msg[:7]
                    mm = msg[7] if len(msg) > 7 else None
                    try:
                        engine.add_request(rid, prompt, params, ids, arrival_time=arrival,
                                           priority=prio, multi_modal_data=mm)
                        if log_requests:
                            logger.info("request %s added", rid)
                    except Exception as e:   # noqa: BLE001 - validation error -> the client
                        sock.sendall(encode_frame(("err", rid, e)))
                elif k == "abort":
                    engine.abort_request(msg[1])
                elif k == "op":
                    _, cid, op = msg
                    try:
                        res = ("opres", cid, True, _run_op(engine, op))
                    except Exception as e:   # noqa: BLE001 - returned to the caller
                        res = ("opres", cid, False, e)
                    sock.sendall(encode_frame(res))
                elif k == "shutdown":
                    return 0
            if not engine.has_unfinished_requests():
                continue
            t0 = time.time()
            t1 = perf()
            if delay:
                time.sleep(delay)
            outs = engine.step()
            t2 = perf()
            steps += 1
            if crash_after is not None and steps >= crash_after:
                raise RuntimeError("EIA_FAULT_INJECT crash")
            snap = EngineMetrics.engine_snapshot(engine, time.time() - t0)
            frame = encode_frame(("out", snap, [_pack(o) for o in outs]))
            t3 = perf()
            sock.sendall(frame)
            t4 = perf()
            lt["step"] += t2 - t1
            lt["frame"] += t3 - t2
            lt["send"] += t4 - t3
    except (EOFError, ConnectionError):
        logger.info("API process went away; engine core exiting")
    except SystemExit:
        logger.info("engine core terminated")
    except BaseException as e:   # noqa: BLE001
        logger.exception("engine loop died")
        rc = 1
        try:
            sock.sendall(encode_frame(("dead", f"engine loop died: {e!r}")))
        except OSError:
            pass
    finally:
        try:
            engine.shutdown()
        except Exception:   # noqa: BLE001
            logger.exception("engine shutdown failed")
    return rc


# --------------------------------------------------------------------------- API side

class _ReqState:
    __slots__ = ("queue", "prompt", "prompt_ids")

    def __init__(self, queue, prompt, prompt_ids):
        self.queue = queue
        self.prompt = prompt
        self.prompt_ids = prompt_ids


class MPEngineClient:
    """Asyncio client of an engine-core process; a drop-in for ``AsyncLLMEngine`` in the
    OpenAI server (``generate`` / ``abort`` / ``healthy`` / ``dead`` / ``run_op``).

    Construct it *before* anything in this process touches the GPU: the core is started
    with ``subprocess.Popen`` and the API process itself never initialises HIP."""

    def __init__(self, cfg, metrics=None, log_requests: bool = True, tokenizer=None,
                 env: Optional[dict] = None):
        from ..tokenizer import get_tokenizer

        self.cfg = cfg
        self.metrics = metrics
        m = cfg.model
        self.tokenizer = tokenizer or get_tokenizer(
            cfg.tokenizer or cfg.model_path, m.vocab_size, m.eos_token_id, m.bos_token_id,
            cfg.trust_remote_code, allow_byte_fallback=not cfg.strict_tokenizer)
        self.timeout_s = float(os.environ.get("VLLM_ENGINE_ITERATION_TIMEOUT_S",
                                              cfg.engine_iteration_timeout_s))
        self.dead: Optional[BaseException] = None
        self.ready = False
        self.info: dict = {}
        self._reqs: Dict[str, _ReqState] = {}
        self._ops: Dict[int, asyncio.Future] = {}
        self._op_ids = itertools.count()
        self._last_msg = time.time()
        self._writer = None
        self._reader_task = None
        self._starting: Optional[asyncio.Future] = None
        self._ready_evt: Optional[asyncio.Event] = None
        parent, child = socket.socketpair()
        self._sock = parent
        cmd = [sys.executable, "-m", "enterprise_inference_amd.engine.core_proc",
               "--fd", str(child.fileno())]
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        penv = dict(os.environ if env is None else env)
        penv["PYTHONPATH"] = root + os.pathsep + penv.get("PYTHONPATH", "")
        self.proc = subprocess.Popen(cmd, pass_fds=[child.fileno()], env=penv)
        child.close()
        parent.sendall(encode_frame(("init", cfg, {
            "log_requests": log_requests, "fault": os.environ.get("EIA_FAULT_INJECT", "")})))

    # ------------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        """Attach the socket to the running event loop (FastAPI startup hook; also called
        lazily by the first request when the app runs without lifespan events)."""
        if self._starting is None:
            self._starting = asyncio.get_running_loop().create_future()
            self._ready_evt = asyncio.Event()
            if self.ready or self.dead is not None:
                self._ready_evt.set()
            reader, writer = await asyncio.open_connection(sock=self._sock)
            self._writer = writer
            self._reader_task = asyncio.get_running_loop().create_task(self._read_loop(reader))
            self._starting.set_result(True)
        else:
            await self._starting

    async def wait_ready(self, timeout: Optional[float] = None) -> None:
        await asyncio.wait_for(self._ready_evt.wait(), timeout)
        if self.dead is not None:
            raise EngineDeadError(str(self.dead))

    def shutdown(self, timeout: float = 30.0) -> None:
        frame = encode_frame(("shutdown",))
        sent = False
        try:
            if self._writer is not None and not self._writer.is_closing():
                self._writer.write(frame)
                sent = True
        except Exception:   # noqa: BLE001 - loop already closed: fall back to the raw socket
            pass
        if not sent:
            try:
                self._sock.setblocking(True)
                self._sock.sendall(frame)
            except OSError:
                pass        # the core is already gone
        try:
            self.proc.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            self.proc.terminate()
            try:
                self.proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
        if self.metrics is not None:
            self.metrics.set_healthy(False)

    # ------------------------------------------------------------------ state
    @property
    def healthy(self) -> bool:
        if self.dead is not None or not self.ready:
            return False
        if self.proc.poll() is not None:
            return False
        return not self._reqs or (time.time() - self._last_msg) < self.timeout_s

    def check_health(self) -> None:
        if self.dead is not None:
            raise EngineDeadError(f"engine loop died: {self.dead}")
        if self.ready and not self.healthy:
            raise EngineDeadError("engine step exceeded VLLM_ENGINE_ITERATION_TIMEOUT_S")

    # ------------------------------------------------------------------ API
    def _send(self, obj) -> None:
        self._writer.write(encode_frame(obj))

    async def generate(self, request_id: str, prompt: Optional[str], params,
                       prompt_token_ids=None, priority: int = 0, multi_modal_data=None):
        self.check_health()
        if self._writer is None:
            await self.start()
        if not self.ready:
            await self.wait_ready()
        async for item in self.submit(request_id, prompt, params, prompt_token_ids, priority,
                                      multi_modal_data):
            yield item

    @property
    def can_submit(self) -> bool:
        return self._writer is not None and self.ready

    def submit(self, request_id: str, prompt: Optional[str], params, prompt_token_ids=None,
               priority: int = 0, multi_modal_data=None):
        """Hand the request to the core NOW (the "add" frame is written before this returns)
        and return the async iterator of its outputs.  ``generate`` only sends when its
        iterator is first advanced -- for a streaming response that is after the handler has
        returned and the response started, so a burst of concurrent requests reached the core
        spread over the event loop's interleaving of their handlers.  Needs ``can_submit``."""
        self.check_health()
        if prompt_token_ids is None:
            prompt_token_ids = self.tokenizer.encode(prompt)
        q: asyncio.Queue = asyncio.Queue()
        if not self._reqs:
            self._last_msg = time.time()       # idle gap is not a stuck step
        self._reqs[request_id] = _ReqState(q, prompt, list(prompt_token_ids))
        self._send(("add", request_id, prompt, params, prompt_token_ids, time.time(), priority,
                    multi_modal_data))
        return SubmittedStream(self._outputs(request_id, q),
                               lambda: self._release(request_id, abort=True))

    def _release(self, request_id: str, abort: bool) -> None:
        """Forget the request; abort it in the core if it was still open (idempotent: the
        output generator and the stream's finaliser may both call it)."""
        if self._reqs.pop(request_id, None) is not None and abort and self.dead is None:
            self.abort(request_id)

    async def _outputs(self, request_id: str, q: asyncio.Queue):
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
            # client disconnected / generator closed early -> abort in the core
            self._release(request_id, abort=not finished)

    def abort(self, request_id: str) -> None:
        if self._writer is not None and not self._writer.is_closing():
            self._send(("abort", request_id))

    async def run_op(self, op: str):
        """Run a named engine operation between steps (profile_start/stop, sync, stats)."""
        self.check_health()
        if self._writer is None:
            await self.start()
        await self.wait_ready()
        cid = next(self._op_ids)
        fut = asyncio.get_running_loop().create_future()
        self._ops[cid] = fut
        self._send(("op", cid, op))
        return await fut

    # ------------------------------------------------------------------ reader
    def _die(self, reason: str) -> None:
        if self.dead is None:
            self.dead = EngineDeadError(reason)
            logger.error("engine core: %s", reason)
        if self.metrics is not None:
            self.metrics.set_healthy(False)
        for st in self._reqs.values():
            st.queue.put_nowait(self.dead)
        for fut in self._ops.values():
            if not fut.done():
                fut.set_exception(self.dead)
        self._ops.clear()
        if self._ready_evt is not None:
            self._ready_evt.set()

    async def _read_loop(self, reader: asyncio.StreamReader) -> None:
        try:
            while True:
                hdr = await reader.readexactly(4)
                data = await reader.readexactly(_HDR.unpack(hdr)[0])
                self._last_msg = time.time()
                self._dispatch(pickle.loads(data))
        except (asyncio.IncompleteReadError, ConnectionError, OSError) as e:
            self._die(f"engine core exited (rc={self.proc.poll()}): {e!r}")
        except asyncio.CancelledError:
            raise
        except BaseException as e:   # noqa: BLE001
            logger.exception("engine client reader failed")
            self._die(f"engine client reader failed: {e!r}")

    def _dispatch(self, msg) -> None:
        kind = msg[0]
        if kind == "out":
            _, snap, outs = msg
            if self.metrics is not None:
                self.metrics.observe_stats(snap)
            reqs = self._reqs
            for rid, fin, ncached, met, comps in outs:
                st = reqs.get(rid)
                if st is None:
                    continue
                cos = []
                for c in comps:
                    if fin:
                        idx, ntext, nids, nlp, fr, sr, text, ids, lps, cum = c
                    else:
                        idx, ntext, nids, nlp, fr, sr = c
                        text, ids, lps, cum = "", [], None, None
                    cos.append(CompletionOutput(idx, text, ids, cum, lps, fr, sr, ntext, nids, nlp))
                metrics = RequestMetrics(*met) if met else RequestMetrics(0.0)
                ro = RequestOutput(rid, st.prompt, st.prompt_ids, cos, fin, metrics, ncached)
                st.queue.put_nowait(ro)
                if fin and self.metrics is not None:
                    self.metrics.observe_finished(ro)
        elif kind == "err":
            st = self._reqs.get(msg[1])
            if st is not None:
                st.queue.put_nowait(msg[2])
        elif kind == "opres":
            _, cid, ok, res = msg
            fut = self._ops.pop(cid, None)
            if fut is not None and not fut.done():
                if ok:
                    fut.set_result(res)
                else:
                    fut.set_exception(res)
        elif kind == "ready":
            self.ready = True
            self.info = msg[1]
            if self.metrics is not None:
                self.metrics.set_healthy(True)
                if "custom_allreduce" in self.info:
                    self.metrics.set_custom_allreduce(self.info["custom_allreduce"])
            logger.info("engine core ready: %s", self.info)
            self._ready_evt.set()
        elif kind == "dead":
            self._die(msg[1])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="engine-core process (started by the API server)")
    ap.add_argument("--fd", type=int, required=True)
    args = ap.parse_args(argv)
    out = os.environ.get("EIA_CORE_CPROFILE")     # host-side profile of the engine core
    if not out:
        return core_main(args.fd)
    import cProfile
    import pstats
    prof = cProfile.Profile()
    try:
        return prof.runcall(core_main, args.fd)
    finally:
        with open(out, "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(60)


if __name__ == "__main__":
    sys.exit(main())
