"""Synchronous LLM engine: requests in, incremental RequestOutputs out.

One ``step()`` = schedule -> execute on the GPU(s) -> append tokens -> stop
checks -> detokenise.  The OpenAI server drives it from a background thread
(engine/async_engine.py); ``generate()`` is the offline helper used by tests,
``bench.py`` and the ``LLM`` class.
"""

from __future__ import annotations

import dataclasses
import logging
import random
import time
from typing import Dict, Iterable, List, Optional, Sequence as Seq, Union

from ..config import EngineConfig
from ..tokenizer import get_tokenizer
from .detokenizer import Detokenizer
from .sampling_params import SamplingParams
from .scheduler import Scheduler, SchedulerOutput
from .sequence import FINISH_REASON, SeqStatus, Sequence

logger = logging.getLogger(__name__)


@dataclasses.dataclass(slots=True)
class CompletionOutput:
    index: int
    text: str
    token_ids: List[int]
    cumulative_logprob: Optional[float]
    logprobs: Optional[List[Dict[int, float]]]
    finish_reason: Optional[str] = None
    stop_reason: Union[int, str, None] = None
    new_text: str = ""
    new_token_ids: List[int] = dataclasses.field(default_factory=list)
    new_logprobs: Optional[List[Dict[int, float]]] = None

    def finished(self) -> bool:
        return self.finish_reason is not None


@dataclasses.dataclass(slots=True)
class RequestMetrics:
    arrival_time: float
    first_scheduled_time: Optional[float] = None
    first_token_time: Optional[float] = None
    last_token_time: Optional[float] = None
    finished_time: Optional[float] = None

    @property
    def ttft(self) -> Optional[float]:
        return None if self.first_token_time is None else self.first_token_time - self.arrival_time


@dataclasses.dataclass(slots=True)
class RequestOutput:
    request_id: str
    prompt: Optional[str]
    prompt_token_ids: List[int]
    outputs: List[CompletionOutput]
    finished: bool
    metrics: RequestMetrics
    num_cached_tokens: int = 0
    prompt_logprobs: Optional[list] = None


class _Request:
    __slots__ = ("request_id", "prompt", "prompt_token_ids", "params", "seqs", "arrival_time",
                 "n", "finished_emitted", "beam")

    def __init__(self, request_id, prompt, prompt_token_ids, params, seqs, arrival_time):
        self.request_id = request_id
        self.prompt = prompt
        self.prompt_token_ids = prompt_token_ids
        self.params = params
        self.seqs = seqs
        self.arrival_time = arrival_time
        self.n = params.n
        self.finished_emitted = False
        self.beam = None


@dataclasses.dataclass
class EngineStats:
    num_prompt_tokens: int = 0          # prompt tokens computed (excl. prefix-cache hits)
    num_generation_tokens: int = 0
    num_steps: int = 0
    num_preemptions: int = 0
    step_time_s: float = 0.0
    # overlapped-scheduling decisions (LLMEngine.step): launched ahead of the previous step's
    # token read-back vs run synchronously because a row needed host-side token processing
    num_overlapped_steps: int = 0
    num_sync_steps: int = 0


class LLMEngine:
    def __init__(self, cfg: EngineConfig, tokenizer=None, executor=None):
        self.cfg = cfg
        if executor is None:
            from .executor import make_executor
            executor = make_executor(cfg)
        self.executor = executor
        self.num_blocks = executor.num_blocks
        self.scheduler = Scheduler(cfg.scheduler, cfg.cache, self.num_blocks)
        # K14 swap space (GPU engines, every TP/PP rank; executor.swap_enabled)
        alloc = getattr(executor, "allocate_swap", None)
        if alloc is not None and cfg.cache.swap_space_gb > 0:
            from .swap import SwapSpace
            n = alloc(cfg.cache.swap_space_gb)
            if n > 0:
                self.scheduler.swap = SwapSpace(n)
        m = cfg.model
        self.tokenizer = tokenizer or get_tokenizer(
            cfg.tokenizer or cfg.model_path, m.vocab_size, m.eos_token_id, m.bos_token_id,
            cfg.trust_remote_code, allow_byte_fallback=not cfg.strict_tokenizer)
        eos = m.eos_token_id
        eos_ids = set(eos if isinstance(eos, list) else ([eos] if eos is not None else []))
        tok_eos = getattr(self.tokenizer, "eos_token_id", None)
        if tok_eos is not None:
            eos_ids.add(tok_eos)
        self.eos_ids = {e for e in eos_ids if e is not None and e < m.vocab_size}
        self.detok = Detokenizer(self.tokenizer)
        self.requests: Dict[str, _Request] = {}
        self.stats = EngineStats()
        self.finished_log: List[RequestOutput] = []      # consumed by the metrics exporter
        self.served_model_name = cfg.served_model_name or m.name or "model"
        self._step_listeners = []
        from ..utils.profiling import StepProfiler, invariants_enabled
        self.profiler = StepProfiler()
        self._check_invariants = invariants_enabled()
        # Overlapped scheduling (the reference's VLLM_DELAYED_SAMPLING knob,
        # core/helm-charts/vllm/gaudi-values.yaml:54): step k+1 is scheduled and launched
        # while step k's sampled tokens are still on the GPU; its input ids are read there.
        self._overlap = bool(cfg.scheduler.delayed_sampling) and \
            getattr(executor, "supports_overlap", False)
        self._pending = None        # StepHandle of the launched, not yet processed step
        self.phase_times: Dict[str, float] = {}   # host seconds per step phase (overlap path)
        # Servers consume only the per-step deltas until a request finishes: with
        # ``delta_outputs`` the full text / token list / logprobs of a request are materialised
        # once, in its final RequestOutput, instead of being copied every step (O(n^2)).
        self.delta_outputs = False

    # ------------------------------------------------------------------ requests
    def add_request(self, request_id: str, prompt: Optional[str] = None,
                    params: Optional[SamplingParams] = None,
                    prompt_token_ids: Optional[List[int]] = None,
                    arrival_time: Optional[float] = None, priority: int = 0,
                    multi_modal_data: Optional[dict] = None) -> None:
        if request_id in self.requests:
            raise ValueError(f"duplicate request id {request_id}")
        params = params or SamplingParams()
        if prompt_token_ids is None:
            if prompt is None:
                raise ValueError("prompt or prompt_token_ids required")
            prompt_token_ids = self.tokenizer.encode(prompt)
        if not prompt_token_ids:
            raise ValueError("empty prompt")
        maxlen = self.cfg.scheduler.max_model_len
        if len(prompt_token_ids) >= maxlen:
            raise ValueError(f"prompt has {len(prompt_token_ids)} tokens; max_model_len is {maxlen}")
        vocab = self.cfg.model.vocab_size
        if max(prompt_token_ids) >= vocab or min(prompt_token_ids) < 0:
            raise ValueError("prompt token id out of vocabulary range")
        if params.max_tokens is None:
            params = params.clone(max_tokens=maxlen - len(prompt_token_ids))
        params.eos_ids = sorted(self.eos_ids)
        if params.best_of > params.n and params.logprobs is None:
            params = params.clone(logprobs=0)
            params.eos_ids = sorted(self.eos_ids)
        arrival = arrival_time if arrival_time is not None else time.time()
        if params.use_beam_search:
            self._add_beam_request(request_id, prompt, list(prompt_token_ids), params, arrival,
                                   priority)
            return
        mm = self._encode_images(multi_modal_data, prompt_token_ids) if multi_modal_data else None
        seqs = []
        for i in range(params.best_of):
            seed = (params.seed + i) if params.seed is not None else random.getrandbits(63)
            s = Sequence(request_id, prompt_token_ids, params, index=i, arrival_time=arrival,
                         seed=seed, priority=priority)
            if (params.guided_choice or params.guided_regex or params.guided_json is not None
                    or params.guided_grammar):
                from .guided import make_guided_state
                s.guided_state = make_guided_state(params, self.tokenizer, vocab)
            if mm is not None:
                s.mm_embeds, s.mm_positions, s.cache_salt = mm
            seqs.append(s)
            self.scheduler.add(s)
        self.requests[request_id] = _Request(request_id, prompt, list(prompt_token_ids), params,
                                             seqs, arrival)

    def _add_beam_request(self, request_id, prompt, prompt_ids, params, arrival, priority):
        """Beam search: one sequence to start with (the prompt is prefilled once); it reports
        the top-2W log-probs of every step to its BeamGroup (engine/beam_search.py)."""
        from .beam_search import BeamGroup
        width = max(params.best_of, params.n)
        group = BeamGroup(request_id, len(prompt_ids), width, params.n, params.length_penalty,
                          params.early_stopping, params.eos_ids, params.stop_token_ids,
                          params.ignore_eos, params.max_tokens, self.cfg.scheduler.max_model_len)
        bparams = params.clone(n=1, best_of=1, temperature=0.0, logprobs=2 * width)
        bparams.eos_ids = params.eos_ids
        seq = Sequence(request_id, prompt_ids, bparams, index=0, arrival_time=arrival, seed=0,
                       priority=priority)
        seq.beam = group
        group.beams.append(seq)
        self.scheduler.add(seq)
        r = _Request(request_id, prompt, prompt_ids, params, [seq], arrival)
        r.beam = group
        self.requests[request_id] = r

    def _beam_steps(self, groups, touched: Dict[str, "_Request"]) -> None:
        """Advance the beam groups that reported this step (see BeamGroup.advance)."""
        from .beam_search import fork_sequence
        bm = self.scheduler.bm
        copies = []
        for g in groups:
            r = self.requests.get(g.request_id)
            if r is None:            # aborted meanwhile
                g.take_partial()
                continue
            if not g.ready():
                for s in g.take_partial():
                    s.num_computed_tokens -= 1   # recompute its logits with its siblings
                continue
            appends, forks, dropped = g.advance()
            now = time.time()
            for parent, tok, lp in forks:
                if bm.num_free_blocks() < 2:
                    continue                   # no room to copy-on-write: drop the candidate
                child = fork_sequence(parent)
                bm.native.fork(parent.seq_id, child.seq_id)
                bm._committed[child.seq_id] = bm._committed.get(parent.seq_id, 0)
                if parent.num_computed_tokens % bm.block_size:
                    src, dst = bm.native.cow_last(child.seq_id)
                    if src >= 0:
                        copies.append((src, dst))
                self._beam_append(child, tok, lp, now)
                self.scheduler.running.append(child)
                g.beams.append(child)
                r.seqs.append(child)
            for seq, tok, lp in appends:
                self._beam_append(seq, tok, lp, now)
            for seq in dropped:
                self.scheduler.finish(seq, SeqStatus.FINISHED_ABORTED)
                g.beams.remove(seq)
            if g.done:
                touched[g.request_id] = r
        if copies:
            self.executor.copy_blocks(copies)

    @staticmethod
    def _beam_append(seq: Sequence, tok: int, lp: float, now: float) -> None:
        seq.output_token_ids.append(tok)
        seq.cumulative_logprob += lp
        if seq.first_token_time is None:
            seq.first_token_time = now
        seq.last_token_time = now

    def _emit_beam(self, r: "_Request") -> RequestOutput:
        g = r.beam
        comps = []
        for i, h in enumerate(g.results()):
            text = self.tokenizer.decode(h.tokens,
                                         skip_special_tokens=r.params.skip_special_tokens)
            comps.append(CompletionOutput(index=i, text=text, token_ids=list(h.tokens),
                                          cumulative_logprob=h.cum_logprob, logprobs=None,
                                          finish_reason=h.finish_reason,
                                          stop_reason=h.stop_reason, new_text=text,
                                          new_token_ids=list(h.tokens)))
        s0 = r.seqs[0]
        now = time.time()
        metrics = RequestMetrics(r.arrival_time, s0.first_scheduled_time,
                                 min((s.first_token_time for s in r.seqs if s.first_token_time),
                                     default=None), now, now)
        return RequestOutput(r.request_id, r.prompt, r.prompt_token_ids, comps, True, metrics,
                             s0.num_cached_tokens)

    def abort_request(self, request_id: Union[str, Iterable[str]]) -> None:
        ids = [request_id] if isinstance(request_id, str) else list(request_id)
        for rid in ids:
            self.scheduler.abort_request(rid)
            self.requests.pop(rid, None)

    def has_unfinished_requests(self) -> bool:
        return self.scheduler.num_unfinished() > 0 or self._pending is not None

    def num_unfinished_requests(self) -> int:
        return len(self.requests)

    # ------------------------------------------------------------------ step
    @staticmethod
    def _needs_host_tokens(seq: Sequence) -> bool:
        from .sequence import needs_host_processing
        return needs_host_processing(seq)

    def step(self) -> List[RequestOutput]:
        if not self._overlap:
            return self._step_sync()
        t0 = time.time()
        sched = self.scheduler.schedule()
        self._apply_swaps(sched)
        touched: Dict[str, _Request] = {}
        for s in self.scheduler.finished_since_last:
            r = self.requests.get(s.request_id)
            if r:
                touched[r.request_id] = r
        self.scheduler.finished_since_last.clear()
        deltas: Dict[int, tuple] = {}
        prev, self._pending = self._pending, None
        if sched.empty:
            if prev is not None:
                self._process(prev, touched, deltas)
            return self._emit(touched, deltas)
        pt = self.phase_times
        t1 = time.time()
        sample_items = sched.decodes + [p for p in sched.prefills if p.samples]
        overlap = not any(self._needs_host_tokens(it.seq) for it in sample_items)
        if overlap:
            self.stats.num_overlapped_steps += 1
        else:
            self.stats.num_sync_steps += 1
        handle = self.profiler.step(
            lambda: self.executor.launch(self.scheduler.bm, sched, overlap))
        t2 = time.time()
        for it in sample_items:
            it.seq.num_pending += 1
        if prev is not None:
            self._process(prev, touched, deltas)    # the GPU is busy with `handle` meanwhile
        t3 = time.time()
        self.scheduler.update_after_step(sched)
        if self._check_invariants:
            from ..utils.profiling import check_engine_invariants
            check_engine_invariants(self)
        self.stats.num_steps += 1
        self.stats.num_preemptions = self.scheduler.num_preemptions
        self.stats.num_prompt_tokens += sum(it.num_tokens for it in sched.prefills)
        if overlap:
            self._pending = handle
        else:
            self._process(handle, touched, deltas)
        t4 = time.time()
        outs = self._emit(touched, deltas)
        t5 = time.time()
        for k, v in (("schedule", t1 - t0), ("launch", t2 - t1), ("process", t3 - t2),
                     ("update", t4 - t3), ("emit", t5 - t4)):
            pt[k] = pt.get(k, 0.0) + v
        self.stats.step_time_s += t5 - t0
        return outs

    def _process(self, handle, touched: Dict[str, "_Request"], deltas: Dict[int, tuple]) -> None:
        """Apply a launched step's sampled tokens: append, detokenise, stop checks."""
        tw = time.time()
        res = handle.result()
        now = time.time()
        self.phase_times["wait"] = self.phase_times.get("wait", 0.0) + now - tw
        beams = set()
        for r, it in enumerate(handle.items):
            seq = it.seq
            if seq.num_pending:
                seq.num_pending -= 1
            if seq.finished:
                continue
            tok = res.tokens[r]
            lp = res.logprobs[r] if res.logprobs is not None else None
            if seq.beam is not None:
                seq.beam.report(seq, lp)
                beams.add(seq.beam)
                self.stats.num_generation_tokens += 1
                continue
            self._append_token(seq, tok, lp, now)
            before = len(seq.output_text)
            new_text = self.detok.step(seq)
            self._check_stop(seq, tok, new_text)
            new_text = seq.output_text[before:]
            d = deltas.get(seq.seq_id)
            if d is None:
                deltas[seq.seq_id] = (new_text, [tok], [lp] if lp is not None else None)
            else:   # two tokens of one sequence surfaced in one step() call
                deltas[seq.seq_id] = (d[0] + new_text, d[1] + [tok],
                                      (d[2] or []) + [lp] if lp is not None else d[2])
            touched[seq.request_id] = self.requests[seq.request_id]
            self.stats.num_generation_tokens += 1
        if beams:
            self._beam_steps(beams, touched)

    def _step_sync(self) -> List[RequestOutput]:
        t0 = time.time()
        sched = self.scheduler.schedule()
        self._apply_swaps(sched)
        touched: Dict[str, _Request] = {}
        for s in self.scheduler.finished_since_last:
            r = self.requests.get(s.request_id)
            if r:
                touched[r.request_id] = r
        self.scheduler.finished_since_last.clear()
        if sched.empty:
            return self._emit(touched, {})
        res = self.profiler.step(lambda: self.executor.execute(self.scheduler.bm, sched))
        self.scheduler.update_after_step(sched)
        if self._check_invariants:
            from ..utils.profiling import check_engine_invariants
            check_engine_invariants(self)
        now = time.time()
        self.stats.num_steps += 1
        self.stats.num_preemptions = self.scheduler.num_preemptions
        self.stats.num_prompt_tokens += sum(it.num_tokens for it in sched.prefills) + sum(
            it.num_tokens for it in sched.decodes if it.seq.is_prefill)
        deltas: Dict[int, tuple] = {}
        sample_items = sched.decodes + [p for p in sched.prefills if p.samples]
        beams = set()
        for r, it in enumerate(sample_items):
            seq = it.seq
            if seq.finished:
                continue
            tok = res.tokens[r]
            lp = res.logprobs[r] if res.logprobs is not None else None
            if seq.beam is not None:
                seq.beam.report(seq, lp)
                beams.add(seq.beam)
                self.stats.num_generation_tokens += 1
                continue
            self._append_token(seq, tok, lp, now)
            before = len(seq.output_text)
            new_text = self.detok.step(seq)
            self._check_stop(seq, tok, new_text)
            new_text = seq.output_text[before:]
            deltas[seq.seq_id] = (new_text, [tok], [lp] if lp is not None else None)
            touched[seq.request_id] = self.requests[seq.request_id]
            self.stats.num_generation_tokens += 1
        if beams:
            self._beam_steps(beams, touched)
        self.stats.step_time_s += time.time() - t0
        return self._emit(touched, deltas)

    def _append_token(self, seq: Sequence, tok: int, lp, now: float) -> None:
        seq.output_token_ids.append(tok)
        if lp is not None:
            seq.output_logprobs.append(lp)
            seq.cumulative_logprob += lp.get(tok, 0.0)
        if seq.first_token_time is None:
            seq.first_token_time = now
        seq.last_token_time = now

    def _check_stop(self, seq: Sequence, tok: int, new_text: str) -> None:
        p = seq.params
        n_out = len(seq.output_token_ids)
        status = None
        if n_out >= p.min_tokens:
            if not p.ignore_eos and tok in self.eos_ids:
                status = SeqStatus.FINISHED_STOPPED
            elif tok in p.stop_token_ids:
                status = SeqStatus.FINISHED_STOPPED
                seq.stop_reason = tok
            else:
                hit = self.detok.check_stop_strings(seq, new_text)
                if hit is not None:
                    status = SeqStatus.FINISHED_STOPPED
                    seq.stop_reason = hit[0]
        if status is None and (n_out >= p.max_tokens or
                               seq.num_real_tokens >= self.cfg.scheduler.max_model_len):
            status = SeqStatus.FINISHED_LENGTH
        if status is None and seq.guided_state is not None:
            seq.guided_state.advance(tok)
            if seq.guided_state.is_done():
                status = SeqStatus.FINISHED_STOPPED
        if status is not None:
            self.scheduler.finish(seq, status)

    def _emit(self, touched: Dict[str, _Request], deltas: Dict[int, tuple]) -> List[RequestOutput]:
        outs = []
        for rid, r in touched.items():
            if r.beam is not None:
                if r.beam.done and rid in self.requests:
                    ro = self._emit_beam(r)
                    outs.append(ro)
                    self.requests.pop(rid, None)
                    self.finished_log.append(ro)
                continue
            finished = all(s.finished for s in r.seqs)
            seqs = r.seqs
            if finished and r.params.best_of > r.params.n:
                seqs = sorted(seqs, key=lambda s: s.cumulative_logprob, reverse=True)[:r.params.n]
            elif r.params.best_of > r.params.n:
                continue     # best_of is only returned at the end
            full = finished or not self.delta_outputs
            want_lp = full and r.params.logprobs is not None
            comps = []
            for i, s in enumerate(seqs):
                d = deltas.get(s.seq_id, ("", [], None))
                comps.append(CompletionOutput(
                    index=i if r.params.best_of > r.params.n else s.index,
                    text=s.output_text if full else "",
                    token_ids=list(s.output_token_ids) if full else [],
                    cumulative_logprob=s.cumulative_logprob if want_lp else None,
                    logprobs=s.output_logprobs if want_lp else None,
                    finish_reason=FINISH_REASON.get(s.status), stop_reason=s.stop_reason,
                    new_text=d[0], new_token_ids=d[1], new_logprobs=d[2]))
            s0 = r.seqs[0]
            metrics = RequestMetrics(r.arrival_time, s0.first_scheduled_time,
                                     min((s.first_token_time for s in r.seqs if s.first_token_time),
                                         default=None),
                                     max((s.last_token_time for s in r.seqs if s.last_token_time),
                                         default=None),
                                     max((s.finish_time for s in r.seqs if s.finish_time), default=None)
                                     if finished else None)
            ro = RequestOutput(rid, r.prompt, r.prompt_token_ids, comps, finished, metrics,
                               s0.num_cached_tokens)
            outs.append(ro)
            if finished:
                self.requests.pop(rid, None)
                self.finished_log.append(ro)
                if len(self.finished_log) > 10000:
                    del self.finished_log[:5000]
        return outs

    # ------------------------------------------------------------------ helpers
    def generate(self, prompts: Optional[Seq[str]] = None, params=None,
                 prompt_token_ids: Optional[Seq[List[int]]] = None,
                 multi_modal_data: Optional[Seq[Optional[dict]]] = None) -> List[RequestOutput]:
        n = len(prompts) if prompts is not None else len(prompt_token_ids)
        plist = params if isinstance(params, list) else [params or SamplingParams()] * n
        ids = []
        for i in range(n):
            rid = f"gen-{time.time_ns()}-{i}"
            self.add_request(rid, prompts[i] if prompts is not None else None, plist[i],
                             prompt_token_ids[i] if prompt_token_ids is not None else None,
                             multi_modal_data=multi_modal_data[i] if multi_modal_data else None)
            ids.append(rid)
        done: Dict[str, RequestOutput] = {}
        while len(done) < n:
            for o in self.step():
                if o.finished:
                    done[o.request_id] = o
        return [done[i] for i in ids]

    def kv_cache_usage(self) -> float:
        return self.scheduler.kv_usage()

    def _encode_images(self, mm: dict, prompt_token_ids: List[int]):
        """Vision tower at admission: -> (embeddings [n, hidden] on the device, prompt positions
        of the n image-placeholder tokens, prefix-cache salt from the image bytes)."""
        import hashlib

        import numpy as np
        import torch

        images = mm.get("image") or []
        if not isinstance(images, (list, tuple)):
            images = [images]
        if not images:
            return None
        enc = getattr(self.executor, "encode_images", None)
        model = getattr(getattr(self.executor, "runner", None), "model", None)
        tower = getattr(model, "vision", None)
        if enc is None or tower is None:
            raise ValueError("this deployment does not accept image inputs (needs a vision "
                             "checkpoint served with tensor_parallel_size=1)")
        from ..models.llama4_vision import preprocess
        h = hashlib.blake2b(digest_size=8)
        embeds = []
        for img in images:
            if isinstance(img, torch.Tensor):
                pv = img
                h.update(pv.float().numpy().tobytes())
            else:
                pv, _ = preprocess(img, tile=tower.image_size)
                h.update(img if isinstance(img, (bytes, bytearray)) else str(img).encode())
            embeds.append(enc(pv))
        emb = torch.cat(embeds)
        pos = np.flatnonzero(np.asarray(prompt_token_ids) == model.image_token_id).astype(np.int64)
        if len(pos) != emb.shape[0]:
            raise ValueError(f"prompt has {len(pos)} image placeholder tokens but the images "
                             f"produce {emb.shape[0]} embeddings")
        return emb, pos, int.from_bytes(h.digest(), "little") & ((1 << 63) - 1)

    def cpu_cache_usage(self) -> float:
        return self.scheduler.cpu_usage()

    def _apply_swaps(self, sched) -> None:
        """K14: victims' blocks out to host memory, returning sequences' blocks back in --
        on the step stream, before the step's kernels (out first: an in-swap may reuse a
        block an out-swap just released)."""
        for gpu, cpu in sched.swap_out:
            self.executor.swap_out(gpu, cpu)
        for cpu, gpu in sched.swap_in:
            self.executor.swap_in(cpu, gpu)

    def shutdown(self) -> None:
        ex = getattr(self.executor, "shutdown", None)
        if ex:
            ex()
