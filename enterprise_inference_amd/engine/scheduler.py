"""Continuous-batching scheduler with a per-step token budget.

Implements the knobs the reference passes to vLLM:
``--max-num-seqs``, ``--max-num-prefill-seqs``, ``--max-num-batched-tokens``,
``--enable_chunked_prefill`` (core/helm-charts/vllm/gaudi-values.yaml:160,
xeon-values.yaml:80-83).  Policy per step:
  1. running sequences first (decodes, then unfinished prefill chunks), growing
     their block tables; on KV exhaustion the most recently admitted running
     sequence is preempted (recompute mode) until the allocation fits;
  2. then waiting sequences FCFS with prefix-cache lookup, chunked to the
     remaining token budget when chunked prefill is enabled.
Batch layout handed to the runner: [decode tokens | prefill chunks].
"""

from __future__ import annotations

import collections
import dataclasses
import time
from typing import Deque, Dict, List, Optional

import numpy as np

from ..config import CacheConfig, SchedulerConfig
from .block_manager import BlockManager
from .sequence import Sequence, SeqStatus


@dataclasses.dataclass
class ScheduledSeq:
    seq: Sequence
    start: int
    num_tokens: int

    @property
    def samples(self) -> bool:
        return self.start + self.num_tokens >= self.seq.num_tokens


@dataclasses.dataclass
class SchedulerOutput:
    decodes: List[ScheduledSeq]
    prefills: List[ScheduledSeq]
    preempted: List[Sequence]
    num_batched_tokens: int

    @property
    def empty(self) -> bool:
        return not self.decodes and not self.prefills

    @property
    def all(self) -> List[ScheduledSeq]:
        return self.decodes + self.prefills


class Scheduler:
    def __init__(self, sched: SchedulerConfig, cache: CacheConfig, num_blocks: int,
                 block_manager: Optional[BlockManager] = None):
        self.cfg = sched
        self.cache_cfg = cache
        self.bm = block_manager or BlockManager(num_blocks, cache.block_size,
                                                cache.enable_prefix_caching)
        self.waiting: Deque[Sequence] = collections.deque()
        self.running: List[Sequence] = []
        self.num_preemptions = 0
        self.finished_since_last: List[Sequence] = []

    # ------------------------------------------------------------------ queue ops
    def add(self, seq: Sequence) -> None:
        seq.status = SeqStatus.WAITING
        self.waiting.append(seq)

    def num_unfinished(self) -> int:
        return len(self.waiting) + len(self.running)

    def finish(self, seq: Sequence, status: SeqStatus) -> None:
        if seq.finished:
            return
        seq.status = status
        seq.finish_time = time.time()
        if seq in self.running:
            self.running.remove(seq)
        else:
            try:
                self.waiting.remove(seq)
            except ValueError:
                pass
        self.bm.free(seq)

    def abort_request(self, request_id: str) -> List[Sequence]:
        out = [s for s in list(self.running) + list(self.waiting) if s.request_id == request_id]
        for s in out:
            self.finish(s, SeqStatus.FINISHED_ABORTED)
        return out

    # ------------------------------------------------------------------ scheduling
    def _preempt(self, seq: Sequence) -> None:
        self.running.remove(seq)
        self.bm.free(seq)
        seq.status = SeqStatus.PREEMPTED
        seq.num_computed_tokens = 0
        seq.num_preemptions += 1
        self.num_preemptions += 1
        self.waiting.appendleft(seq)

    def schedule(self) -> SchedulerOutput:
        budget = self.cfg.max_num_batched_tokens
        decodes: List[ScheduledSeq] = []
        prefills: List[ScheduledSeq] = []
        preempted: List[Sequence] = []
        scheduled_ids = set()

        # 1. running sequences (oldest first)
        i = 0
        while i < len(self.running) and budget > 0:
            seq = self.running[i]
            if seq.num_pending and (len(seq.output_token_ids) + seq.num_pending >= seq.params.max_tokens
                                    or seq.num_tokens >= self.cfg.max_model_len):
                i += 1        # its final token is in flight: nothing left to compute
                continue
            remaining = seq.num_tokens - seq.num_computed_tokens
            n = min(remaining, budget)
            if n < remaining and not self.cfg.enable_chunked_prefill and remaining > 1:
                i += 1
                continue
            while not self.bm.ensure(seq, seq.num_computed_tokens + n):
                victim = self.running[-1]
                self._preempt(victim)
                preempted.append(victim)
                if victim is seq:
                    break
            if seq.status == SeqStatus.PREEMPTED:
                continue          # seq itself was evicted; list shrank
            item = ScheduledSeq(seq, seq.num_computed_tokens, n)
            (decodes if remaining == 1 else prefills).append(item)
            scheduled_ids.add(seq.seq_id)
            budget -= n
            i += 1

        # 2. waiting sequences, FCFS
        n_prefill = len(prefills)
        while (self.waiting and budget > 0 and len(self.running) < self.cfg.max_num_seqs
               and n_prefill < self.cfg.max_num_prefill_seqs and not preempted):
            seq = self.waiting[0]
            if seq.num_tokens > self.cfg.max_model_len:
                self.waiting.popleft()
                seq.status = SeqStatus.FINISHED_LENGTH
                seq.finish_time = time.time()
                self.finished_since_last.append(seq)
                continue
            if not self.bm.has(seq):
                seq.num_computed_tokens = self.bm.allocate_prefix(seq)
                seq.num_cached_tokens = seq.num_computed_tokens
            remaining = seq.num_tokens - seq.num_computed_tokens
            if remaining > budget and not self.cfg.enable_chunked_prefill:
                break
            n = min(remaining, budget)
            if not self.bm.ensure(seq, seq.num_computed_tokens + n):
                break          # keep it (and its prefix blocks) at the head of the queue
            self.waiting.popleft()
            seq.status = SeqStatus.RUNNING
            if seq.first_scheduled_time is None:
                seq.first_scheduled_time = time.time()
            self.running.append(seq)
            item = ScheduledSeq(seq, seq.num_computed_tokens, n)
            (decodes if remaining == 1 else prefills).append(item)
            budget -= n
            n_prefill += remaining > 1

        total = sum(s.num_tokens for s in decodes) + sum(s.num_tokens for s in prefills)
        return SchedulerOutput(decodes, prefills, preempted, total)

    def update_after_step(self, out: SchedulerOutput) -> None:
        """Advance computed-token counters and register full blocks for prefix reuse."""
        for item in out.decodes + out.prefills:
            seq = item.seq
            if seq.finished:
                continue
            seq.num_computed_tokens = item.start + item.num_tokens
            self.bm.commit(seq)

    def kv_usage(self) -> float:
        return self.bm.usage()
