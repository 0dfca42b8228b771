"""Continuous-batching scheduler with a per-step token budget.

Implements the knobs the reference passes to vLLM:
``--max-num-seqs``, ``--max-num-prefill-seqs``, ``--max-num-batched-tokens``,
``--enable_chunked_prefill`` (core/helm-charts/vllm/gaudi-values.yaml:160,
xeon-values.yaml:80-83).  Policy per step:
  1. running sequences first (decodes, then unfinished prefill chunks), growing
     their block tables; on KV exhaustion the most recently admitted running
     sequence is preempted until the allocation fits -- swapped to pinned host memory
     when the swap space (K14, --swap-space) can hold its blocks, else recompute;
  2. swapped sequences come back first (FCFS) when their blocks fit again;
  3. then waiting sequences FCFS with prefix-cache lookup, chunked to the
     remaining token budget when chunked prefill is enabled.
Batch layout handed to the runner: [decode tokens | prefill chunks].
"""

from __future__ import annotations

import collections
import dataclasses
import time
from typing import Deque, Dict, List, Optional, Tuple

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
    # KV swap copies to run before this step's kernels: (device blocks, host blocks)
    swap_out: List[Tuple[List[int], List[int]]] = dataclasses.field(default_factory=list)
    swap_in: List[Tuple[List[int], List[int]]] = dataclasses.field(default_factory=list)

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
        self.swapped: Deque[Sequence] = collections.deque()
        self.swap = None                  # engine.swap.SwapSpace when --swap-space > 0
        self._swap_out: List[Tuple[List[int], List[int]]] = []
        self.num_preemptions = 0
        self.num_swapouts = 0
        self.finished_since_last: List[Sequence] = []

    # ------------------------------------------------------------------ queue ops
    def add(self, seq: Sequence) -> None:
        seq.status = SeqStatus.WAITING
        self.waiting.append(seq)

    def num_unfinished(self) -> int:
        return len(self.waiting) + len(self.running) + len(self.swapped)

    def num_swapped(self) -> int:
        return len(self.swapped)

    def cpu_usage(self) -> float:
        return self.swap.usage() if self.swap is not None else 0.0

    def finish(self, seq: Sequence, status: SeqStatus) -> None:
        if seq.finished:
            return
        seq.status = status
        seq.finish_time = time.time()
        if seq in self.running:
            self.running.remove(seq)
        elif seq in self.swapped:
            self.swapped.remove(seq)
            self.swap.free(seq.swap_blocks)
            seq.swap_blocks = None
        else:
            try:
                self.waiting.remove(seq)
            except ValueError:
                pass
        self.bm.free(seq)

    def abort_request(self, request_id: str) -> List[Sequence]:
        out = [s for s in list(self.running) + list(self.waiting) + list(self.swapped)
               if s.request_id == request_id]
        for s in out:
            self.finish(s, SeqStatus.FINISHED_ABORTED)
        return out

    # ------------------------------------------------------------------ scheduling
    def _preempt(self, seq: Sequence) -> None:
        self.running.remove(seq)
        seq.num_preemptions += 1
        self.num_preemptions += 1
        nblk = -(-seq.num_computed_tokens // self.cache_cfg.block_size)
        if self.swap is not None and nblk and self.swap.can_allocate(nblk):
            gpu = list(self.bm.block_table(seq))[:nblk]
            cpu = self.swap.allocate(nblk)
            self._swap_out.append((gpu, cpu))
            seq.swap_blocks = cpu
            self.bm.free(seq)
            seq.status = SeqStatus.SWAPPED
            self.swapped.append(seq)
            self.num_swapouts += 1
            return
        self.bm.free(seq)
        seq.status = SeqStatus.PREEMPTED
        seq.num_computed_tokens = 0
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
            if seq.status in (SeqStatus.PREEMPTED, SeqStatus.SWAPPED):
                continue          # seq itself was evicted; list shrank
            item = ScheduledSeq(seq, seq.num_computed_tokens, n)
            (decodes if remaining == 1 else prefills).append(item)
            scheduled_ids.add(seq.seq_id)
            budget -= n
            i += 1

        # 2. swapped sequences back in, FCFS (not in a step that had to evict; not while a
        # sampled token of theirs is still in flight)
        swap_in: List[Tuple[List[int], List[int]]] = []
        while (self.swapped and budget > 0 and not preempted
               and len(self.running) < self.cfg.max_num_seqs):
            seq = self.swapped[0]
            if seq.num_pending:
                break
            remaining = seq.num_tokens - seq.num_computed_tokens
            n = min(remaining, budget)
            if n < remaining and not self.cfg.enable_chunked_prefill and remaining > 1:
                break
            if not self.bm.ensure(seq, seq.num_computed_tokens + n):
                break
            self.swapped.popleft()
            nblk = len(seq.swap_blocks)
            gpu = list(self.bm.block_table(seq))[:nblk]
            swap_in.append((seq.swap_blocks, gpu))
            self.swap.free(seq.swap_blocks)
            seq.swap_blocks = None
            seq.status = SeqStatus.RUNNING
            self.running.append(seq)
            item = ScheduledSeq(seq, seq.num_computed_tokens, n)
            (decodes if remaining == 1 else prefills).append(item)
            budget -= n

        # 3. waiting sequences, FCFS
        n_prefill = len(prefills)
        while (self.waiting and budget > 0 and len(self.running) < self.cfg.max_num_seqs
               and n_prefill < self.cfg.max_num_prefill_seqs and not preempted
               and not self.swapped):
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
        swap_out, self._swap_out = self._swap_out, []
        return SchedulerOutput(decodes, prefills, preempted, total, swap_out, swap_in)

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
