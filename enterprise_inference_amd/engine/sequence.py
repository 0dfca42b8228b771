"""Request / sequence state tracked by the scheduler."""

from __future__ import annotations

import enum
import itertools
import time
from typing import Dict, List, Optional

from .sampling_params import SamplingParams

_seq_counter = itertools.count(1)


def needs_host_processing(seq: "Sequence") -> bool:
    """Rows whose sampling needs the host (penalties over the output, logits processors,
    guided decoding, logprobs, best_of ranking): their logits are gathered in full and their
    step is read back before the next one is planned."""
    p = seq.params
    return (p.needs_penalties or p.needs_logit_processing or p.logprobs is not None
            or p.prompt_logprobs is not None or seq.guided_state is not None
            or p.best_of > p.n or seq.beam is not None)


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    PREEMPTED = 2
    FINISHED_STOPPED = 3
    FINISHED_LENGTH = 4
    FINISHED_ABORTED = 5
    SWAPPED = 6                      # preempted with its KV parked in the host swap space

    @property
    def finished(self) -> bool:
        return 3 <= self.value <= 5


FINISH_REASON = {
    SeqStatus.FINISHED_STOPPED: "stop",
    SeqStatus.FINISHED_LENGTH: "length",
    SeqStatus.FINISHED_ABORTED: "abort",
}


class Sequence:
    """One generation stream (a request with n>1 owns n sequences)."""

    __slots__ = ("seq_id", "request_id", "index", "prompt_token_ids", "output_token_ids",
                 "params", "status", "num_computed_tokens", "num_cached_tokens", "arrival_time",
                 "first_scheduled_time", "first_token_time", "last_token_time", "finish_time",
                 "stop_reason", "output_logprobs", "cumulative_logprob", "prompt_logprobs",
                 "detok_offset", "output_text", "prefix_offset", "read_offset", "lora",
                 "num_preemptions", "seed", "guided_state", "swap_blocks", "mm_embeds",
                 "mm_positions", "cache_salt", "token_times", "priority",
                 "num_pending", "beam")

    def __init__(self, request_id: str, prompt_token_ids: List[int], params: SamplingParams,
                 index: int = 0, arrival_time: Optional[float] = None, seed: int = 0,
                 priority: int = 0):
        self.seq_id = next(_seq_counter)
        self.request_id = request_id
        self.index = index
        self.prompt_token_ids = list(prompt_token_ids)
        self.output_token_ids: List[int] = []
        self.params = params
        self.status = SeqStatus.WAITING
        self.num_computed_tokens = 0
        self.num_cached_tokens = 0
        self.arrival_time = arrival_time if arrival_time is not None else time.time()
        self.first_scheduled_time: Optional[float] = None
        self.first_token_time: Optional[float] = None
        self.last_token_time: Optional[float] = None
        self.finish_time: Optional[float] = None
        self.stop_reason = None
        self.output_logprobs: List[Dict[int, float]] = []
        self.cumulative_logprob = 0.0
        self.prompt_logprobs = None
        self.detok_offset = 0
        self.output_text = ""
        self.prefix_offset = 0
        self.read_offset = 0
        self.lora = None
        self.num_preemptions = 0
        self.seed = seed
        self.guided_state = None
        self.swap_blocks = None
        self.mm_embeds = None          # [n image tokens, hidden] on the device
        self.mm_positions = None       # prompt positions of those tokens (sorted int64)
        self.cache_salt = 0            # prefix-cache key salt (image content hash)
        self.token_times: List[float] = []
        self.priority = priority
        # tokens sampled by a launched, not yet read-back step (overlapped scheduling): they
        # count toward num_tokens so the next step can be planned before the values are known
        self.num_pending = 0
        self.beam = None               # engine.beam_search.BeamGroup of a beam-search request

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_token_ids) + len(self.output_token_ids) + self.num_pending

    @property
    def num_real_tokens(self) -> int:
        """Tokens whose ids are known on the host (excludes in-flight samples)."""
        return len(self.prompt_token_ids) + len(self.output_token_ids)

    @property
    def num_prompt_tokens(self) -> int:
        return len(self.prompt_token_ids)

    @property
    def all_token_ids(self) -> List[int]:
        return self.prompt_token_ids + self.output_token_ids

    def token_at(self, i: int) -> int:
        """Token id at position i; 0 for an in-flight sample (its id is filled in on device)."""
        n = len(self.prompt_token_ids)
        if i < n:
            return self.prompt_token_ids[i]
        j = i - n
        return self.output_token_ids[j] if j < len(self.output_token_ids) else 0

    @property
    def is_prefill(self) -> bool:
        """True while tokens other than the newest sampled one remain uncomputed."""
        return self.num_computed_tokens < self.num_tokens - 1

    @property
    def finished(self) -> bool:
        return self.status.finished

    def __repr__(self) -> str:
        return (f"Sequence(id={self.seq_id}, req={self.request_id}, status={self.status.name}, "
                f"prompt={self.num_prompt_tokens}, out={len(self.output_token_ids)}, "
                f"computed={self.num_computed_tokens})")
