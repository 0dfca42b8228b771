"""Sampling parameters (the request fields of docs/api-spec.yaml:259-525 / :614-845)."""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Union


@dataclasses.dataclass
class SamplingParams:
    n: int = 1
    best_of: Optional[int] = None
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = -1
    min_p: float = 0.0
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    repetition_penalty: float = 1.0
    seed: Optional[int] = None
    stop: Union[None, str, List[str]] = None
    stop_token_ids: Optional[List[int]] = None
    ignore_eos: bool = False
    max_tokens: Optional[int] = 16
    min_tokens: int = 0
    logprobs: Optional[int] = None
    prompt_logprobs: Optional[int] = None
    skip_special_tokens: bool = True
    spaces_between_special_tokens: bool = True
    include_stop_str_in_output: bool = False
    logit_bias: Optional[Dict[int, float]] = None
    allowed_token_ids: Optional[List[int]] = None
    # guided decoding (choice / regex / json / grammar handled in engine/guided.py)
    guided_choice: Optional[List[str]] = None
    guided_regex: Optional[str] = None
    guided_json: Optional[object] = None
    guided_grammar: Optional[str] = None
    # beam search (width = best_of), vLLM semantics (engine/beam_search.py)
    use_beam_search: bool = False
    length_penalty: float = 1.0
    early_stopping: bool = False

    def __post_init__(self) -> None:
        if isinstance(self.stop, str):
            self.stop = [self.stop]
        elif self.stop is None:
            self.stop = []
        self.stop_token_ids = list(self.stop_token_ids or [])
        if self.best_of is None:
            self.best_of = self.n
        self.verify()

    def verify(self) -> None:
        if self.n < 1:
            raise ValueError("n must be >= 1")
        if self.best_of < self.n:
            raise ValueError("best_of must be >= n")
        if self.temperature < 0:
            raise ValueError("temperature must be non-negative")
        if not 0.0 < self.top_p <= 1.0:
            raise ValueError("top_p must be in (0, 1]")
        if self.top_k == 0 or self.top_k < -1:
            raise ValueError("top_k must be -1 (disable) or at least 1")
        if not 0.0 <= self.min_p <= 1.0:
            raise ValueError("min_p must be in [0, 1]")
        if not -2.0 <= self.presence_penalty <= 2.0:
            raise ValueError("presence_penalty must be in [-2, 2]")
        if not -2.0 <= self.frequency_penalty <= 2.0:
            raise ValueError("frequency_penalty must be in [-2, 2]")
        if self.repetition_penalty <= 0:
            raise ValueError("repetition_penalty must be > 0")
        if self.max_tokens is not None and self.max_tokens < 1:
            raise ValueError("max_tokens must be at least 1")
        if self.min_tokens < 0:
            raise ValueError("min_tokens must be >= 0")
        if self.logprobs is not None and self.logprobs < 0:
            raise ValueError("logprobs must be non-negative")
        if self.use_beam_search:
            if self.temperature > 1e-5:
                raise ValueError("beam search requires temperature 0")
            if self.top_p < 1.0 or self.top_k not in (-1,) or self.min_p > 0.0:
                raise ValueError("beam search does not combine with top_p / top_k / min_p")
            if self.needs_penalties or self.guided_choice or self.guided_regex or \
                    self.guided_json is not None or self.guided_grammar:
                raise ValueError("beam search does not combine with penalties or guided decoding")

    @property
    def greedy(self) -> bool:
        return self.temperature < 1e-5

    @property
    def needs_penalties(self) -> bool:
        return (self.presence_penalty != 0.0 or self.frequency_penalty != 0.0
                or self.repetition_penalty != 1.0)

    @property
    def needs_logit_processing(self) -> bool:
        return bool(self.logit_bias or self.allowed_token_ids or self.guided_choice
                    or self.guided_regex or self.guided_json is not None or self.guided_grammar
                    or self.min_tokens > 0)

    def clone(self, **kw) -> "SamplingParams":
        return dataclasses.replace(self, **kw)
