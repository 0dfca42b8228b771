"""Beam search (``use_beam_search`` / ``length_penalty`` / ``early_stopping``,
docs/api-spec.yaml:385-408 of the reference; vLLM's beam search semantics).

A beam request starts as ONE sequence: its prompt is prefilled once.  Every decode step each
live beam returns its top-2W next-token log-probs (W = beam width = ``best_of``) through the
logprobs path of the sampler; the group then

  1. ranks every (beam, token) candidate by cumulative log-prob, keeps the best 2W,
  2. moves candidates that end a hypothesis (EOS / stop token / length) to the finished
     list, which keeps the best W by length-penalised score
     cum_logprob / seq_len ** length_penalty (seq_len counts the prompt, EOS excluded),
  3. continues the best W others: a parent chosen once appends its token in place, a parent
     chosen k times forks k-1 children that SHARE its KV blocks (native block-table fork);
     the partially filled last block is copied on write (cow_last + a device block copy run
     before the next step), parents chosen by no candidate are dropped,
  4. stops when no beam runs, or W hypotheses are finished and either ``early_stopping`` is
     set or no running beam can still beat the worst finished score.

The request returns the best ``n`` hypotheses once the group is done (no streaming of
intermediate beams, as in vLLM).
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

from .sequence import Sequence, SeqStatus


@dataclasses.dataclass
class Hypothesis:
    tokens: List[int]
    cum_logprob: float
    finish_reason: str
    stop_reason: object = None
    score: float = 0.0


def beam_score(cum_logprob: float, seq_len: int, length_penalty: float) -> float:
    return cum_logprob / (max(1, seq_len) ** length_penalty)


class BeamGroup:
    def __init__(self, request_id: str, prompt_len: int, width: int, n: int,
                 length_penalty: float, early_stopping: bool, eos_ids, stop_token_ids,
                 ignore_eos: bool, max_tokens: int, max_model_len: int):
        self.request_id = request_id
        self.prompt_len = prompt_len
        self.width = width
        self.n = n
        self.length_penalty = length_penalty
        self.early_stopping = early_stopping
        self.eos_ids = set(eos_ids or [])
        self.stop_token_ids = set(stop_token_ids or [])
        self.ignore_eos = ignore_eos
        self.max_tokens = max_tokens
        self.max_model_len = max_model_len
        self.beams: List[Sequence] = []
        self.finished: List[Hypothesis] = []
        self.done = False
        self._stash: Dict[int, Tuple[Sequence, Dict[int, float]]] = {}

    # ------------------------------------------------------------------ scoring
    def _score(self, cum: float, out_len: int, ends_eos: bool) -> float:
        return beam_score(cum, self.prompt_len + out_len - (1 if ends_eos else 0),
                          self.length_penalty)

    # ------------------------------------------------------------------ step
    def report(self, seq: Sequence, logprobs: Dict[int, float]) -> None:
        self._stash[seq.seq_id] = (seq, logprobs)

    def ready(self) -> bool:
        return bool(self._stash) and all(b.seq_id in self._stash for b in self.beams)

    def take_partial(self) -> List[Sequence]:
        """Beams that reported while a sibling did not run this step (preemption split the
        group): their result is dropped and recomputed next step."""
        out = [s for s, _ in self._stash.values()]
        self._stash.clear()
        return out

    def advance(self):
        """One group step.  Returns (appends [(seq, tok, lp)], forks [(parent, tok, lp)],
        dropped [seq]); the engine applies them (it owns the scheduler / block manager)."""
        W = self.width
        cands = []
        for seq, d in self._stash.values():
            for tok, lp in d.items():
                cands.append((seq.cumulative_logprob + lp, seq.seq_id, tok, seq, lp))
        self._stash.clear()
        cands.sort(key=lambda c: (-c[0], c[1], c[2]))
        running = []
        for cum, _, tok, seq, lp in cands[:2 * W]:
            out_len = len(seq.output_token_ids) + 1
            stop = tok in self.stop_token_ids or (not self.ignore_eos and tok in self.eos_ids)
            if stop:
                sr = tok if tok in self.stop_token_ids else None
                self.finished.append(Hypothesis(seq.output_token_ids + [tok], cum, "stop", sr,
                                                self._score(cum, out_len, tok in self.eos_ids)))
            elif out_len >= self.max_tokens or self.prompt_len + out_len >= self.max_model_len:
                self.finished.append(Hypothesis(seq.output_token_ids + [tok], cum, "length",
                                                None, self._score(cum, out_len, False)))
            elif len(running) < W:
                running.append((cum, tok, seq, lp))
        self.finished.sort(key=lambda h: -h.score)
        del self.finished[W:]
        if not running:
            self.done = True
        elif len(self.finished) >= W:
            if self.early_stopping:
                self.done = True
            else:
                best_run = max(self._score(c[0], len(c[2].output_token_ids) + 1, False)
                               for c in running)
                self.done = self.finished[-1].score >= best_run
        if self.done:
            return [], [], list(self.beams)
        chosen: Dict[int, List[tuple]] = {}
        for cum, tok, seq, lp in running:
            chosen.setdefault(seq.seq_id, []).append((seq, tok, lp))
        appends, forks, dropped = [], [], []
        for b in self.beams:
            picks = chosen.get(b.seq_id)
            if not picks:
                dropped.append(b)
                continue
            for seq, tok, lp in picks[1:]:
                forks.append((seq, tok, lp))
            appends.append(picks[0])
        return appends, forks, dropped

    def results(self) -> List[Hypothesis]:
        """Best n hypotheses (running beams fill up if fewer than n finished)."""
        hyps = list(self.finished)
        if len(hyps) < self.n:
            for b in sorted(self.beams, key=lambda s: -s.cumulative_logprob):
                hyps.append(Hypothesis(list(b.output_token_ids), b.cumulative_logprob, "length",
                                       None, self._score(b.cumulative_logprob,
                                                         len(b.output_token_ids), False)))
        hyps.sort(key=lambda h: -h.score)
        return hyps[:self.n]


def fork_sequence(parent: Sequence) -> Sequence:
    """A new beam sharing the parent's history (the KV block table is forked by the caller)."""
    child = Sequence(parent.request_id, parent.prompt_token_ids, parent.params,
                     index=parent.index, arrival_time=parent.arrival_time, seed=parent.seed,
                     priority=parent.priority)
    child.output_token_ids = list(parent.output_token_ids)
    child.output_logprobs = list(parent.output_logprobs)
    child.cumulative_logprob = parent.cumulative_logprob
    child.num_computed_tokens = parent.num_computed_tokens
    child.num_cached_tokens = parent.num_cached_tokens
    child.first_scheduled_time = parent.first_scheduled_time
    child.first_token_time = parent.first_token_time
    child.last_token_time = parent.last_token_time
    child.status = SeqStatus.RUNNING
    child.beam = parent.beam
    return child
