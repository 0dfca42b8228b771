"""Per-request logits processing before sampling (K13 folded into K8's input).

Handles presence/frequency/repetition penalties (sparse, HIP kernel on GPU),
``logit_bias``, ``allowed_token_ids``, ``min_tokens`` (EOS/stop-token masking)
and guided decoding masks.  Rows that need nothing are untouched, so the
common path costs nothing.
"""

from __future__ import annotations

from typing import List

import numpy as np
import torch

from ..ops import sampling as sampling_ops


def apply_logits_processors(logits: torch.Tensor, items: List) -> torch.Tensor:
    need_pen = [i for i, it in enumerate(items) if it.seq.params.needs_penalties]
    need_other = [i for i, it in enumerate(items) if it.seq.params.needs_logit_processing]
    if not need_pen and not need_other:
        return logits
    if need_pen:
        rows, toks, cnts = [], [], []
        V = logits.shape[-1]
        rep = np.ones(len(items), np.float32)
        freq = np.zeros(len(items), np.float32)
        pres = np.zeros(len(items), np.float32)
        for r in need_pen:
            s = items[r].seq
            p = s.params
            rep[r], freq[r], pres[r] = p.repetition_penalty, p.frequency_penalty, p.presence_penalty
            out = np.asarray(s.output_token_ids, dtype=np.int64)
            u, c = (np.unique(out, return_counts=True) if out.size else
                    (np.zeros(0, np.int64), np.zeros(0, np.int64)))
            if p.repetition_penalty != 1.0:
                pu = np.unique(np.asarray(s.prompt_token_ids, dtype=np.int64))
                pu = np.setdiff1d(pu, u, assume_unique=True)
                u = np.concatenate([u, pu])
                c = np.concatenate([c, np.zeros(len(pu), np.int64)])
            keep = (u >= 0) & (u < V)
            u, c = u[keep], c[keep]
            rows.append(np.full(len(u), r, np.int32))
            toks.append(u.astype(np.int32))
            cnts.append(c.astype(np.int32))
        dev = logits.device
        t = lambda a, dt: torch.from_numpy(np.concatenate(a) if isinstance(a, list) else a).to(dev)
        sampling_ops.apply_penalties(logits, t(rows, None), t(toks, None), t(cnts, None),
                                     torch.from_numpy(rep).to(dev), torch.from_numpy(freq).to(dev),
                                     torch.from_numpy(pres).to(dev))
    for r in need_other:
        s = items[r].seq
        p = s.params
        row = logits[r]
        if p.allowed_token_ids:
            mask = torch.full_like(row, float("-inf"))
            idx = torch.tensor(p.allowed_token_ids, device=row.device, dtype=torch.long)
            mask[idx] = 0.0
            row += mask
        if p.logit_bias:
            idx = torch.tensor([int(k) for k in p.logit_bias], device=row.device, dtype=torch.long)
            val = torch.tensor([float(v) for v in p.logit_bias.values()], device=row.device,
                               dtype=row.dtype)
            row.index_add_(0, idx, val)
        if p.min_tokens and len(s.output_token_ids) < p.min_tokens:
            stop_ids = list(p.stop_token_ids or [])
            eos = getattr(p, "eos_ids", None)
            if eos and not p.ignore_eos:
                stop_ids += list(eos)
            if stop_ids:
                row[torch.tensor(stop_ids, device=row.device, dtype=torch.long)] = float("-inf")
        if s.guided_state is not None:
            # cached device mask per FSM state: no per-step host->device copy of token lists
            row.masked_fill_(~s.guided_state.allowed_mask(row.device, row.shape[0]),
                             float("-inf"))
    return logits
