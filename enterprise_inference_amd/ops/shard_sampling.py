"""Exact filtered sampling on a vocab-sharded LM head.

At tensor parallelism each rank holds the logits of its vocab shard only.  Rows without
top-k / top-p / min-p are sampled per shard and only (value, id) winners cross xGMI
(``sampling.sample_shard``).  Rows WITH filters used to all-gather the full B x V logits
(33 MB per step for Llama-3 at B=65); here they cost a few tiny exchanges instead.  Top-k and
min-p thresholds match the full-row kernel (csrc/kernels/sampling.hip ``sample_kernel``)
exactly; the top-p threshold matches it up to the fp32 summation order of the bin masses (the
shard histograms are summed in rank order, the kernel sums one row), so a token sitting exactly
on the nucleus boundary can land on either side:

  1. global row max m                      <- gather of [B] shard maxima
  2. top-k threshold (k-th largest)         <- gather of each shard's top-kmax values [B, kmax]
     (the k-th largest of the union of per-shard top-k lists IS the global k-th largest)
  3. top-p threshold inside the top-k set   <- the kernel's 4-round radix select by mass,
     distributed: each round every shard histograms its keys ([B, 256], radix_hist kernel),
     the histograms are summed over shards, every rank picks the same digit
  4. min-p threshold                        <- closed form from m: key(m + T ln(min_p))
  5. Gumbel-max over the admissible keys    <- shard winners with the global floor, merged
     (the RNG is keyed by the GLOBAL token id, so the race is the full row's race)

The algorithm is written once as a generator that yields its collectives (``("gather", t)``
-> the [W, ...] stack of every rank's ``t``); ``run_spmd`` executes it over the TP group and
``run_simulated`` runs W shards in lockstep inside one process (kernel tests).  Every
exchange is an all-gather reduced in rank order, so all ranks compute bit-identical
thresholds.
"""

from __future__ import annotations

from typing import Generator, List, Optional

import torch

from . import sampling as S

_DIGIT_SHIFTS = (24, 16, 8, 0)


def _pick_digit(H: torch.Tensor, remaining: torch.Tensor):
    """Per row: the digit whose bin reaches ``remaining`` counting mass from the top bin down
    (sample_kernel's radix_select loop); returns (digit, mass above it).  When no bin reaches
    it (fp32 rounding of the total), the kernel settles on digit 0 with the WHOLE histogram
    mass subtracted -- mirrored here so later rounds pick the same threshold."""
    rev = H.flip(-1)
    cum = rev.cumsum(-1)
    hit = cum >= remaining[:, None]
    any_hit = hit.any(-1)
    idx = torch.where(any_hit, hit.to(torch.int32).argmax(-1),
                      torch.full_like(remaining, 255, dtype=torch.int64))
    above = cum.gather(1, idx[:, None])[:, 0] - rev.gather(1, idx[:, None])[:, 0]
    above = torch.where(any_hit, above, H.sum(-1))
    return (255 - idx).to(torch.int64), above


def filtered_shard_sample(local: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
                          top_p: torch.Tensor, min_p: torch.Tensor, seeds: torch.Tensor,
                          vocab_offset: int, vocab_size: int, kmax: int, any_top_p: bool,
                          any_min_p: bool) -> Generator:
    """SPMD body for one shard.  ``local`` fp32 [B, V_shard] (valid columns only); the
    filter flags / kmax are host-side facts every rank derives from the same staged params.
    Yields ("gather", tensor); returns int32 [B] tokens."""
    B = local.shape[0]
    dev = local.device
    t = temperature.float()
    sampling = t > 0
    # 1. global row max
    lm = local.max(-1).values if local.shape[1] else torch.full((B,), float("-inf"), device=dev)
    m = (yield ("gather", lm)).max(0).values
    floor = torch.zeros(B, dtype=torch.int64, device=dev)
    # 2. top-k threshold: k-th largest of the union of the shards' top-kmax lists
    if kmax > 0:
        kk = min(kmax, local.shape[1])
        tv = local.topk(kk, -1).values if kk else local.new_empty((B, 0))
        if kk < kmax:
            tv = torch.cat([tv, tv.new_full((B, kmax - kk), float("-inf"))], -1)
        allv = (yield ("gather", tv)).permute(1, 0, 2).reshape(B, -1)
        srt = allv.sort(-1, descending=True).values
        k = top_k.to(torch.int64)
        use_k = (k > 0) & (k < vocab_size) & sampling
        kth = srt.gather(1, (k.clamp(1, kmax) - 1)[:, None])[:, 0]
        floor = torch.where(use_k, S.f2key_t(kth), floor)
    # 3. top-p threshold inside the top-k set: distributed 4-round radix select by mass
    if any_top_p:
        use_p = (top_p < 1.0) & sampling
        prefix = torch.zeros(B, dtype=torch.int64, device=dev)
        pmask = torch.zeros(B, dtype=torch.int64, device=dev)
        remaining = None
        for shift in _DIGIT_SHIFTS:
            h = S.radix_hist(local, m, temperature, floor, prefix, pmask, shift)
            H = (yield ("gather", h)).sum(0)
            if remaining is None:
                remaining = top_p.float() * H.sum(-1)        # p * z (z over the top-k set)
            digit, above = _pick_digit(H, remaining)
            remaining = remaining - above
            prefix = prefix | (digit << shift)
            pmask = pmask | (0xFF << shift)
        floor = torch.where(use_p, torch.maximum(floor, prefix), floor)
    # 4. min-p: p_i / p_max >= min_p  <=>  l_i >= m + T ln(min_p)
    if any_min_p:
        use_m = (min_p > 0) & sampling
        tm = S.f2key_t(m + t * torch.log(min_p.float().clamp_min(1e-30)))
        floor = torch.where(use_m, torch.maximum(floor, tm), floor)
    # 5. shard race over the admissible keys, winners merged in rank order
    v, i = S.sample_shard(local, temperature, seeds, vocab_offset, floor_keys=floor)
    g = yield ("gather", torch.cat([v, i.view(torch.float32)]))
    return S.merge_shard_winners(g[:, :B], g[:, B:].contiguous().view(torch.int32))


def run_spmd(gen: Generator, gather) -> torch.Tensor:
    """Drive the generator over a process group; ``gather(t) -> [W, *t.shape]``."""
    try:
        req = next(gen)
        while True:
            kind, t = req
            assert kind == "gather"
            req = gen.send(gather(t.contiguous()))
    except StopIteration as e:
        return e.value


def run_simulated(gens: List[Generator]) -> List[torch.Tensor]:
    """W shards of one row block in lockstep inside one process (tests / single-GPU checks)."""
    reqs = [next(g) for g in gens]
    while True:
        stack = torch.stack([r[1] for r in reqs])
        out: List[Optional[torch.Tensor]] = []
        nxt = []
        done = False
        for g in gens:
            try:
                nxt.append(g.send(stack))
            except StopIteration as e:
                out.append(e.value)
                done = True
        if done:
            assert len(out) == len(gens), "shards diverged"
            return out
        reqs = nxt


def host_filter_facts(top_k, top_p, min_p, temperature, vocab_size: int):
    """(kmax, any_top_p, any_min_p) from the staged host arrays (numpy), identical on every
    rank because every rank stages the same parameters."""
    import numpy as np
    samp = np.asarray(temperature) > 0
    k = np.asarray(top_k)
    ks = k[samp & (k > 0) & (k < vocab_size)]
    kmax = int(ks.max()) if ks.size else 0
    return (kmax, bool((samp & (np.asarray(top_p) < 1.0)).any()),
            bool((samp & (np.asarray(min_p) > 0.0)).any()))
