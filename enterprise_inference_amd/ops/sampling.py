"""Token sampling (K8) -> csrc/kernels/sampling.hip.

The CPU reference implements the SAME counter-based RNG (splitmix64 over
(seed, token id)) so a seeded request samples identically on both paths.
"""

from __future__ import annotations

from typing import Optional

import torch

from . import reference as ref
from ._dispatch import check, lib, ptr, require, stream, use_hip

_M64 = (1 << 64) - 1


def _s64(x: int) -> int:
    x &= _M64
    return x - (1 << 64) if x >= (1 << 63) else x


_C0 = _s64(0x9E3779B97F4A7C15)
_C1 = _s64(0xBF58476D1CE4E5B9)
_C2 = _s64(0x94D049BB133111EB)
_CI = _s64(0xD1B54A32D192ED03)


def _lsr(x: torch.Tensor, k: int) -> torch.Tensor:
    return (x >> k) & ((1 << (64 - k)) - 1)


def splitmix64_t(x: torch.Tensor) -> torch.Tensor:
    x = x + _C0
    x = (x ^ _lsr(x, 30)) * _C1
    x = (x ^ _lsr(x, 27)) * _C2
    return x ^ _lsr(x, 31)


def splitmix64_int(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def row_seed(request_seed: int, step: int) -> int:
    """Per (request, output index) seed, as a signed int64 for torch."""
    return _s64(splitmix64_int((request_seed & _M64) ^ (step * 0x2545F4914F6CDD1D & _M64)))


def uniform_t(seeds: torch.Tensor, V: int, offset: int = 0) -> torch.Tensor:
    """[B, V] float32 uniforms in (0,1) for global token ids offset..offset+V-1, bit-identical
    to rng_uniform() in the kernel."""
    idx = torch.arange(offset + 1, offset + V + 1, dtype=torch.int64, device=seeds.device)
    h = splitmix64_t(seeds.to(torch.int64)[:, None] ^ (idx[None, :] * _CI))
    return (_lsr(h, 40).to(torch.float32) + 0.5) * (1.0 / 16777216.0)


def sample_reference(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
                     top_p: torch.Tensor, min_p: torch.Tensor, seeds: torch.Tensor) -> torch.Tensor:
    logits = logits.float()
    greedy = logits.argmax(-1).to(torch.int32)
    t = temperature.float()
    if not bool((t > 0).any()):
        return greedy
    tt = torch.where(t > 0, t, torch.ones_like(t))
    masked = ref.top_k_top_p_min_p_mask(logits / tt[:, None], top_k, top_p.float(), min_p.float())
    u = uniform_t(seeds, logits.shape[-1])
    g = masked - torch.log(-torch.log(u))
    sampled = g.argmax(-1).to(torch.int32)
    return torch.where(t > 0, sampled, greedy)


SPLIT_CHUNK = 4096     # tokens per workgroup of the split-row sampler


def f2key_t(x: torch.Tensor) -> torch.Tensor:
    """Order-preserving uint32 key of fp32 values (as int64), bit-identical to f2key()."""
    u = x.float().contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    return torch.where(u >= 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)


def sample_shard(logits: torch.Tensor, temperature: torch.Tensor, seeds: torch.Tensor,
                 vocab_offset: int, floor_keys: Optional[torch.Tensor] = None):
    """Sampling restricted to one tensor-parallel vocab shard.

    logits fp32 [B, V_shard] hold global ids vocab_offset..; returns (value fp32 [B], global
    id int32 [B]) of the shard's Gumbel-max winner (greedy rows: the plain max).  The max over
    shards (lowest id on ties) equals ``sample(full_logits, ...)``: unfiltered rows directly,
    filtered rows with ``floor_keys`` [B] (int64 holding uint32 keys: the admissible-set
    threshold computed over ALL shards by ops/shard_sampling.py)."""
    B, V = logits.shape
    if not use_hip(logits):
        l = logits.float()
        t = temperature.float()
        tt = torch.where(t > 0, t, torch.ones_like(t))
        g = l / tt[:, None] - torch.log(-torch.log(uniform_t(seeds, V, vocab_offset)))
        if floor_keys is not None:
            g = g.masked_fill(f2key_t(l) < floor_keys.to(torch.int64)[:, None], float("-inf"))
        v = torch.where((t > 0)[:, None], g, l)
        best_v, best_i = v.max(-1)          # first max = lowest id on ties
        return best_v, (best_i + vocab_offset).to(torch.int32)
    require(logits.dtype == torch.float32 and logits.stride(-1) == 1, "sample_shard: fp32")
    C = (V + SPLIT_CHUNK - 1) // SPLIT_CHUNK
    ws = torch.empty(2 * B * C, dtype=torch.int32, device=logits.device)
    out_v = torch.empty(B, dtype=torch.float32, device=logits.device)
    out_i = torch.empty(B, dtype=torch.int32, device=logits.device)
    fk = None
    if floor_keys is not None:
        require(floor_keys.numel() >= B and floor_keys.is_cuda, "sample_shard: floor keys")
        fk = floor_keys.to(torch.int64).to(torch.int32).contiguous()     # uint32 bit pattern
    check(lib().eia_sample_shard(ptr(logits), logits.stride(0), B, V, SPLIT_CHUNK, vocab_offset,
                                 ptr(temperature), ptr(seeds), ptr(ws), ws.data_ptr() + 4 * B * C,
                                 ptr(out_v), ptr(out_i), None if fk is None else ptr(fk),
                                 stream(logits)), "sample_shard")
    return out_v, out_i


def radix_hist(logits: torch.Tensor, row_max: torch.Tensor, temperature: torch.Tensor,
               floor_key: torch.Tensor, prefix: torch.Tensor, pmask: torch.Tensor,
               shift: int) -> torch.Tensor:
    """[B, 256] fp32 mass histogram of one radix round over this shard (see
    radix_hist_kernel); key tensors are int64 holding uint32 values."""
    B, V = logits.shape
    if not use_hip(logits):
        l = logits.float()
        k = f2key_t(l)
        t = temperature.float()
        ok = (k >= floor_key[:, None]) & ((k & pmask[:, None]) == prefix[:, None]) & \
            (t > 0)[:, None]
        tt = torch.where(t > 0, t, torch.ones_like(t))
        w = torch.exp((l - row_max[:, None]) / tt[:, None]).masked_fill(~ok, 0.0)
        h = torch.zeros(B, 256, dtype=torch.float32, device=logits.device)
        return h.scatter_add_(1, (k >> shift) & 0xFF, w)
    require(logits.dtype == torch.float32 and logits.stride(-1) == 1, "radix_hist: fp32")
    out = torch.empty(B, 256, dtype=torch.float32, device=logits.device)
    i32 = [x.to(torch.int32).contiguous() for x in (floor_key, prefix, pmask)]
    check(lib().eia_radix_hist(ptr(logits), logits.stride(0), B, V, ptr(row_max.float().contiguous()),
                               ptr(temperature), ptr(i32[0]), ptr(i32[1]), ptr(i32[2]), shift,
                               ptr(out), stream(logits)), "radix_hist")
    return out


def merge_shard_winners(vals: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """[W, B] shard winners (rank order = vocab order) -> [B] int32 global token ids."""
    best = vals.argmax(0)                   # first max = lowest rank = lowest id on ties
    return ids.gather(0, best[None, :])[0].to(torch.int32)


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
           top_p: torch.Tensor, min_p: torch.Tensor, seeds: torch.Tensor,
           out: Optional[torch.Tensor] = None, unfiltered: bool = False) -> torch.Tensor:
    """logits fp32 [B, V]; per-row params on the same device. Returns int32 [B].

    ``unfiltered`` (caller-asserted: no row uses top-k / top-p / min-p) selects the split-row
    kernel, which spreads each row over V/4096 workgroups; same result as the full kernel."""
    if not use_hip(logits):
        r = sample_reference(logits, temperature, top_k, top_p, min_p, seeds)
        if out is not None:
            out.copy_(r)
            return out
        return r
    require(logits.dtype == torch.float32 and logits.stride(-1) == 1, "sample: fp32 logits")
    B, V = logits.shape
    for t, dt in ((temperature, torch.float32), (top_k, torch.int32), (top_p, torch.float32),
                  (min_p, torch.float32), (seeds, torch.int64)):
        require(t.dtype == dt and t.is_cuda and t.numel() >= B, f"sample: param {dt}")
    o = torch.empty(B, dtype=torch.int32, device=logits.device) if out is None else out
    if unfiltered:
        C = (V + SPLIT_CHUNK - 1) // SPLIT_CHUNK
        ws = torch.empty(2 * B * C, dtype=torch.int32, device=logits.device)
        check(lib().eia_sample_split(ptr(logits), logits.stride(0), B, V, SPLIT_CHUNK,
                                     ptr(temperature), ptr(seeds), ptr(ws), ws.data_ptr() + 4 * B * C,
                                     ptr(o), stream(logits)), "sample_split")
        return o
    check(lib().eia_sample(ptr(logits), logits.stride(0), B, V, ptr(temperature), ptr(top_k),
                           ptr(top_p), ptr(min_p), ptr(seeds), ptr(o), stream(logits)), "sample")
    return o


def apply_penalties(logits: torch.Tensor, rows: torch.Tensor, toks: torch.Tensor,
                    counts: torch.Tensor, rep: torch.Tensor, freq: torch.Tensor,
                    pres: torch.Tensor) -> torch.Tensor:
    """In-place sparse penalties; (row, tok) pairs must be unique."""
    n = rows.numel()
    if n == 0:
        return logits
    if not use_hip(logits):
        r, t = rows.long(), toks.long()
        l = logits[r, t]
        rp = rep[r]
        l = torch.where(l > 0, l / rp, l * rp)
        c = counts.float()
        l = torch.where(c > 0, l - freq[r] * c - pres[r], l)
        logits[r, t] = l
        return logits
    check(lib().eia_apply_penalties(ptr(logits), logits.stride(0), ptr(rows), ptr(toks),
                                    ptr(counts), n, ptr(rep), ptr(freq), ptr(pres),
                                    stream(logits)), "apply_penalties")
    return logits


def fill_ids(ids: torch.Tensor, src: torch.Tensor, tok: torch.Tensor) -> torch.Tensor:
    """ids[i] = tok[src[i]] where src[i] >= 0 (in place; int32).  Feeds a step the tokens the
    previous, still in-flight step sampled on the device (overlapped scheduling)."""
    n = ids.numel()
    if n == 0:
        return ids
    if not use_hip(ids):
        m = src >= 0
        if bool(m.any()):
            ids[m] = tok[src[m].long()].to(ids.dtype)
        return ids
    require(ids.dtype == torch.int32 and src.dtype == torch.int32 and tok.dtype == torch.int32,
            "fill_ids: int32 tensors")
    require(src.numel() >= n and ids.is_contiguous(), "fill_ids: shapes")
    check(lib().eia_fill_ids(ptr(ids), ptr(src), ptr(tok), n, stream(ids)), "fill_ids")
    return ids
