"""Paged attention ops (K1 decode, K2 varlen prefill) -> csrc/kernels/attention.hip.

A step's token batch is laid out as [decode tokens (1 per sequence) | prefill
tokens (varlen chunks)].  Both parts read K/V from the paged cache (the K4
kernel has already written this step's K/V), so chunked prefill and prefix
caching need no special path.
"""

from __future__ import annotations

import dataclasses
import math
import os
from typing import List, Optional, Sequence

import torch

from . import reference as ref
from ._dispatch import check, lib, ptr, require, stream, use_hip

EIA_UNSUPPORTED = 1002       # csrc/include/eia_common.h EiaStatus


def heads_per_workgroup(num_heads: int, num_kv_heads: int) -> int:
    g = num_heads // num_kv_heads
    return 4 if g % 4 == 0 else 2 if g % 2 == 0 else 1


# 16-query tiles per prefill wave (csrc/kernels/attention.hip paged_prefill_kernel): every K/V
# unit a wave loads feeds QT tiles.
# The wave keeps QT tiles of O accumulators and Q fragments plus two K/V unit buffers in
# registers; QT = 4 at D = 128 spills (hipcc kernel-resource-usage).  Measured on MI355X
# (scripts/bench_prefill_attn.py, profiles/prefill_attn_r1.log): D = 128 causal 1x8192
# qt 1/2/3 = 3831/2076/1792 us; D = 64 (BERT, 12 heads, 32x512) qt 1/2/3/4 = 131/85/119/109 us.
def prefill_tiles(head_dim: int) -> int:
    return 2 if head_dim <= 64 else 3 if head_dim <= 128 else 1


PREFILL_LDS = 16          # kernel variant flag: K/V units shared by the workgroup through LDS
# LDS form, D = 128 causal (profiles/prefill_attn_lds_r1.log): qt 1/2/3/4 = 1296/1905/1865/2186 us
# at 1x8192 (register form qt 3: 1867 us).  qt 1 needs 185 registers -> 2 waves/SIMD, and with
# the K/V traffic already cut 4x by LDS sharing, occupancy is what pays.  After the VALU trim
# (softmax_pv_lean: uniform unmasked units, scale folded into the exponent FMA; PMC counts had
# ~9 VALU per MFMA, profiles/pmc_prefill_r1.md) and a 2-wave register bound for qt 2, qt 2
# wins at 1x8192 / 4x2048 / 65x128 = 1045 / 270 / 52.5 us vs qt 1 1181 / 276 / 55.1 us, and
# loses at 16x512 (90 vs 85 us) (profiles/prefill_attn_lean_r1.log).  With the bank-conflict-
# free swizzled LDS layout: qt 2 = 1018 / 269 / 89 / 51.7 us, qt 1 = 1090 / 254 / 80 / 54.2 us
# at 1x8192 / 4x2048 / 16x512 / 65x128 (profiles/prefill_attn_swizzle_r1.log).
PREFILL_LDS_QT = {64: 1, 128: 2}


# Flash-attention form (csrc/kernels/attention_fa.hip): 8 waves, 64 queries x 4 heads of one KV
# group per workgroup, 64-key K/V tiles in swizzled LDS, v_mfma_f32_32x32x16_bf16 with P^T fed
# from the S^T accumulators.  D = 128, G % 4 == 0, block size % 64 == 0.
PREFILL_FA = 32
_FA_ENV = os.environ.get("EIA_PREFILL_FA", "1") != "0"
PREFILL_FA_QB = 64


def fa_supported(num_heads: int, num_kv_heads: int, head_dim: int,
                 block_size: Optional[int]) -> bool:
    return (_FA_ENV and head_dim == 128 and (num_heads // num_kv_heads) % 4 == 0
            and block_size is not None and block_size % 64 == 0)


def prefill_variant(num_heads: int, num_kv_heads: int, head_dim: int,
                    block_size: Optional[int] = None) -> int:
    """Kernel variant code: PREFILL_FA for the flash form where it applies; else tiles per
    wave, | PREFILL_LDS for the LDS-shared form (the four waves of a workgroup are four query
    heads of one KV group; needs 32 | block size)."""
    if fa_supported(num_heads, num_kv_heads, head_dim, block_size):
        return PREFILL_FA
    if (heads_per_workgroup(num_heads, num_kv_heads) == 4 and block_size is not None
            and block_size % 32 == 0 and head_dim in PREFILL_LDS_QT):
        return PREFILL_LDS | PREFILL_LDS_QT[head_dim]
    return prefill_tiles(head_dim)


def prefill_query_block(num_heads: int, num_kv_heads: int, head_dim: int = 128,
                        qt: Optional[int] = None, block_size: Optional[int] = None) -> int:
    """Queries covered by one prefill workgroup (4 waves x QT x 16 columns / heads-per-WG;
    64 for the flash form)."""
    code = qt or prefill_variant(num_heads, num_kv_heads, head_dim, block_size)
    if code & PREFILL_FA:
        return PREFILL_FA_QB
    return 16 * (code & 15) * (4 // heads_per_workgroup(num_heads, num_kv_heads))


def build_prefill_work(q_lens: Sequence[int], qblock: int) -> List[int]:
    """[seq, first query] pairs, latest query blocks first: under the causal mask a block's
    work grows with its position, so dispatching the long ones first balances the CUs' tails
    (longest-processing-time order)."""
    items = [(q0, s) for s, n in enumerate(q_lens) for q0 in range(0, n, qblock)]
    items.sort(key=lambda it: -it[0])
    work: List[int] = []
    for q0, s in items:
        work += [s, q0]
    return work


def decode_partitions(batch: int, num_kv_heads: int, num_heads: int, max_len: int,
                      cus: int = 256, max_parts: int = 8) -> int:
    """Context partitions (flash-decoding split) for a decode batch.

    Fitted to scripts/bench_attn.py on MI355X (graph-timed, Llama-8B heads): short contexts
    never split (the partial write + merge costs more than it hides); grids of >= 4 workgroups
    per CU do not split; small grids split up to one workgroup per CU (B=16: P=2, B=1: P=8);
    mid-size grids split 2x with the in-kernel merge (the engine passes the arrival counters):
    B=65 ctx 4096 233 us at P 2 vs 256 us at P 4, B=32 97 vs 102 us
    (profiles/decode_attn_wave_r3_on.log, attn_decode_lean_r1.log).
    EIA_DECODE_P forces a partition count (tuning / A-B runs)."""
    forced = int(os.environ.get("EIA_DECODE_P", "0"))
    if forced > 0:
        return max(1, min(forced, max_parts, max(1, max_len // 64)))
    if max_len <= 512:
        return 1
    g = num_heads // num_kv_heads
    wgs = max(1, batch * num_kv_heads * ((g + 15) // 16))
    if wgs >= 4 * cus:
        return 1
    if wgs >= cus:
        # one to three items per CU: 2 partitions fill the chip evenly only when the items do
        # (wgs a multiple of the CU count); otherwise 4 spread the remainder thinner once the
        # context is long enough to pay for the merge: B 35 (280 items) ctx 4096 120.4 us at
        # P 4 vs 126.5 at P 2, ctx 2048 67.7 vs 69.5 (profiles/attn_long_r4.log); B 65 (520
        # items) ctx 4096 206.5 vs 215.7, ctx 8192 389.7 vs 418.1, ctx 2048 a tie
        # (profiles/attn_long_p_r5.log); B 32 (256 items) and B 96 (768) keep P 2
        p = 4 if (wgs < 3 * cus and wgs % cus and max_len >= 2048 * (wgs // cus)) else 2
    else:
        p = 2
        while p < max_parts and wgs * p * 2 <= cus:
            p *= 2
    return max(1, min(p, max_parts, max_len // 128))


@dataclasses.dataclass
class AttentionMetadata:
    num_decode: int
    num_prefill_tokens: int
    slot_mapping: torch.Tensor                 # [T] int32
    positions: torch.Tensor                    # [T] int32
    # decode part (rows may be padded with seq_len 0 for HIP-graph buckets)
    decode_block_tables: Optional[torch.Tensor] = None   # [Bd, maxb] int32
    decode_seq_lens: Optional[torch.Tensor] = None       # [Bd] int32
    decode_partitions: int = 1
    decode_part_o: Optional[torch.Tensor] = None
    decode_part_ml: Optional[torch.Tensor] = None
    decode_part_cnt: Optional[torch.Tensor] = None      # zeroed int32 [Bd*Hkv*ceil(G/16)]
    decode_p_dyn: Optional[torch.Tensor] = None         # device int32 [1]: partitions this step
    # prefill part
    prefill_block_tables: Optional[torch.Tensor] = None  # [Sp, maxb] int32
    prefill_seq_lens: Optional[torch.Tensor] = None      # [Sp] int32 (context + new)
    prefill_cu_q: Optional[torch.Tensor] = None          # [Sp+1] int32
    prefill_work: Optional[torch.Tensor] = None          # [n_work*2] int32
    prefill_n_work: int = 0
    causal: bool = True
    # multimodal: batch rows whose token embedding is replaced (image placeholders)
    mm_rows: Optional[torch.Tensor] = None               # [n] int64
    mm_embeds: Optional[torch.Tensor] = None             # [n, hidden]

    @property
    def num_tokens(self) -> int:
        return self.num_decode + self.num_prefill_tokens


def paged_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                 block_tables: torch.Tensor, seq_lens: torch.Tensor, scale: float,
                 partitions: int = 1, part_o: Optional[torch.Tensor] = None,
                 part_ml: Optional[torch.Tensor] = None,
                 out: Optional[torch.Tensor] = None, sliding_window: Optional[int] = None,
                 chunk_size: Optional[int] = None,
                 part_cnt: Optional[torch.Tensor] = None,
                 p_dyn: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q [B, Hq, D] -> out [B, Hq, D].

    With ``partitions > 1`` the context is split over grid.z; ``part_cnt`` (zeroed int32,
    >= B*Hkv*ceil(G/16) entries, left zeroed by the kernel) lets the last partition merge the
    partials in-kernel, otherwise a separate reduce kernel runs.  ``p_dyn`` (device int32[1])
    makes ``partitions`` an upper bound and reads the partitions actually used from device
    memory (HIP graphs captured once per batch bucket)."""
    if not (use_hip(q, k_cache) and q.dtype == torch.bfloat16):
        r = ref.paged_attention_decode(q, k_cache, v_cache, block_tables, seq_lens, scale,
                                       sliding_window, chunk_size)
        if out is not None:
            out.copy_(r)
            return out
        return r
    B, Hq, D = q.shape
    Hkv, bs = k_cache.shape[1], k_cache.shape[2]
    require(q.stride(2) == 1 and q.stride(1) == D, "paged_decode: q layout [B,Hq,D]")
    require(block_tables.dtype == torch.int32 and seq_lens.dtype == torch.int32, "int32 metadata")
    require(block_tables.shape[0] >= B and seq_lens.shape[0] >= B, "metadata rows < batch")
    require(block_tables.stride(1) == 1, "block_tables rows must be contiguous")
    o = torch.empty_like(q) if out is None else out
    if partitions > 1:
        need = B * Hq * partitions
        require(part_o is not None and part_o.numel() >= need * D and part_ml.numel() >= need * 2,
                "decode workspace too small")
        if part_cnt is not None:
            G = Hq // Hkv
            require(part_cnt.dtype == torch.int32 and
                    part_cnt.numel() >= B * Hkv * ((G + 15) // 16), "decode counters too small")
    check(lib().eia_paged_decode(
        ptr(q), q.stride(0), ptr(k_cache), ptr(v_cache), ptr(block_tables), block_tables.stride(0),
        ptr(seq_lens), ptr(o), o.stride(0), ptr(part_o) if partitions > 1 else None,
        ptr(part_ml) if partitions > 1 else None,
        ptr(part_cnt) if (partitions > 1 and part_cnt is not None) else None,
        float(scale), B, Hq, Hkv, D, bs, partitions,
        sliding_window or 0, chunk_size or 0,
        ptr(p_dyn) if (partitions > 1 and p_dyn is not None) else None, stream(q)), "paged_decode")
    return o


def paged_prefill(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                  block_tables: torch.Tensor, seq_lens: torch.Tensor, cu_q: torch.Tensor,
                  work: Optional[torch.Tensor], n_work: int, scale: float, causal: bool = True,
                  sliding_window: Optional[int] = None, chunk_size: Optional[int] = None,
                  out: Optional[torch.Tensor] = None, qt: Optional[int] = None) -> torch.Tensor:
    """q [T, Hq, D] (varlen, cu_q) -> out [T, Hq, D].  `work` must be built with
    prefill_query_block(Hq, Hkv, D, qt, block_size) (qt = variant code, default
    prefill_variant(Hq, Hkv, D, block_size))."""
    if not (use_hip(q, k_cache) and q.dtype == torch.bfloat16):
        r = ref.paged_attention_prefill(q, k_cache, v_cache, block_tables, cu_q, seq_lens, scale,
                                        causal, sliding_window, chunk_size)
        if out is not None:
            out.copy_(r)
            return out
        return r
    T, Hq, D = q.shape
    Hkv, bs = k_cache.shape[1], k_cache.shape[2]
    require(q.stride(2) == 1 and q.stride(1) == D, "paged_prefill: q layout [T,Hq,D]")
    for t in (block_tables, seq_lens, cu_q, work):
        require(t is not None and t.dtype == torch.int32 and t.is_cuda, "int32 device metadata")
    require(block_tables.stride(1) == 1, "block_tables rows must be contiguous")
    o = torch.empty_like(q) if out is None else out
    hpw = heads_per_workgroup(Hq, Hkv)
    code = qt or prefill_variant(Hq, Hkv, D, bs)
    if code & PREFILL_FA:
        rc = lib().eia_paged_prefill_fa(
            ptr(q), q.stride(0), ptr(o), o.stride(0), ptr(k_cache), ptr(v_cache),
            ptr(block_tables), block_tables.stride(0), ptr(seq_lens), ptr(cu_q), ptr(work), n_work,
            float(scale), Hq, Hkv, D, bs, 1 if causal else 0, sliding_window or 0, chunk_size or 0,
            stream(q))
        if rc != EIA_UNSUPPORTED:
            check(rc, "paged_prefill_fa")
            return o
        code = PREFILL_LDS | (PREFILL_FA_QB // 16)   # same query blocks (HPW 4 x QT x 16)
        require(hpw == 4, "paged_prefill: flash work list needs 4 heads per workgroup")
    check(lib().eia_paged_prefill(
        ptr(q), q.stride(0), ptr(o), o.stride(0), ptr(k_cache), ptr(v_cache), ptr(block_tables),
        block_tables.stride(0), ptr(seq_lens), ptr(cu_q), ptr(work), n_work, float(scale), Hq, Hkv,
        D, bs, hpw, 1 if causal else 0, sliding_window or 0, chunk_size or 0, code, stream(q)),
        "paged_prefill")
    return o


_FUSED_ENV = os.environ.get("EIA_DECODE_FUSED_ROPE", "1") != "0"
# rows of D fp32 the fused decode prologue stages split-K QKV slabs in (the kernel's merge
# buffer, NW * 17 = 68 rows; csrc/kernels/attention.hip `staged`): sk * (q heads per group + 2)
DECODE_STAGE_ROWS = 68


def decode_rope_attention(qkv, md: AttentionMetadata, k_cache: torch.Tensor,
                          v_cache: torch.Tensor, rotary, num_heads: int, num_kv_heads: int,
                          head_dim: int, scale: float, bias: Optional[torch.Tensor] = None,
                          q_norm_w: Optional[torch.Tensor] = None,
                          k_norm_w: Optional[torch.Tensor] = None, norm_eps: float = 1e-6,
                          sliding_window: Optional[int] = None,
                          chunk_size: Optional[int] = None) -> Optional[torch.Tensor]:
    """Pure-decode step: QKV reduce + bias + qk-norm + RoPE + KV write + attention in ONE
    kernel (csrc/kernels/attention.hip eia_paged_decode_rope) -> out [B, Hq, D].

    Returns None when the fused form does not apply (CPU, prefill tokens in the step, GPT-J
    rotary, G > 16, D not 64/128, block size not a multiple of 32, EIA_DECODE_FUSED_ROPE=0);
    the caller then runs rope_qkv_cache + attention.  Same bits as the two-kernel path."""
    from .gemm import SplitK
    if not _FUSED_ENV or md.num_prefill_tokens != 0 or md.num_decode == 0 or rotary is None:
        return None
    if not rotary.is_neox or head_dim not in (64, 128) or num_heads // num_kv_heads > 16:
        return None
    if k_cache.shape[2] % 32 != 0 or md.positions is None:
        return None
    split = isinstance(qkv, SplitK)
    if split and qkv.sk * (min(16, num_heads // num_kv_heads) + 2) > DECODE_STAGE_ROWS:
        # more slabs than the prologue stages in LDS (it would sum them one round trip per
        # slab): one reduce launch first -- a tall split-K (e.g. the 405B TP8 rank's QKV,
        # K 16384) still beats the library GEMM with it (scripts/bench_gemm.py "defer" rows)
        qkv = qkv.materialize()
        split = False
    src = qkv.part if split else qkv
    if not (use_hip(src, k_cache) and k_cache.dtype == torch.bfloat16):
        return None
    if split:
        if qkv.bias is not None:
            require(bias is None, "decode_rope_attention: bias given twice")
            bias = qkv.bias
        if not qkv.part.is_contiguous():
            return None
        T = qkv.M
    else:
        if qkv.dtype != torch.bfloat16 or qkv.stride(-1) != 1:
            return None
        T = qkv.shape[0]
    require((qkv.N if split else qkv.shape[1]) == (num_heads + 2 * num_kv_heads) * head_dim,
            "decode_rope_attention: qkv width")
    B = md.num_decode
    bt, sl = md.decode_block_tables, md.decode_seq_lens
    require(bt.dtype == torch.int32 and sl.dtype == torch.int32 and bt.stride(1) == 1,
            "int32 decode metadata")
    require(md.slot_mapping.dtype == torch.int32 and md.positions.dtype == torch.int32,
            "int32 slot_mapping / positions")
    P = md.decode_partitions
    if P > 1:
        require(md.decode_part_o is not None and md.decode_part_ml is not None and
                md.decode_part_o.numel() >= B * num_heads * P * head_dim, "decode workspace")
    o = torch.empty((B, num_heads, head_dim), dtype=torch.bfloat16, device=k_cache.device)
    rc = lib().eia_paged_decode_rope(
        None if split else ptr(qkv), 0 if split else qkv.stride(0),
        ptr(qkv.part) if split else None, qkv.sk if split else 0,
        ptr(bias), ptr(q_norm_w), ptr(k_norm_w), float(norm_eps), ptr(md.positions),
        ptr(rotary.cos_sin), ptr(md.slot_mapping), T, ptr(k_cache), ptr(v_cache), ptr(bt),
        bt.stride(0), ptr(sl), ptr(o), o.stride(0),
        ptr(md.decode_part_o) if P > 1 else None, ptr(md.decode_part_ml) if P > 1 else None,
        ptr(md.decode_part_cnt) if (P > 1 and md.decode_part_cnt is not None) else None,
        float(scale), B, num_heads, num_kv_heads, head_dim, k_cache.shape[2], P,
        sliding_window or 0, chunk_size or 0,
        ptr(md.decode_p_dyn) if (P > 1 and md.decode_p_dyn is not None) else None, stream(o))
    if rc == EIA_UNSUPPORTED:
        return None
    check(rc, "paged_decode_rope")
    return o


def attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
              md: AttentionMetadata, scale: float, sliding_window: Optional[int] = None,
              chunk_size: Optional[int] = None) -> torch.Tensor:
    """Dispatch the step's decode and prefill parts. q [T, Hq, D]."""
    nd = md.num_decode
    if md.num_prefill_tokens == 0:
        return paged_decode(q[:nd], k_cache, v_cache, md.decode_block_tables, md.decode_seq_lens,
                            scale, md.decode_partitions, md.decode_part_o, md.decode_part_ml,
                            sliding_window=sliding_window, chunk_size=chunk_size,
                            part_cnt=md.decode_part_cnt, p_dyn=md.decode_p_dyn)
    out = torch.empty_like(q)
    if nd:
        paged_decode(q[:nd], k_cache, v_cache, md.decode_block_tables, md.decode_seq_lens, scale,
                     md.decode_partitions, md.decode_part_o, md.decode_part_ml, out=out[:nd],
                     sliding_window=sliding_window, chunk_size=chunk_size,
                     part_cnt=md.decode_part_cnt, p_dyn=md.decode_p_dyn)
    paged_prefill(q[nd:], k_cache, v_cache, md.prefill_block_tables, md.prefill_seq_lens,
                  md.prefill_cu_q, md.prefill_work, md.prefill_n_work, scale, md.causal,
                  sliding_window, chunk_size, out=out[nd:])
    return out
