"""Plain-PyTorch reference implementations of every fused op.

These are (a) the CPU execution path (BASELINE config #1, the Xeon path the
reference serves with vLLM-CPU, core/helm-charts/vllm/xeon-values.yaml) and
(b) the fp32 numerics oracle that every HIP kernel test compares against.

KV-cache layout (shared with csrc/kernels/attention.hip):
  k_cache[num_blocks, num_kv_heads, block_size, head_dim]   token-major
  v_cache[num_blocks, num_kv_heads, head_dim, block_size]   dim-major (V^T)
Storing V transposed lets the MFMA P·V product take V straight from HBM as
the A operand (4 consecutive tokens per lane = one 8-byte load) with no LDS
transpose, see attention.hip.
"""

from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- norms

def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return (xf * torch.rsqrt(var + eps) * weight.float()).to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor,
                       eps: float) -> tuple[torch.Tensor, torch.Tensor]:
    """residual <- x + residual ; return (rms_norm(residual), residual)."""
    r = (x.float() + residual.float()).to(x.dtype)
    return rms_norm(r, weight, eps), r


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
               eps: float) -> torch.Tensor:
    return F.layer_norm(x.float(), (x.shape[-1],), weight.float(),
                        None if bias is None else bias.float(), eps).to(x.dtype)


def fused_add_layer_norm(x, residual, weight, bias, eps):
    r = (x.float() + residual.float()).to(x.dtype)
    return layer_norm(r, weight, bias, eps), r


# ----------------------------------------------------------------------------- activations

def silu_and_mul(x: torch.Tensor) -> torch.Tensor:
    d = x.shape[-1] // 2
    xf = x.float()
    return (F.silu(xf[..., :d]) * xf[..., d:]).to(x.dtype)


def gelu_and_mul(x: torch.Tensor) -> torch.Tensor:
    d = x.shape[-1] // 2
    xf = x.float()
    return (F.gelu(xf[..., :d], approximate="tanh") * xf[..., d:]).to(x.dtype)


def gelu(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x.float()).to(x.dtype)


def relu(x: torch.Tensor) -> torch.Tensor:
    return F.relu(x)


# ----------------------------------------------------------------------------- rotary

def rope_inv_freq(head_dim: int, theta: float, scaling: Optional[dict],
                  rotary_dim: Optional[int] = None) -> torch.Tensor:
    rd = rotary_dim or head_dim
    inv = 1.0 / (theta ** (torch.arange(0, rd, 2, dtype=torch.float64) / rd))
    if not scaling:
        return inv
    kind = scaling.get("rope_type", scaling.get("type", "default"))
    if kind == "llama3":
        factor = scaling["factor"]
        lo = scaling.get("low_freq_factor", 1.0)
        hi = scaling.get("high_freq_factor", 4.0)
        orig = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = orig / lo, orig / hi
        wl = 2 * math.pi / inv
        smooth = (orig / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        return torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    if kind == "linear":
        return inv / scaling["factor"]
    # dynamic / yarn / default: base frequencies (yarn mscale handled by caller if needed)
    return inv


def rope_cos_sin_cache(max_pos: int, head_dim: int, theta: float,
                       scaling: Optional[dict] = None) -> torch.Tensor:
    """[max_pos, head_dim] fp32: cos in [:, :D/2], sin in [:, D/2:]."""
    inv = rope_inv_freq(head_dim, theta, scaling)
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv)
    return torch.cat([freqs.cos(), freqs.sin()], dim=-1).float()


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """Neox-style rotation. x: [T, H, D]; positions [T]."""
    d2 = x.shape[-1] // 2
    cs = cos_sin[positions.long()]
    cos = cs[:, None, :d2]
    sin = cs[:, None, d2:]
    xf = x.float()
    x1, x2 = xf[..., :d2], xf[..., d2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


def apply_rope_gptj(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """Interleaved (GPT-J / Llama-4) rotation of pairs (2i, 2i+1) by frequency i."""
    d2 = x.shape[-1] // 2
    cs = cos_sin[positions.long()]
    cos, sin = cs[:, None, :d2], cs[:, None, d2:]
    xf = x.float()
    x1, x2 = xf[..., 0::2], xf[..., 1::2]
    out = torch.stack([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)
    return out.flatten(-2).to(x.dtype)


def rope_qkv_cache(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: Optional[torch.Tensor],
                   slot_mapping: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                   num_heads: int, num_kv_heads: int, head_dim: int,
                   bias: Optional[torch.Tensor] = None,
                   q_norm_w: Optional[torch.Tensor] = None,
                   k_norm_w: Optional[torch.Tensor] = None,
                   norm_eps: float = 1e-6, is_neox: bool = True) -> torch.Tensor:
    """Reference for the fused K4 kernel (bias → qk-norm → RoPE → KV write).

    Returns q [T, Hq, D] (rotated). K/V are written into the paged cache at
    ``slot_mapping`` (slot = block * block_size + offset; negative = skip).
    """
    T = qkv.shape[0]
    if bias is not None:
        qkv = (qkv.float() + bias.float()).to(qkv.dtype)
    qs, ks = num_heads * head_dim, num_kv_heads * head_dim
    q = qkv[:, :qs].reshape(T, num_heads, head_dim)
    k = qkv[:, qs:qs + ks].reshape(T, num_kv_heads, head_dim)
    v = qkv[:, qs + ks:qs + 2 * ks].reshape(T, num_kv_heads, head_dim)
    if q_norm_w is not None:
        q = rms_norm(q, q_norm_w, norm_eps)
        k = rms_norm(k, k_norm_w, norm_eps)
    if cos_sin is not None:
        rot = apply_rope if is_neox else apply_rope_gptj
        q = rot(q, positions, cos_sin)
        k = rot(k, positions, cos_sin)
    write_kv_cache(k, v, slot_mapping, k_cache, v_cache)
    return q.contiguous()


def write_kv_cache(k: torch.Tensor, v: torch.Tensor, slot_mapping: torch.Tensor,
                   k_cache: torch.Tensor, v_cache: torch.Tensor) -> None:
    bs = k_cache.shape[2]
    sm = slot_mapping.long()
    valid = sm >= 0
    if not bool(valid.any()):
        return
    sm, k, v = sm[valid], k[valid], v[valid]
    blk, off = sm // bs, sm % bs
    k_cache[blk, :, off, :] = k.to(k_cache.dtype)
    v_cache[blk, :, :, off] = v.to(v_cache.dtype)


# ----------------------------------------------------------------------------- attention

def _gather_kv(k_cache, v_cache, block_table: torch.Tensor, n: int):
    bs = k_cache.shape[2]
    nb = (n + bs - 1) // bs
    blocks = block_table[:nb].long()
    k = k_cache[blocks]                       # [nb, Hkv, bs, D]
    k = k.permute(0, 2, 1, 3).reshape(nb * bs, k.shape[1], k.shape[3])[:n]
    v = v_cache[blocks]                       # [nb, Hkv, D, bs]
    v = v.permute(0, 3, 1, 2).reshape(nb * bs, v.shape[1], v.shape[2])[:n]
    return k, v                               # [n, Hkv, D]


def _attend(q, k, v, scale, causal_offset: Optional[int], chunk: Optional[int] = None,
            sliding: Optional[int] = None):
    """q [Tq, Hq, D]; k,v [Tk, Hkv, D]; fp32 math. causal_offset = pos of q[0]."""
    Hq, Hkv = q.shape[1], k.shape[1]
    g = Hq // Hkv
    kf = k.float().repeat_interleave(g, dim=1)
    vf = v.float().repeat_interleave(g, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), kf) * scale
    if causal_offset is not None:
        qpos = causal_offset + torch.arange(q.shape[0], device=q.device)
        kpos = torch.arange(k.shape[0], device=q.device)
        mask = kpos[None, :] > qpos[:, None]
        if sliding:
            mask |= kpos[None, :] <= qpos[:, None] - sliding
        if chunk:
            mask |= (kpos[None, :] // chunk) != (qpos[:, None] // chunk)
        s = s.masked_fill(mask[None], float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("hqk,khd->qhd", p, vf)


def paged_attention_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                           block_tables: torch.Tensor, seq_lens: torch.Tensor,
                           scale: float, sliding_window: Optional[int] = None,
                           chunk_size: Optional[int] = None) -> torch.Tensor:
    """q [B, Hq, D] (one new token per sequence, already in the cache)."""
    out = torch.empty_like(q)
    for b in range(q.shape[0]):
        n = int(seq_lens[b])
        if n == 0:
            out[b] = 0
            continue
        lo = 0
        if sliding_window:
            lo = max(lo, n - sliding_window)
        if chunk_size:
            lo = max(lo, ((n - 1) // chunk_size) * chunk_size)
        k, v = _gather_kv(k_cache, v_cache, block_tables[b], n)
        out[b] = _attend(q[b:b + 1], k[lo:], v[lo:], scale, None)[0].to(q.dtype)
    return out


def paged_attention_prefill(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                            block_tables: torch.Tensor, cu_seqlens_q: torch.Tensor,
                            seq_lens: torch.Tensor, scale: float, causal: bool = True,
                            sliding_window: Optional[int] = None,
                            chunk_size: Optional[int] = None) -> torch.Tensor:
    """Varlen (chunked) prefill over the paged cache.

    q [T, Hq, D]; sequence s owns q rows cu_seqlens_q[s]:cu_seqlens_q[s+1]; its
    total KV length (context + new) is seq_lens[s]; query i sits at absolute
    position seq_lens[s] - q_len + i.
    """
    out = torch.empty_like(q)
    for s in range(len(seq_lens)):
        a, b = int(cu_seqlens_q[s]), int(cu_seqlens_q[s + 1])
        if b == a:
            continue
        n = int(seq_lens[s])
        k, v = _gather_kv(k_cache, v_cache, block_tables[s], n)
        off = n - (b - a) if causal else None
        out[a:b] = _attend(q[a:b], k, v, scale, off, chunk_size, sliding_window).to(q.dtype)
    return out


def attention_varlen(q, k, v, cu_seqlens: torch.Tensor, scale: float, causal: bool):
    """Non-paged varlen attention (encoder models). q,k,v [T, H, D]."""
    out = torch.empty_like(q)
    for s in range(len(cu_seqlens) - 1):
        a, b = int(cu_seqlens[s]), int(cu_seqlens[s + 1])
        out[a:b] = _attend(q[a:b], k[a:b], v[a:b], scale, 0 if causal else None).to(q.dtype)
    return out


# ----------------------------------------------------------------------------- MoE

def topk_softmax(router_logits: torch.Tensor, topk: int, renormalize: bool = True):
    """Returns (weights fp32 [T, k], ids int32 [T, k])."""
    p = torch.softmax(router_logits.float(), dim=-1)
    w, ids = torch.topk(p, topk, dim=-1)
    if renormalize:
        w = w / w.sum(-1, keepdim=True)
    return w, ids.to(torch.int32)


def fused_moe(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor, topk_w: torch.Tensor,
              topk_ids: torch.Tensor, act: str = "silu") -> torch.Tensor:
    """x [T, H]; w13 [E, 2F, H]; w2 [E, H, F]."""
    T, H = x.shape
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    for e in range(w13.shape[0]):
        tok, slot = (topk_ids == e).nonzero(as_tuple=True)
        if tok.numel() == 0:
            continue
        h = x[tok].float() @ w13[e].float().t()
        F_ = h.shape[-1] // 2
        h = F.silu(h[:, :F_]) * h[:, F_:]
        h = h.to(x.dtype).float() @ w2[e].float().t()
        out.index_add_(0, tok, h * topk_w[tok, slot, None])
    return out.to(x.dtype)


# ----------------------------------------------------------------------------- sampling

def apply_penalties(logits: torch.Tensor, output_counts: torch.Tensor,
                    prompt_mask: torch.Tensor, presence: torch.Tensor,
                    frequency: torch.Tensor, repetition: torch.Tensor) -> torch.Tensor:
    """OpenAI presence/frequency + HF repetition penalty. counts [B, V] int."""
    logits = logits.clone()
    seen = (output_counts > 0) | prompt_mask
    rep = repetition[:, None].expand_as(logits)
    logits = torch.where(seen & (logits > 0), logits / rep, logits)
    logits = torch.where(seen & (logits <= 0), logits * rep, logits)
    logits -= frequency[:, None] * output_counts.float()
    logits -= presence[:, None] * (output_counts > 0).float()
    return logits


def top_k_top_p_min_p_mask(logits: torch.Tensor, top_k: torch.Tensor, top_p: torch.Tensor,
                           min_p: torch.Tensor) -> torch.Tensor:
    """Mask logits outside top-k / nucleus top-p / min-p with -inf. Per-row params."""
    V = logits.shape[-1]
    sorted_l, idx = logits.sort(dim=-1, descending=True)
    ranks = torch.arange(V, device=logits.device)[None, :]
    k = torch.where(top_k <= 0, torch.full_like(top_k, V), top_k).clamp(max=V)
    drop = ranks >= k[:, None]
    # vLLM order: top-k first, then nucleus over the renormalised top-k set
    probs = sorted_l.masked_fill(drop, float("-inf")).softmax(-1)
    cum = probs.cumsum(-1)
    drop |= (cum - probs) > top_p[:, None]
    drop |= probs < (min_p[:, None] * probs[:, :1])
    drop[:, 0] = False
    sorted_l = sorted_l.masked_fill(drop, float("-inf"))
    return torch.empty_like(logits).scatter_(-1, idx, sorted_l)
