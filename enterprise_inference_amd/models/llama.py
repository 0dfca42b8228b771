"""Llama-family decoder (Llama 3.x, CodeLlama, DeepSeek-R1-Distill-Llama,
Falcon3, Mistral, Qwen2/2.5 incl. DeepSeek-R1-Distill-Qwen, Qwen3).

Catalog: core/lib/models/model-selection.sh:26-51.  Per-layer
hot path:
  fused add+RMSNorm (K5) -> QKV GEMM (hipBLASLt) -> bias+qk-norm+RoPE+KV write (K4)
  -> paged attention (K1/K2) -> O GEMM -> all-reduce (C1) -> add+RMSNorm (K5)
  -> gate_up GEMM -> SiLU*mul (K7) -> down GEMM -> all-reduce (C2)
"""

from __future__ import annotations

import math
from typing import Iterable, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config import ModelConfig
from ..ops import activation, gemm  # noqa: F401
from ..ops.attention import AttentionMetadata, attention, decode_rope_attention
from ..ops.rotary import RotaryCache, rope_qkv_cache
from ..parallel import state
from ..ops.gemm import SplitK
from .layers import (MergedColumnParallelLinear, ParallelLMHead, PPMissingLayer, QKVParallelLinear,
                     RMSNorm, RowParallelLinear, VocabParallelEmbedding, default_loader)

KVCache = Tuple[torch.Tensor, torch.Tensor]


class LlamaAttention(nn.Module):
    def __init__(self, cfg: ModelConfig, layer_idx: int, rotary: RotaryCache, dtype, device):
        super().__init__()
        self.cfg = cfg
        self.layer_idx = layer_idx
        D = cfg.head_dim
        self.qkv_proj = QKVParallelLinear(cfg.hidden_size, D, cfg.num_attention_heads,
                                          cfg.num_key_value_heads, bias=cfg.attention_bias,
                                          dtype=dtype, device=device)
        self.o_proj = RowParallelLinear(cfg.num_attention_heads * D, cfg.hidden_size, bias=False,
                                        dtype=dtype, device=device)
        self.num_heads = self.qkv_proj.num_heads
        self.num_kv_heads = self.qkv_proj.num_kv_heads
        self.head_dim = D
        self.scale = D ** -0.5
        self.rotary = rotary
        if cfg.qk_norm:
            self.q_norm = RMSNorm(D, cfg.rms_norm_eps, dtype, device)
            self.k_norm = RMSNorm(D, cfg.rms_norm_eps, dtype, device)
        else:
            self.q_norm = self.k_norm = None
        self.sliding_window = cfg.sliding_window
        self.chunk_size = None
        if cfg.attention_chunk_size and cfg.extra.get("no_rope_layers"):
            # Llama-4: chunked local attention on RoPE layers
            if cfg.extra["no_rope_layers"][layer_idx]:
                self.chunk_size = cfg.attention_chunk_size

    def forward(self, h: torch.Tensor, md: AttentionMetadata, kv: KVCache) -> torch.Tensor:
        T = h.shape[0]
        qkv = gemm.linear(h, self.qkv_proj.weight, defer_reduce=True)   # split-K summed in K4
        qn = None if self.q_norm is None else self.q_norm.weight
        kn = None if self.k_norm is None else self.k_norm.weight
        # pure decode: K4 (reduce/bias/qk-norm/RoPE/KV write) runs inside the attention kernel
        o = decode_rope_attention(qkv, md, kv[0], kv[1], self.rotary, self.num_heads,
                                  self.num_kv_heads, self.head_dim, self.scale,
                                  self.qkv_proj.bias, qn, kn, self.cfg.rms_norm_eps,
                                  self.sliding_window, self.chunk_size)
        if o is None:
            q = rope_qkv_cache(qkv, md.positions, self.rotary, md.slot_mapping, kv[0], kv[1],
                               self.num_heads, self.num_kv_heads, self.head_dim,
                               bias=self.qkv_proj.bias, q_norm_w=qn, k_norm_w=kn,
                               norm_eps=self.cfg.rms_norm_eps)
            o = attention(q, kv[0], kv[1], md, self.scale, self.sliding_window, self.chunk_size)
        return self.o_proj(o.view(-1, self.num_heads * self.head_dim)[:T], defer_reduce=True)


class LlamaMLP(nn.Module):
    def __init__(self, hidden: int, inter: int, act: str, dtype, device):
        super().__init__()
        self.gate_up_proj = MergedColumnParallelLinear(hidden, [inter, inter], dtype=dtype,
                                                       device=device)
        self.down_proj = RowParallelLinear(inter, hidden, dtype=dtype, device=device)
        self.act = "silu" if act in ("silu", "swish") else act

    def forward(self, x: torch.Tensor):
        return self.down_proj(self.gate_up_proj.forward_act_and_mul(x, self.act), defer_reduce=True)


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, idx: int, rotary: RotaryCache, dtype, device,
                 mlp: Optional[nn.Module] = None):
        super().__init__()
        self.self_attn = LlamaAttention(cfg, idx, rotary, dtype, device)
        self.mlp = mlp if mlp is not None else LlamaMLP(cfg.hidden_size, cfg.intermediate_size,
                                                        cfg.hidden_act, dtype, device)
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, dtype, device)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, dtype, device)

    def forward(self, h, residual, md, kv):
        if residual is None:
            residual = h
            h = self.input_layernorm(h)
        else:
            h, residual = self.input_layernorm(h, residual)
        h = self.self_attn(h, md, kv)
        fuse = getattr(self.mlp, "norm_and_route", None)
        if fuse is not None:            # MoE: router + top-k inside the add + RMSNorm launch
            r = fuse(h, residual, self.post_attention_layernorm, md)
            if r is not None:
                h, residual, routing = r
                return self.mlp(h, routing=routing), residual
        h, residual = self.post_attention_layernorm(h, residual)
        return self.mlp(h), residual


class LlamaForCausalLM(nn.Module):
    """Also serves MistralForCausalLM / Qwen2ForCausalLM / Qwen3ForCausalLM."""

    supports_pp = True

    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None,
                 layer_factory=None):
        super().__init__()
        self.cfg = cfg
        self.dtype = dtype
        device = torch.device(device) if device is not None else torch.device("cpu")
        self.rotary = RotaryCache(cfg.head_dim, cfg.max_position_embeddings, cfg.rope_theta,
                                  cfg.rope_scaling, device,
                                  is_neox=not cfg.extra.get("rope_interleaved", False))
        # pipeline stage: own layers [start, end); embeddings on the first stage (and the last
        # when tied), final norm + LM head on the last
        self.first, self.last = state.is_first_stage(), state.is_last_stage()
        self.start_layer, self.end_layer = state.stage_layer_range(cfg.num_hidden_layers)
        need_embed = self.first or (self.last and cfg.tie_word_embeddings)
        self.embed_tokens = VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, dtype,
                                                   device) if need_embed else None
        make = layer_factory or (lambda i: LlamaDecoderLayer(cfg, i, self.rotary, dtype, device))
        self.layers = nn.ModuleList([make(i) if self.start_layer <= i < self.end_layer
                                     else PPMissingLayer() for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, dtype, device) if self.last else None
        self.lm_head = ParallelLMHead(cfg.vocab_size, cfg.hidden_size, dtype, device,
                                      tied=self.embed_tokens if cfg.tie_word_embeddings else None
                                      ) if self.last else None

    # kv-cache geometry for the engine
    def kv_heads_per_rank(self) -> int:
        return self.layers[self.start_layer].self_attn.num_kv_heads

    def forward(self, input_ids: torch.Tensor, md: AttentionMetadata,
                kv_caches: List[KVCache], intermediate=None):
        """Last stage: final hidden states.  Other stages: (hidden, residual) for the next
        stage, which passes them back in as ``intermediate``."""
        if self.first:
            h, residual = self.embed_tokens(input_ids), None
            if getattr(md, "mm_rows", None) is not None:   # image placeholders (Llama-4 vision)
                h = h.index_copy(0, md.mm_rows, md.mm_embeds.to(h.dtype))
        else:
            h, residual = intermediate
        for i in range(self.start_layer, self.end_layer):
            h, residual = self.layers[i](h, residual, md, kv_caches[i])
        if not self.last:
            if hasattr(h, "materialize"):      # SplitK / PendingAllReduce
                h = h.materialize()
            return h, residual
        h, _ = self.norm(h, residual)
        return h

    def compute_logits(self, h: torch.Tensor) -> torch.Tensor:
        return self.lm_head.forward_f32(h)

    def compute_logits_local(self, h: torch.Tensor) -> torch.Tensor:
        """TP: this rank's vocab shard of the logits (model dtype, no gather)."""
        return self.lm_head.forward_local(h)

    # ------------------------------------------------------------------ weights
    _STACKED = [
        ("qkv_proj", "q_proj", "q"), ("qkv_proj", "k_proj", "k"), ("qkv_proj", "v_proj", "v"),
        ("gate_up_proj", "gate_proj", 0), ("gate_up_proj", "up_proj", 1),
    ]

    def map_weight_name(self, name: str):
        name = name.replace("model.", "", 1) if name.startswith("model.") else name
        for fused, part, sid in self._STACKED:
            if f".{part}." in name:
                return name.replace(part, fused), sid
        return name, None

    def load_weights(self, weights: Iterable[Tuple[str, torch.Tensor]]) -> List[str]:
        params = dict(self.named_parameters())
        loaded = []
        for name, t in weights:
            if "rotary_emb.inv_freq" in name:
                continue
            pname, sid = self.map_weight_name(name)
            if pname not in params:
                if pname == "lm_head.weight" and self.cfg.tie_word_embeddings:
                    continue
                continue
            p = params[pname]
            loader = getattr(p, "weight_loader", default_loader)
            t = t.to(p.dtype)
            if sid is None:
                loader(p, t)
            else:
                loader(p, t, sid)
            loaded.append(pname)
        return loaded


MistralForCausalLM = LlamaForCausalLM
Qwen2ForCausalLM = LlamaForCausalLM
Qwen3ForCausalLM = LlamaForCausalLM
