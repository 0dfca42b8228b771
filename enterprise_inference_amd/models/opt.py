"""OPT decoder (facebook/opt-125m: BASELINE.json config #1, the CPU/Xeon-path
functional check; also runs on the GPU kernels).

Pre-LN (``do_layer_norm_before``) or post-LN blocks, learned positions with the
+2 offset, biased q/k/v/out projections, ReLU FFN, optional project_in/out when
``word_embed_proj_dim != hidden_size``, tied LM head.  Attention uses the same
paged-KV path as the Llama family (K4 kernel without rotary + K1/K2).
"""

from __future__ import annotations

from typing import Iterable, List, Tuple

import torch
import torch.nn as nn

from ..config import ModelConfig
from ..ops import activation as act_ops
from ..ops.attention import AttentionMetadata, attention
from ..ops.rotary import rope_qkv_cache
from .layers import (ColumnParallelLinear, LayerNorm, ParallelLMHead, QKVParallelLinear,
                     ReplicatedLinear, RowParallelLinear, VocabParallelEmbedding, _param,
                     default_loader)


class OPTAttention(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype, device):
        super().__init__()
        H = cfg.hidden_size
        D = H // cfg.num_attention_heads
        self.qkv_proj = QKVParallelLinear(H, D, cfg.num_attention_heads, cfg.num_attention_heads,
                                          bias=True, dtype=dtype, device=device)
        self.out_proj = RowParallelLinear(H, H, bias=True, dtype=dtype, device=device)
        self.nh, self.nkv, self.hd = self.qkv_proj.num_heads, self.qkv_proj.num_kv_heads, D
        self.scale = D ** -0.5

    def forward(self, h, md: AttentionMetadata, kv):
        T = h.shape[0]
        qkv = self.qkv_proj(h)
        q = rope_qkv_cache(qkv, md.positions, None, md.slot_mapping, kv[0], kv[1], self.nh,
                           self.nkv, self.hd)
        o = attention(q, kv[0], kv[1], md, self.scale)
        return self.out_proj(o.reshape(T, self.nh * self.hd))


class OPTDecoderLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype, device):
        super().__init__()
        H = cfg.hidden_size
        self.pre_ln = cfg.do_layer_norm_before
        self.self_attn = OPTAttention(cfg, dtype, device)
        self.self_attn_layer_norm = LayerNorm(H, cfg.layer_norm_eps, dtype=dtype, device=device)
        self.fc1 = ColumnParallelLinear(H, cfg.intermediate_size, bias=True, dtype=dtype,
                                        device=device)
        self.fc2 = RowParallelLinear(cfg.intermediate_size, H, bias=True, dtype=dtype, device=device)
        self.final_layer_norm = LayerNorm(H, cfg.layer_norm_eps, dtype=dtype, device=device)
        self.act = cfg.hidden_act

    def forward(self, h, md, kv):
        r = h
        if self.pre_ln:
            h = self.self_attn_layer_norm(h)
        h = self.self_attn(h, md, kv) + r
        if not self.pre_ln:
            h = self.self_attn_layer_norm(h)
        r = h
        if self.pre_ln:
            h = self.final_layer_norm(h)
        h = self.fc2(act_ops.activation(self.fc1(h), self.act)) + r
        if not self.pre_ln:
            h = self.final_layer_norm(h)
        return h


class OPTForCausalLM(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        H = cfg.hidden_size
        E = cfg.word_embed_proj_dim or H
        self.embed_tokens = VocabParallelEmbedding(cfg.vocab_size, E, dtype, device)
        self.embed_positions = _param((cfg.max_position_embeddings + cfg.position_offset, H),
                                      dtype, device)
        self.embed_positions.weight_loader = default_loader
        self.project_in = ReplicatedLinear(E, H, dtype=dtype, device=device) if E != H else None
        self.project_out = ReplicatedLinear(H, E, dtype=dtype, device=device) if E != H else None
        self.layers = nn.ModuleList([OPTDecoderLayer(cfg, dtype, device)
                                     for _ in range(cfg.num_hidden_layers)])
        self.final_layer_norm = LayerNorm(H, cfg.layer_norm_eps, dtype=dtype, device=device) \
            if cfg.do_layer_norm_before else None
        self.lm_head = ParallelLMHead(cfg.vocab_size, E, dtype, device,
                                      tied=self.embed_tokens if cfg.tie_word_embeddings else None)

    def kv_heads_per_rank(self) -> int:
        return self.layers[0].self_attn.nkv

    def forward(self, input_ids, md: AttentionMetadata, kv_caches):
        h = self.embed_tokens(input_ids)
        if self.project_in is not None:
            h = self.project_in(h)
        pos = md.positions.long() + self.cfg.position_offset
        h = h + self.embed_positions[pos]
        for layer, kv in zip(self.layers, kv_caches):
            h = layer(h, md, kv)
        if self.final_layer_norm is not None:
            h = self.final_layer_norm(h)
        if self.project_out is not None:
            h = self.project_out(h)
        return h

    def compute_logits(self, h):
        return self.lm_head(h).float()

    def load_weights(self, weights: Iterable[Tuple[str, torch.Tensor]]) -> List[str]:
        params = dict(self.named_parameters())
        loaded = []
        for name, t in weights:
            n = name
            for p in ("model.decoder.", "decoder."):
                if n.startswith(p):
                    n = n[len(p):]
            sid = None
            for part, s in (("q_proj", "q"), ("k_proj", "k"), ("v_proj", "v")):
                if f".{part}." in n:
                    n, sid = n.replace(part, "qkv_proj"), s
            if n == "embed_positions.weight":
                n = "embed_positions"
            if n == "lm_head.weight" and self.cfg.tie_word_embeddings:
                continue
            if n not in params:
                continue
            p = params[n]
            loader = getattr(p, "weight_loader", default_loader)
            t = t.to(p.dtype)
            loader(p, t) if sid is None else loader(p, t, sid)
            loaded.append(n)
        return loaded
