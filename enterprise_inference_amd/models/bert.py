"""Encoder models for the TEI-compatible servers.

* ``BertEmbeddingModel``  -- BAAI/bge-base-en-v1.5 (BertModel), served by the
  reference's ``tei`` chart (core/helm-charts/tei/values.yaml:20, port 2081):
  CLS pooling + L2 normalisation -> ``/embed``, ``/v1/embeddings``.
* ``CrossEncoderModel``  -- BAAI/bge-reranker-base (XLMRobertaForSequenceClassification),
  served by ``teirerank`` (core/helm-charts/teirerank/values.yaml:20, port 2082):
  classifier head on CLS -> ``/rerank`` scores.

Post-LN BERT blocks.  Attention reuses the decoder kernels: the fused K4 kernel
(no rotary) writes K/V of the batch into a scratch paged cache and the K2 prefill
kernel runs non-causally over it -- the same MFMA path as LLM prefill.
"""

from __future__ import annotations

from typing import Iterable, List, Optional, Tuple

import torch
import torch.nn as nn

from ..config import ModelConfig
from ..ops import activation as act_ops
from ..ops import attention as attn_ops
from ..ops import norm as norm_ops
from ..ops import reference as ref
from ..ops.rotary import rope_qkv_cache
from .layers import LayerNorm, ReplicatedLinear, _param, default_loader

_ENC_BLOCK = 128


class EncoderBatch:
    """Packed varlen batch: tokens of all sequences back to back."""

    def __init__(self, seqs: List[List[int]], type_ids: Optional[List[List[int]]], device,
                 position_offset: int = 0):
        lens = [len(s) for s in seqs]
        self.num_seqs = len(seqs)
        self.lens = lens
        self.ids = torch.tensor([t for s in seqs for t in s], dtype=torch.long, device=device)
        tt = [t for s in (type_ids or [[0] * n for n in lens]) for t in s]
        self.type_ids = torch.tensor(tt, dtype=torch.long, device=device)
        self.positions = torch.tensor([position_offset + i for n in lens for i in range(n)],
                                      dtype=torch.long, device=device)
        cu = [0]
        for n in lens:
            cu.append(cu[-1] + n)
        self.cu = cu
        self.cu_t = torch.tensor(cu, dtype=torch.int32, device=device)
        self.first_idx = torch.tensor(cu[:-1], dtype=torch.long, device=device)
        # scratch paged layout: each sequence starts on its own block
        bs = _ENC_BLOCK
        nblk = [(n + bs - 1) // bs for n in lens]
        starts = [0]
        for b in nblk:
            starts.append(starts[-1] + b)
        self.num_blocks = max(1, starts[-1])
        maxb = max(1, max(nblk) if nblk else 1)
        bt = [[starts[s] + j if j < nblk[s] else 0 for j in range(maxb)] for s in range(len(lens))]
        self.block_tables = torch.tensor(bt, dtype=torch.int32, device=device)
        self.slots = torch.tensor([starts[s] * bs + i for s, n in enumerate(lens) for i in range(n)],
                                  dtype=torch.int32, device=device)
        self.seq_lens = torch.tensor(lens, dtype=torch.int32, device=device)


class BertLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype, device):
        super().__init__()
        H = cfg.hidden_size
        self.nh = cfg.num_attention_heads
        self.hd = H // self.nh
        self.qkv = ReplicatedLinear(H, 3 * H, bias=True, dtype=dtype, device=device)
        self.o = ReplicatedLinear(H, H, bias=True, dtype=dtype, device=device)
        self.ln1 = LayerNorm(H, cfg.layer_norm_eps, dtype=dtype, device=device)
        self.up = ReplicatedLinear(H, cfg.intermediate_size, bias=True, dtype=dtype, device=device)
        self.down = ReplicatedLinear(cfg.intermediate_size, H, bias=True, dtype=dtype, device=device)
        self.ln2 = LayerNorm(H, cfg.layer_norm_eps, dtype=dtype, device=device)
        self.act = "gelu" if cfg.hidden_act in ("gelu", "gelu_erf") else cfg.hidden_act

    def attention(self, qkv: torch.Tensor, b: EncoderBatch) -> torch.Tensor:
        T = qkv.shape[0]
        nh, hd = self.nh, self.hd
        scale = hd ** -0.5
        if qkv.is_cuda and qkv.dtype == torch.bfloat16:
            kc = torch.empty(b.num_blocks, nh, _ENC_BLOCK, hd, dtype=qkv.dtype, device=qkv.device)
            vc = torch.zeros(b.num_blocks, nh, hd, _ENC_BLOCK, dtype=qkv.dtype, device=qkv.device)
            q = rope_qkv_cache(qkv, None, None, b.slots, kc, vc, nh, nh, hd)
            qb = attn_ops.prefill_query_block(nh, nh, hd, block_size=_ENC_BLOCK)
            work = attn_ops.build_prefill_work(b.lens, qb)
            wt = torch.tensor(work, dtype=torch.int32, device=qkv.device)
            o = attn_ops.paged_prefill(q, kc, vc, b.block_tables, b.seq_lens, b.cu_t, wt,
                                       len(work) // 2, scale, causal=False)
            return o.view(T, nh * hd)
        q, k, v = qkv.view(T, 3, nh, hd).unbind(1)
        return ref.attention_varlen(q, k, v, b.cu_t, scale, causal=False).reshape(T, nh * hd)

    def forward(self, h: torch.Tensor, b: EncoderBatch) -> torch.Tensor:
        a = self.o(self.attention(self.qkv(h), b))
        h = self.ln1(a, residual=h)           # LN(h + attn)
        f = self.down(act_ops.activation(self.up(h), self.act))
        return self.ln2(f, residual=h)        # LN(h + ffn)


class BertEncoder(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        H = cfg.hidden_size
        self.word = _param((cfg.vocab_size, H), dtype, device)
        self.pos = _param((cfg.max_position_embeddings, H), dtype, device)
        self.type_emb = _param((max(1, cfg.type_vocab_size), H), dtype, device)
        for p in (self.word, self.pos, self.type_emb):
            p.weight_loader = default_loader
        self.emb_ln = LayerNorm(H, cfg.layer_norm_eps, dtype=dtype, device=device)
        self.layers = nn.ModuleList([BertLayer(cfg, dtype, device)
                                     for _ in range(cfg.num_hidden_layers)])

    def forward(self, b: EncoderBatch) -> torch.Tensor:
        x = self.word[b.ids] + self.pos[b.positions] + self.type_emb[b.type_ids]
        h = self.emb_ln(x)
        for layer in self.layers:
            h = layer(h, b)
        return h

    # HF names -> ours
    def load_encoder_weights(self, weights: Iterable[Tuple[str, torch.Tensor]], prefix_drop=()):
        params = dict(self.named_parameters())
        qkv_parts = {}
        loaded = []
        for name, t in weights:
            for p in prefix_drop:
                if name.startswith(p):
                    name = name[len(p):]
            m = self._map(name)
            if m is None:
                continue
            tgt, part = m
            if part is not None:   # q/k/v pieces of the fused projection
                qkv_parts.setdefault(tgt, {})[part] = t
                if len(qkv_parts[tgt]) == 3:
                    d = qkv_parts.pop(tgt)
                    params[tgt].data.copy_(torch.cat([d["q"], d["k"], d["v"]], 0).to(params[tgt].dtype))
                    loaded.append(tgt)
                continue
            if tgt in params:
                params[tgt].data.copy_(t.to(params[tgt].dtype))
                loaded.append(tgt)
        return loaded

    @staticmethod
    def _map(name: str):
        simple = {"embeddings.word_embeddings.weight": "word",
                  "embeddings.position_embeddings.weight": "pos",
                  "embeddings.token_type_embeddings.weight": "type_emb",
                  "embeddings.LayerNorm.weight": "emb_ln.weight",
                  "embeddings.LayerNorm.bias": "emb_ln.bias"}
        if name in simple:
            return simple[name], None
        if not name.startswith("encoder.layer."):
            return None
        rest = name[len("encoder.layer."):]
        i, _, sub = rest.partition(".")
        base = f"layers.{i}."
        for hf, part in (("attention.self.query.", "q"), ("attention.self.key.", "k"),
                         ("attention.self.value.", "v")):
            if sub.startswith(hf):
                return base + "qkv." + sub[len(hf):], part
        table = {"attention.output.dense.": "o.", "attention.output.LayerNorm.": "ln1.",
                 "intermediate.dense.": "up.", "output.dense.": "down.",
                 "output.LayerNorm.": "ln2."}
        for hf, ours in table.items():
            if sub.startswith(hf):
                return base + ours + sub[len(hf):], None
        return None


class BertEmbeddingModel(nn.Module):
    """Sentence embeddings: CLS (default) or mean pooling, optional L2 normalisation."""

    is_encoder = True

    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None, pooling: str = "cls"):
        super().__init__()
        self.cfg = cfg
        self.encoder = BertEncoder(cfg, dtype, device)
        self.pooling = pooling

    def forward(self, b: EncoderBatch, normalize: bool = True) -> torch.Tensor:
        h = self.encoder(b)
        if self.pooling == "mean":
            pooled = torch.stack([h[b.cu[i]:b.cu[i + 1]].float().mean(0)
                                  for i in range(b.num_seqs)])
        else:
            pooled = h.index_select(0, b.first_idx).float()
        if normalize:
            pooled = torch.nn.functional.normalize(pooled, dim=-1)
        return pooled

    def load_weights(self, weights):
        return self.encoder.load_encoder_weights(weights, prefix_drop=("bert.", "roberta.", "model."))


class CrossEncoderModel(nn.Module):
    """Sequence-pair classifier (reranker): dense -> tanh -> out_proj on the CLS token."""

    is_encoder = True

    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.cfg = cfg
        self.encoder = BertEncoder(cfg, dtype, device)
        H = cfg.hidden_size
        nl = max(1, cfg.num_labels)
        self.roberta_head = cfg.architecture.startswith("XLMRoberta")
        self.dense = ReplicatedLinear(H, H, bias=True, dtype=dtype, device=device)
        self.out_proj = ReplicatedLinear(H, nl, bias=True, dtype=dtype, device=device)

    def forward(self, b: EncoderBatch) -> torch.Tensor:
        h = self.encoder(b)
        cls = h.index_select(0, b.first_idx)
        x = torch.tanh(self.dense(cls).float()).to(cls.dtype)
        return self.out_proj(x).float()            # [num_seqs, num_labels] logits

    def load_weights(self, weights):
        head = []
        rest = []
        for n, t in weights:
            if ".pooler.dense." in n or n.startswith("pooler.dense."):
                head.append(("classifier.dense." + n.split("pooler.dense.")[1], t))
            elif n.startswith("classifier."):
                head.append((n, t))
            else:
                rest.append((n, t))
        loaded = self.encoder.load_encoder_weights(rest, prefix_drop=("bert.", "roberta.", "model."))
        params = dict(self.named_parameters())
        for n, t in head:
            key = n.replace("classifier.", "")
            if key.startswith("out_proj.") or key.startswith("dense."):
                params[key].data.copy_(t.to(params[key].dtype))
            elif key in ("weight", "bias"):        # BertForSequenceClassification: plain Linear
                params["out_proj." + key].data.copy_(t.to(params["out_proj." + key].dtype))
            loaded.append(key)
        return loaded
