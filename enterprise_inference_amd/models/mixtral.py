"""Mixture-of-experts decoders (Mixtral-8x7B #9, Llama-4-Scout #5;
plus Qwen2-MoE / Qwen3-MoE).

* ``MixtralForCausalLM``  softmax top-2 routing over 8 SwiGLU experts
  (core/helm-charts/vllm/gaudi-values.yaml:354-375); also Qwen3-MoE
  (``norm_topk_prob``) and Qwen2-MoE (+ gated shared expert).
* ``Llama4ForCausalLM``   text path of Llama-4-Scout-17B-16E
  (core/helm-charts/vllm/gaudi-values.yaml:258-278, gaudi3-values.yaml:492-501):
  sigmoid top-1 routing applied to the expert *input*, a shared expert, chunked
  local attention (8192) on RoPE layers, GPT-J-style (interleaved) RoPE, weightless
  QK L2-norm on RoPE layers, NoPE every 4th layer with attention temperature tuning.

Experts live in one ``FusedMoE`` module ([E, 2I, H] / [E, H, I] tensors, K9 kernels in
ops/moe.py).  Tensor parallel shards each expert's I; ``--enable-expert-parallel``
instead gives each rank E/tp whole experts (the reference's EP on Gaudi 3,
``VLLM_EP_SIZE``); either way the layer output is all-reduced over the TP group.
"""

from __future__ import annotations

import math
import os
from typing import Iterable, List, Optional, Tuple

import torch
import torch.nn as nn

from ..config import ModelConfig
from ..ops import moe as moe_ops
from ..parallel import comm, state
from .layers import (MergedColumnParallelLinear, PendingAllReduce, ReplicatedLinear,
                     RowParallelLinear, _param)


def _deferred_reduce(out: torch.Tensor):
    """TP>1: hand the MoE partial sums to the next add+RMSNorm (fused xGMI all-reduce)."""
    return PendingAllReduce(out) if state.tp_size() > 1 else out
from .llama import LlamaAttention, LlamaDecoderLayer, LlamaForCausalLM, LlamaMLP


class FusedMoE(nn.Module):
    def __init__(self, num_experts: int, top_k: int, hidden: int, inter: int,
                 renormalize: bool = True, scoring: str = "softmax", scale_input: bool = False,
                 dtype=torch.bfloat16, device=None):
        super().__init__()
        tp, r = state.tp_size(), state.tp_rank()
        self.E, self.k, self.H = num_experts, top_k, hidden
        self.ep = state.ep_enabled()
        if self.ep:
            if num_experts % tp:
                raise ValueError("num_experts must be divisible by the EP size")
            self.e_per = num_experts // tp
            self.e_lo = r * self.e_per
            self.I_local = inter
        else:
            self.e_per, self.e_lo = num_experts, 0
            if inter % tp:
                raise ValueError("moe intermediate size must be divisible by tp")
            self.I_local = inter // tp
        self.I = inter
        self.renormalize, self.scoring, self.scale_input = renormalize, scoring, scale_input
        self.w13 = _param((self.e_per, 2 * self.I_local, hidden), dtype, device)
        self.w2 = _param((self.e_per, hidden, self.I_local), dtype, device)
        self.w13.weight_loader = self._load_w13
        self.w2.weight_loader = self._load_w2

    # shard helpers: loaded tensors are full [I, H] / [H, I] per expert
    def _local(self, expert: int) -> Optional[int]:
        e = expert - self.e_lo
        return e if 0 <= e < self.e_per else None

    def _ishard(self, t: torch.Tensor, dim: int) -> torch.Tensor:
        if self.ep or state.tp_size() == 1:
            return t
        n = self.I_local
        return t.narrow(dim, state.tp_rank() * n, n)

    def _load_w13(self, param, loaded, shard_id):
        expert, which = shard_id               # which: "w1" (gate) | "w3" (up) | "w13"
        e = self._local(expert)
        if e is None:
            return
        if which == "w13":                     # fused [2I, H] (gate rows then up rows)
            g, u = loaded.chunk(2, dim=0)
            param.data[e, :self.I_local].copy_(self._ishard(g, 0))
            param.data[e, self.I_local:].copy_(self._ishard(u, 0))
            return
        off = 0 if which == "w1" else self.I_local
        param.data[e, off:off + self.I_local].copy_(self._ishard(loaded, 0))

    def _load_w2(self, param, loaded, shard_id):
        expert, _ = shard_id
        e = self._local(expert)
        if e is not None:
            param.data[e].copy_(self._ishard(loaded, 1))

    def forward(self, x: torch.Tensor, router_logits: Optional[torch.Tensor] = None,
                reduce: bool = True, router_w: Optional[torch.Tensor] = None,
                routing: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                defer_combine: bool = False):
        if routing is not None:       # routed by the preceding norm (MixtralMoE.norm_and_route)
            w, ids = routing
        elif router_logits is None:   # fused router GEMM + top-k
            w, ids = moe_ops.route(x, router_w, self.k, self.renormalize, self.scoring)
        else:
            w, ids = moe_ops.topk_route(router_logits, self.k, self.renormalize, self.scoring)
        if self.scale_input:
            # Llama-4 applies the routing score to the expert input (k = 1), as the reference
            # model does: bf16 score x bf16 activation (one elementwise launch)
            x = x * w[:, :1].to(x.dtype)
            w = self._unit_weights(w)
        if self.a2a:
            from ..parallel.expert_parallel import moe_all_to_all_replicated
            return moe_all_to_all_replicated(x, w, ids, self.w13, self.w2, self.e_lo,
                                             self.e_per, state.tp_group())
        out = moe_ops.fused_moe(x, self.w13, self.w2, w, ids,
                                (self.e_lo, self.e_lo + self.e_per) if self.ep else None,
                                defer_combine=defer_combine and not (reduce and
                                                                     state.tp_size() > 1))
        if reduce and state.tp_size() > 1:
            out = comm.all_reduce(out)
        return out

    def _unit_weights(self, w: torch.Tensor) -> torch.Tensor:
        """All-ones routing weights shaped like ``w``: a slice of a cached buffer (no fill
        launch per layer and step), grown outside graph capture only."""
        buf = getattr(self, "_ones", None)
        if (buf is None or buf.device != w.device or buf.shape[0] < w.shape[0]
                or buf.shape[1] != w.shape[1]):
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                return torch.ones_like(w)
            buf = torch.ones(max(256, w.shape[0]), w.shape[1], dtype=w.dtype, device=w.device)
            self._ones = buf
        return buf[:w.shape[0]]

    @property
    def a2a(self) -> bool:
        """All-to-all EP: the output comes back complete (no all-reduce follows).  Llama-4
        (routing score applied to the expert input, shared expert summed before one
        all-reduce) keeps the all-reduce form."""
        return self.ep and not self.scale_input and state.ep_dispatch() == "all_to_all"


class MixtralMoE(nn.Module):
    """block_sparse_moe (Mixtral) / mlp (Qwen-MoE): router + FusedMoE [+ shared expert]."""

    def __init__(self, cfg: ModelConfig, dtype, device):
        super().__init__()
        H = cfg.hidden_size
        inter = cfg.moe_intermediate_size or cfg.intermediate_size
        self.gate = ReplicatedLinear(H, cfg.num_local_experts, dtype=dtype, device=device)
        renorm = cfg.norm_topk_prob if cfg.architecture.startswith("Qwen") else True
        self.experts = FusedMoE(cfg.num_local_experts, cfg.num_experts_per_tok, H, inter, renorm,
                                dtype=dtype, device=device)
        self.shared_expert = None
        if cfg.shared_expert_intermediate_size:
            self.shared_expert = LlamaMLP(H, cfg.shared_expert_intermediate_size, "silu", dtype,
                                          device)
            self.shared_expert.down_proj.reduce_results = False   # one all-reduce for the sum
            self.shared_expert_gate = ReplicatedLinear(H, 1, dtype=dtype, device=device)

    def norm_and_route(self, h, residual, norm, md=None):
        """Decode: the O projection's split-K add + RMSNorm (``norm``) with this block's router
        and top-k in the same launch -> (x, residual, routing), or None when not applicable.
        A pure-decode batch on one rank (``md``) routes its bucket-padding rows (context 0) to
        no expert."""
        ex = self.experts
        if (self.gate.bias is not None or ex.scale_input or
                not moe_ops.splitk_norm_route_ok(h, residual, self.gate.weight, ex.k)):
            return None
        row_len = None
        if (md is not None and md.num_prefill_tokens == 0 and md.decode_seq_lens is not None
                and md.num_decode == h.M and state.tp_size() == 1 and not ex.ep):
            row_len = md.decode_seq_lens
        return moe_ops.splitk_norm_route(h, residual, norm.weight, norm.eps, self.gate.weight,
                                         ex.k, ex.renormalize, ex.scoring, row_len=row_len)

    def forward(self, x, routing=None):
        # one rank, no shared expert: the combine may be left to the next add + RMSNorm
        defer = self.shared_expert is None and state.tp_size() == 1
        if routing is not None:
            out = self.experts(x, None, reduce=False, routing=routing, defer_combine=defer)
        elif self.gate.bias is None and x.dim() == 2:
            out = self.experts(x, None, reduce=False, router_w=self.gate.weight,
                               defer_combine=defer)
        else:
            out = self.experts(x, self.gate(x), reduce=False)
        a2a = self.experts.a2a          # all-to-all EP: `out` is already complete
        if self.shared_expert is not None:
            s = self.shared_expert(x)
            s = s.materialize() if hasattr(s, "materialize") else s
            if a2a:
                s = comm.all_reduce(s)
            out = out + torch.sigmoid(self.shared_expert_gate(x).float()).to(x.dtype) * s
        if a2a:
            return out
        return _deferred_reduce(out)


class MixtralForCausalLM(LlamaForCausalLM):
    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None):
        super().__init__(cfg, dtype, device, layer_factory=lambda i: LlamaDecoderLayer(
            cfg, i, self.rotary, dtype, device, mlp=MixtralMoE(cfg, dtype, device)))

    def map_weight_name(self, name: str):
        n = name.replace("model.", "", 1) if name.startswith("model.") else name
        n = n.replace("block_sparse_moe.", "mlp.")
        if n.endswith(".mlp.experts.gate_up_proj"):      # transformers>=5 stacked [E, 2I, H]
            return n.replace("experts.gate_up_proj", "experts.w13"), "stacked"
        if n.endswith(".mlp.experts.down_proj"):         # stacked [E, H, I]
            return n.replace("experts.down_proj", "experts.w2"), "stacked"
        if ".mlp.experts." in n:
            pre, rest = n.split(".mlp.experts.", 1)
            e, _, w = rest.partition(".")
            which = {"w1": "w1", "w3": "w3", "w2": "w2", "gate_proj": "w1", "up_proj": "w3",
                     "down_proj": "w2"}[w.split(".")[0]]
            tgt = f"{pre}.mlp.experts.{'w2' if which == 'w2' else 'w13'}"
            return tgt, (int(e), which)
        if ".mlp.shared_expert." in n:
            for part, sid in (("gate_proj", 0), ("up_proj", 1)):
                if f".{part}." in n:
                    return n.replace(part, "gate_up_proj"), sid
            return n, None
        return super().map_weight_name(name)

    def load_weights(self, weights: Iterable[Tuple[str, torch.Tensor]]) -> List[str]:
        return _load_with_stacked_experts(self, weights, super().load_weights)


def _load_with_stacked_experts(model, weights, base_load):
    """Route stacked expert tensors ([E, out, in], or [E, in, out] = "fused_t") through the
    FusedMoE loaders (which shard per rank); everything else through ``base_load``."""
    params = dict(model.named_parameters())
    rest, loaded = [], []
    for name, t in weights:
        pname, sid = model.map_weight_name(name)
        if sid in ("stacked", "fused_t"):
            if pname not in params:          # layer of another pipeline stage
                continue
            p = params[pname]
            kind = "w13" if pname.endswith("w13") else "w2"
            for e in range(t.shape[0]):
                te = t[e].t() if sid == "fused_t" else t[e]
                p.weight_loader(p, te.to(p.dtype), (e, kind))
            loaded.append(pname)
        elif pname != "__skip__":
            rest.append((name, t))
    return loaded + base_load(rest)


# ----------------------------------------------------------------------------- Llama-4


class Llama4Attention(LlamaAttention):
    def __init__(self, cfg: ModelConfig, idx: int, rotary, dtype, device):
        super().__init__(cfg, idx, rotary, dtype, device)
        ex = cfg.extra
        nope = ex.get("no_rope_layers")
        self.use_rope = bool(nope[idx]) if nope else True
        if not self.use_rope:
            self.rotary = None
            self.chunk_size = None
        else:
            self.chunk_size = cfg.attention_chunk_size
        self.qk_l2 = bool(ex.get("use_qk_norm", True)) and self.use_rope
        self.temp_tuning = bool(ex.get("attn_temperature_tuning", True)) and not self.use_rope
        self.floor_scale = float(ex.get("floor_scale", 8192))
        self.attn_scale = float(ex.get("attn_scale", 0.1))
        D = cfg.head_dim
        if self.qk_l2:   # weightless L2 norm == RMSNorm with unit weight (rotation-invariant)
            self.register_buffer("ones", torch.ones(D, dtype=dtype, device=device),
                                 persistent=False)

    def forward(self, h, md, kv):
        from ..ops.attention import attention
        from ..ops.rotary import rope_qkv_cache
        from ..ops import gemm

        T = h.shape[0]
        # split-K QKV slabs are summed inside the RoPE / KV-write kernel (no reduce launch)
        qkv = gemm.linear(h, self.qkv_proj.weight, defer_reduce=True)
        q = rope_qkv_cache(qkv, md.positions, self.rotary, md.slot_mapping, kv[0], kv[1],
                           self.num_heads, self.num_kv_heads, self.head_dim,
                           bias=self.qkv_proj.bias,
                           q_norm_w=self.ones if self.qk_l2 else None,
                           k_norm_w=self.ones if self.qk_l2 else None,
                           norm_eps=self.cfg.rms_norm_eps)
        if self.temp_tuning:
            # the per-position temperature is the same for every NoPE layer of the step:
            # computed once per step (cached on the step's metadata), applied in fp32
            key = (self.floor_scale, self.attn_scale)
            cached = getattr(md, "_l4_attn_temp", None)
            if cached is None or cached[0] != key:
                pos = md.positions.float()
                sc = torch.log1p(torch.floor((pos + 1.0) / self.floor_scale)) * self.attn_scale \
                    + 1.0
                cached = (key, sc[:, None, None])
                md._l4_attn_temp = cached
            q = (q * cached[1]).to(q.dtype)
        o = attention(q, kv[0], kv[1], md, self.scale, None, self.chunk_size)
        return self.o_proj(o.view(T, self.num_heads * self.head_dim), defer_reduce=True)


class Llama4MoE(nn.Module):
    def __init__(self, cfg: ModelConfig, dtype, device):
        super().__init__()
        H = cfg.hidden_size
        self.router = ReplicatedLinear(H, cfg.num_local_experts, dtype=dtype, device=device)
        self.experts = FusedMoE(cfg.num_local_experts, cfg.num_experts_per_tok, H,
                                cfg.intermediate_size, renormalize=False, scoring="sigmoid",
                                scale_input=True, dtype=dtype, device=device)
        self.shared_expert = LlamaMLP(H, cfg.intermediate_size, "silu", dtype, device)
        self.shared_expert.down_proj.reduce_results = False   # one all-reduce for the sum

    def forward(self, x):
        if self.router.bias is None and x.dim() == 2:
            # router GEMM + sigmoid top-1 in one kernel (moe.hip route_kernel)
            routed = self.experts(x, None, reduce=False, router_w=self.router.weight)
        else:
            routed = self.experts(x, self.router(x), reduce=False)
        s = self.shared_expert.down_proj(self.shared_expert.gate_up_proj.forward_act_and_mul(x))
        return _deferred_reduce(routed + s)


class Llama4ForCausalLM(LlamaForCausalLM):
    def __init__(self, cfg: ModelConfig, dtype=torch.bfloat16, device=None):
        cfg.extra.setdefault("rope_interleaved", True)
        ml = cfg.extra.get("moe_layers")
        moe_layers = set(range(cfg.num_hidden_layers) if ml is None else ml)
        inter_mlp = cfg.extra.get("intermediate_size_mlp") or cfg.intermediate_size

        def make(i):
            mlp = Llama4MoE(cfg, dtype, device) if i in moe_layers else \
                LlamaMLP(cfg.hidden_size, inter_mlp, "silu", dtype, device)
            layer = LlamaDecoderLayer(cfg, i, self.rotary, dtype, device, mlp=mlp)
            layer.self_attn = Llama4Attention(cfg, i, self.rotary, dtype, device)
            return layer

        super().__init__(cfg, dtype, device, layer_factory=make)
        self.vision = None
        vc = cfg.extra.get("vision_config")
        if vc and os.environ.get("EIA_DISABLE_VISION", "0") != "1" and self.first:
            from .llama4_vision import Llama4VisionTower
            self.vision = Llama4VisionTower(vc, cfg.hidden_size, dtype, device)
            self.image_token_id = int(cfg.extra.get("image_token_id", 200092))

    def encode_images(self, pixel_values: torch.Tensor) -> torch.Tensor:
        """[tiles, 3, S, S] -> [tiles * 144, hidden] placeholder embeddings."""
        if self.vision is None:
            raise ValueError("this model was loaded without its vision tower")
        return self.vision(pixel_values)

    def map_weight_name(self, name: str):
        n = name
        for p in ("language_model.model.", "language_model.", "model."):
            if n.startswith(p):
                n = n[len(p):]
                break
        if n.startswith("vision_model") or n.startswith("multi_modal_projector"):
            return "__skip__", None
        n = n.replace(".feed_forward.", ".mlp.")
        if ".mlp.experts.gate_up_proj" in n:
            return n.replace("experts.gate_up_proj", "experts.w13"), "fused_t"
        if ".mlp.experts.down_proj" in n:
            return n.replace("experts.down_proj", "experts.w2"), "fused_t"
        if ".mlp.shared_expert." in n:
            for part, sid in (("gate_proj", 0), ("up_proj", 1)):
                if f".{part}." in n:
                    return n.replace(part, "gate_up_proj"), sid
            return n, None
        # dense (non-MoE) layers: feed_forward.{gate,up,down}_proj -> mlp.gate_up_proj / down_proj
        return super().map_weight_name(n)

    def load_weights(self, weights: Iterable[Tuple[str, torch.Tensor]]) -> List[str]:
        strip = lambda n: n[len("language_model."):] if n.startswith("language_model.") else n
        vis_loaded: List[str] = []

        def text_only(ws):
            for n, t in ws:
                m = n[len("model."):] if n.startswith("model.vision_model") or \
                    n.startswith("model.multi_modal_projector") else n
                if m.startswith(("vision_model.", "multi_modal_projector.")):
                    if self.vision is not None and self.vision.load_weight(m, t):
                        vis_loaded.append(n)
                    continue
                yield n, t

        loaded = _load_with_stacked_experts(
            self, text_only(weights), lambda rest: super(Llama4ForCausalLM, self).load_weights(
                (strip(n), t) for n, t in rest))
        return list(loaded) + vis_loaded
