"""Engine configuration objects.

The knobs mirror the vLLM flag subset that the reference's Helm values pass to
the serving container (e.g.
core/helm-charts/vllm/gaudi-values.yaml:160 ``--block-size 128 --max-num-seqs 288
--max-num-prefill-seqs 16 --dtype bfloat16 --max-model-len 33024``) so the same
``modelConfigs[*].extraCmdArgs`` strings drive this runtime.
"""

from __future__ import annotations

import dataclasses
import json
import math
import os
from typing import Any, Dict, Optional

import torch


_DTYPES = {
    "bfloat16": torch.bfloat16,
    "bf16": torch.bfloat16,
    "float16": torch.float16,
    "half": torch.float16,
    "fp16": torch.float16,
    "float32": torch.float32,
    "float": torch.float32,
    "fp32": torch.float32,
}


def parse_dtype(name: str | torch.dtype) -> torch.dtype:
    if isinstance(name, torch.dtype):
        return name
    if name in ("auto", None):
        return torch.bfloat16
    try:
        return _DTYPES[name.lower()]
    except KeyError as e:
        raise ValueError(f"unsupported dtype {name!r}") from e


@dataclasses.dataclass
class ModelConfig:
    """Architecture hyper-parameters (a normalised view over an HF config.json)."""

    architecture: str
    hidden_size: int
    num_hidden_layers: int
    num_attention_heads: int
    vocab_size: int
    intermediate_size: int = 0
    num_key_value_heads: Optional[int] = None
    head_dim: Optional[int] = None
    max_position_embeddings: int = 8192
    rms_norm_eps: float = 1e-5
    layer_norm_eps: float = 1e-12
    rope_theta: float = 10000.0
    rope_scaling: Optional[Dict[str, Any]] = None
    tie_word_embeddings: bool = False
    attention_bias: bool = False          # Qwen2: qkv bias
    qk_norm: bool = False                 # Qwen3: per-head RMSNorm on q and k
    hidden_act: str = "silu"
    # MoE
    num_local_experts: int = 0
    num_experts_per_tok: int = 0
    moe_intermediate_size: int = 0
    shared_expert_intermediate_size: int = 0
    norm_topk_prob: bool = True
    # Encoder / OPT specifics
    type_vocab_size: int = 0
    num_labels: int = 0
    do_layer_norm_before: bool = True
    word_embed_proj_dim: int = 0
    pad_token_id: int = 0
    bos_token_id: Optional[int] = None
    eos_token_id: Any = None
    position_offset: int = 0              # OPT learned positions are offset by 2
    sliding_window: Optional[int] = None
    # Llama-4 style chunked attention (text path)
    attention_chunk_size: Optional[int] = None
    name: str = ""
    extra: Dict[str, Any] = dataclasses.field(default_factory=dict)

    def __post_init__(self) -> None:
        if self.num_key_value_heads is None:
            self.num_key_value_heads = self.num_attention_heads
        if self.head_dim is None:
            self.head_dim = self.hidden_size // self.num_attention_heads

    @property
    def is_moe(self) -> bool:
        return self.num_local_experts > 0

    @property
    def is_encoder(self) -> bool:
        return self.architecture in ("BertModel", "XLMRobertaModel",
                                     "XLMRobertaForSequenceClassification",
                                     "BertForSequenceClassification")

    @property
    def q_size(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_key_value_heads * self.head_dim

    def num_params(self) -> int:
        """Approximate parameter count (decoder LLMs), used for sizing/logging."""
        h, L, v = self.hidden_size, self.num_hidden_layers, self.vocab_size
        attn = h * (self.q_size + 2 * self.kv_size) + self.q_size * h
        if self.is_moe:
            inter = self.moe_intermediate_size or self.intermediate_size
            mlp = self.num_local_experts * 3 * h * inter + h * self.num_local_experts
        else:
            mlp = 3 * h * self.intermediate_size
        emb = v * h * (1 if self.tie_word_embeddings else 2)
        return L * (attn + mlp + 2 * h) + emb

    @classmethod
    def from_hf_dict(cls, d: Dict[str, Any], name: str = "") -> "ModelConfig":
        arch = (d.get("architectures") or [d.get("model_type", "LlamaForCausalLM")])[0]
        text = d.get("text_config")
        outer = d
        if text is not None and "hidden_size" not in d:   # Llama-4 style nesting
            merged = dict(text)
            merged.setdefault("architectures", [arch])
            d = merged
        kw: Dict[str, Any] = dict(
            architecture=arch,
            hidden_size=d["hidden_size"],
            num_hidden_layers=d["num_hidden_layers"],
            num_attention_heads=d["num_attention_heads"],
            vocab_size=d["vocab_size"],
            intermediate_size=d.get("intermediate_size", d.get("ffn_dim", 0)),
            num_key_value_heads=d.get("num_key_value_heads"),
            head_dim=d.get("head_dim"),
            max_position_embeddings=d.get("max_position_embeddings", 8192),
            rms_norm_eps=d.get("rms_norm_eps", 1e-5),
            layer_norm_eps=d.get("layer_norm_eps", 1e-12),
            rope_theta=d.get("rope_theta", 10000.0),
            rope_scaling=d.get("rope_scaling"),
            tie_word_embeddings=d.get("tie_word_embeddings", False),
            attention_bias=d.get("attention_bias", arch.startswith("Qwen2")),
            qk_norm=arch.startswith("Qwen3"),
            hidden_act=d.get("hidden_act", d.get("activation_function", "silu")),
            num_local_experts=d.get("num_local_experts", d.get("num_experts", 0)) or 0,
            num_experts_per_tok=d.get("num_experts_per_tok", 0) or 0,
            moe_intermediate_size=d.get("moe_intermediate_size", 0) or 0,
            shared_expert_intermediate_size=d.get("shared_expert_intermediate_size", 0) or 0,
            norm_topk_prob=d.get("norm_topk_prob", True),
            type_vocab_size=d.get("type_vocab_size", 0),
            num_labels=len(d.get("id2label", {}) or {}) if "id2label" in d else d.get("num_labels", 0),
            do_layer_norm_before=d.get("do_layer_norm_before", True),
            word_embed_proj_dim=d.get("word_embed_proj_dim", 0) or 0,
            pad_token_id=d.get("pad_token_id", 0) or 0,
            bos_token_id=d.get("bos_token_id"),
            eos_token_id=d.get("eos_token_id"),
            sliding_window=d.get("sliding_window"),
            attention_chunk_size=d.get("attention_chunk_size"),
            name=name,
        )
        extra = {}
        L = d["num_hidden_layers"]
        if arch.startswith("Llama4"):
            # an explicit empty list is a real value (e.g. all-dense layers), not "unset"
            nrl = d.get("no_rope_layers")
            extra["no_rope_layers"] = nrl if nrl else [
                int((i + 1) % d.get("no_rope_layer_interval", 4) != 0) for i in range(L)]
            step = d.get("interleave_moe_layer_step", 1) or 1
            ml = d.get("moe_layers")
            extra["moe_layers"] = list(ml) if ml is not None else [
                i for i in range(L) if (i + 1) % step == 0]
            for key in ("use_qk_norm", "attn_temperature_tuning", "floor_scale", "attn_scale",
                        "intermediate_size_mlp"):
                if key in d:
                    extra[key] = d[key]
            extra["rope_interleaved"] = True
            if isinstance(outer.get("vision_config"), dict):    # multimodal checkpoint
                extra["vision_config"] = dict(outer["vision_config"])
                extra["image_token_id"] = outer.get("image_token_index",
                                                    outer.get("image_token_id", 200092))
        kw["extra"] = extra
        if arch.startswith("OPT"):
            kw["position_offset"] = 2
            kw["hidden_act"] = d.get("activation_function", "relu")
        if arch.startswith("XLMRoberta") or d.get("model_type") == "xlm-roberta":
            kw["position_offset"] = (d.get("pad_token_id", 1) or 1) + 1
        return cls(**kw)

    @classmethod
    def from_pretrained(cls, path: str) -> "ModelConfig":
        with open(os.path.join(path, "config.json")) as f:
            return cls.from_hf_dict(json.load(f), name=path)


@dataclasses.dataclass
class CacheConfig:
    block_size: int = 128                    # gaudi-values.yaml:160 --block-size 128
    gpu_memory_utilization: float = 0.90
    num_gpu_blocks: Optional[int] = None     # override (tests / bench)
    cpu_kvcache_space_gb: float = 4.0        # VLLM_CPU_KVCACHE_SPACE analogue
    swap_space_gb: float = 4.0               # --swap-space: pinned host KV for preemption
    enable_prefix_caching: bool = True
    cache_dtype: Optional[torch.dtype] = None   # None -> model dtype

    def __post_init__(self) -> None:
        if self.block_size % 16 != 0 or self.block_size <= 0:
            raise ValueError("block_size must be a positive multiple of 16 (MFMA tile)")


@dataclasses.dataclass
class SchedulerConfig:
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_num_prefill_seqs: int = 64
    max_model_len: int = 8192
    enable_chunked_prefill: bool = True
    # Decode batch-size bucket step for HIP-graph capture (VLLM_DECODE_BS_BUCKET_STEP).  8, not
    # the reference's Gaudi 32: a HIP graph captures in ~20 ms, and every padded row costs the
    # decode GEMMs X-staging bytes (65 users in the 72 bucket instead of 80: endpoint +1.3 %,
    # profiles/bucket_step_ab_r5.log)
    decode_bs_bucket_step: int = 8
    # overlapped scheduling: plan step k+1 while step k runs (VLLM_DELAYED_SAMPLING)
    delayed_sampling: bool = True


@dataclasses.dataclass
class ParallelConfig:
    tensor_parallel_size: int = 1
    pipeline_parallel_size: int = 1
    enable_expert_parallel: bool = False
    distributed_executor_backend: str = "mp"
    # Custom xGMI all-reduce (one-shot/two-shot) below this many bytes; RCCL above.
    custom_allreduce_max_bytes: int = 16 * 1024 * 1024
    disable_custom_all_reduce: bool = False
    # torch.distributed backend: "auto" = nccl (RCCL over xGMI) on GPUs, gloo on the CPU path
    dist_backend: str = "auto"
    # every TP rank on the driver's GPU (EIA_TP_SHARE_DEVICE=1): a rehearsal mode that runs
    # the TP engine's per-rank shapes on a one-GPU box.  RCCL refuses two ranks on one device,
    # so it implies gloo with host-staged collectives, eager decode and no custom all-reduce.
    share_device: bool = False

    def __post_init__(self) -> None:
        if os.environ.get("EIA_TP_SHARE_DEVICE", "0") not in ("0", "", "false"):
            self.share_device = True
        if self.share_device:
            self.dist_backend = "gloo"
            self.disable_custom_all_reduce = True

    @property
    def world_size(self) -> int:
        return self.tensor_parallel_size * self.pipeline_parallel_size


@dataclasses.dataclass
class EngineConfig:
    model: ModelConfig
    cache: CacheConfig = dataclasses.field(default_factory=CacheConfig)
    scheduler: SchedulerConfig = dataclasses.field(default_factory=SchedulerConfig)
    parallel: ParallelConfig = dataclasses.field(default_factory=ParallelConfig)
    dtype: torch.dtype = torch.bfloat16
    device: str = "cuda"
    model_path: Optional[str] = None         # None → random-init weights
    served_model_name: Optional[str] = None
    tokenizer: Optional[str] = None
    seed: int = 0
    enforce_eager: bool = False
    skip_warmup: bool = False                 # VLLM_SKIP_WARMUP: no warm-up runs before capture
    # servers with a real checkpoint: a missing / broken tokenizer is an error (no byte-level
    # stand-in); programmatic token-id-only use may leave it off
    strict_tokenizer: bool = False
    load_format: str = "auto"                 # auto | safetensors | dummy
    trust_remote_code: bool = False
    engine_iteration_timeout_s: float = 120.0  # VLLM_ENGINE_ITERATION_TIMEOUT_S

    def __post_init__(self) -> None:
        if self.device == "cuda" and self.dtype != torch.bfloat16:
            # the HIP kernels (attention, norms, GEMM epilogues, sampling) are bf16-only; any
            # other dtype would silently run the PyTorch reference ops on the GPU
            raise ValueError(f"dtype {self.dtype} is not supported on the MI355X path; serve "
                             "with --dtype bfloat16 (auto)")
        if self.load_format not in ("auto", "safetensors", "pt", "dummy"):
            raise ValueError(f"unknown load_format {self.load_format!r}")
        if self.device == "cuda" and self.parallel.world_size > 1 and (
                self.parallel.share_device or self.parallel.dist_backend == "gloo"):
            self.enforce_eager = True        # host-staged gloo collectives cannot be captured
        if self.cache.cache_dtype is None:
            self.cache.cache_dtype = self.dtype
        if self.scheduler.max_model_len > self.model.max_position_embeddings and \
                os.environ.get("VLLM_ALLOW_LONG_MAX_MODEL_LEN", "0") not in ("1", "true", "True"):
            # Match vLLM behaviour: clamp unless explicitly allowed.
            self.scheduler.max_model_len = self.model.max_position_embeddings
        if self.scheduler.max_num_batched_tokens < self.scheduler.max_num_seqs:
            self.scheduler.max_num_batched_tokens = self.scheduler.max_num_seqs

    @property
    def max_blocks_per_seq(self) -> int:
        return math.ceil(self.scheduler.max_model_len / self.cache.block_size)
