"""Built-in architecture presets for every model in the reference catalog.

The reference deploys models by menu number -> canonical name -> HF id
(core/lib/models/model-selection.sh:26-68, :105-258).  With no
network, the serving runtime cannot fetch config.json, so the public HF configs
of those models are embedded here [ext: public model cards].  Weights are random
unless a local checkpoint directory is given.
"""

from __future__ import annotations

import copy
from typing import Dict

_LLAMA31_ROPE = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                 "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}


def _llama(h, inter, layers, heads, kv, **kw):
    d = {"architectures": ["LlamaForCausalLM"], "hidden_size": h, "intermediate_size": inter,
         "num_hidden_layers": layers, "num_attention_heads": heads, "num_key_value_heads": kv,
         "vocab_size": 128256, "max_position_embeddings": 131072, "rms_norm_eps": 1e-5,
         "rope_theta": 500000.0, "rope_scaling": dict(_LLAMA31_ROPE), "tie_word_embeddings": False,
         "bos_token_id": 128000, "eos_token_id": [128001, 128008, 128009], "hidden_act": "silu"}
    d.update(kw)
    return d


def _qwen2(h, inter, layers, heads, kv, vocab=152064, **kw):
    d = {"architectures": ["Qwen2ForCausalLM"], "hidden_size": h, "intermediate_size": inter,
         "num_hidden_layers": layers, "num_attention_heads": heads, "num_key_value_heads": kv,
         "vocab_size": vocab, "max_position_embeddings": 32768, "rms_norm_eps": 1e-6,
         "rope_theta": 1000000.0, "attention_bias": True, "tie_word_embeddings": False,
         "bos_token_id": 151643, "eos_token_id": 151645, "hidden_act": "silu"}
    d.update(kw)
    return d


def _qwen3(h, inter, layers, heads, kv, **kw):
    d = {"architectures": ["Qwen3ForCausalLM"], "hidden_size": h, "intermediate_size": inter,
         "num_hidden_layers": layers, "num_attention_heads": heads, "num_key_value_heads": kv,
         "head_dim": 128, "vocab_size": 151936, "max_position_embeddings": 40960,
         "rms_norm_eps": 1e-6, "rope_theta": 1000000.0, "tie_word_embeddings": True,
         "bos_token_id": 151643, "eos_token_id": 151645, "hidden_act": "silu"}
    d.update(kw)
    return d


PRESETS: Dict[str, dict] = {
    "meta-llama/Llama-3.1-8B-Instruct": _llama(4096, 14336, 32, 32, 8),
    "meta-llama/Meta-Llama-3-8B-Instruct": _llama(4096, 14336, 32, 32, 8, rope_scaling=None,
                                                  max_position_embeddings=8192),
    "meta-llama/Llama-3.1-70B-Instruct": _llama(8192, 28672, 80, 64, 8),
    "meta-llama/Llama-3.3-70B-Instruct": _llama(8192, 28672, 80, 64, 8),
    "meta-llama/Meta-Llama-3-70B-Instruct": _llama(8192, 28672, 80, 64, 8, rope_scaling=None,
                                                   max_position_embeddings=8192),
    "meta-llama/Llama-3.1-405B-Instruct": _llama(16384, 53248, 126, 128, 8),
    # ONE tensor-parallel rank of Llama-3.3-70B at TP 8 (BASELINE config #3, reference
    # core/playbooks/deploy-inference-models.yml:1884): 8 q / 1 kv heads x 128, I 3584, the
    # vocab-parallel LM head's 16032 rows.  Served at TP 1 it runs exactly the rank's decode
    # GEMMs, attention and norms -- everything but the all-reduces -- so the per-rank step can be
    # profiled on one GPU (scripts/gpu_model_steps.sh).  A profiling proxy, not a real model.
    "eia/Llama-3.3-70B-TP8-rank": _llama(8192, 3584, 80, 8, 1, head_dim=128, vocab_size=16032,
                                         bos_token_id=1, eos_token_id=[2]),
    # ONE rank of Llama-3.1-405B at TP 8 (the reference's 405B deployment,
    # core/playbooks/deploy-inference-models.yml:1884; sizing-guide.md:82-89): 16 q / 1 kv heads
    # x 128, I 6656, 126 layers, LM head 16032 rows -- ~101 GB, the same per-rank profiling proxy.
    "eia/Llama-3.1-405B-TP8-rank": _llama(16384, 6656, 126, 16, 1, head_dim=128, vocab_size=16032,
                                          bos_token_id=1, eos_token_id=[2]),
    "meta-llama/Llama-3.2-3B-Instruct": _llama(3072, 8192, 28, 24, 8, tie_word_embeddings=True,
                                               rope_scaling={**_LLAMA31_ROPE, "factor": 32.0}),
    "deepseek-ai/DeepSeek-R1-Distill-Llama-8B": _llama(4096, 14336, 32, 32, 8,
                                                      eos_token_id=128001),
    "codellama/CodeLlama-34b-Instruct-hf": _llama(8192, 22016, 48, 64, 8, vocab_size=32000,
                                                  max_position_embeddings=16384,
                                                  rope_theta=1000000.0, rope_scaling=None,
                                                  bos_token_id=1, eos_token_id=2),
    "tiiuae/Falcon3-7B-Instruct": _llama(3072, 23040, 28, 12, 4, head_dim=256, vocab_size=131072,
                                         max_position_embeddings=32768, rope_theta=1000042.0,
                                         rope_scaling=None, rms_norm_eps=1e-6, bos_token_id=11,
                                         eos_token_id=11),
    "mistralai/Mistral-7B-Instruct-v0.3": {
        "architectures": ["MistralForCausalLM"], "hidden_size": 4096, "intermediate_size": 14336,
        "num_hidden_layers": 32, "num_attention_heads": 32, "num_key_value_heads": 8,
        "vocab_size": 32768, "max_position_embeddings": 32768, "rms_norm_eps": 1e-5,
        "rope_theta": 1000000.0, "sliding_window": None, "tie_word_embeddings": False,
        "bos_token_id": 1, "eos_token_id": 2, "hidden_act": "silu"},
    "mistralai/Mixtral-8x7B-Instruct-v0.1": {
        "architectures": ["MixtralForCausalLM"], "hidden_size": 4096, "intermediate_size": 14336,
        "num_hidden_layers": 32, "num_attention_heads": 32, "num_key_value_heads": 8,
        "vocab_size": 32000, "max_position_embeddings": 32768, "rms_norm_eps": 1e-5,
        "rope_theta": 1000000.0, "num_local_experts": 8, "num_experts_per_tok": 2,
        "sliding_window": None, "tie_word_embeddings": False, "bos_token_id": 1,
        "eos_token_id": 2, "hidden_act": "silu"},
    "Qwen/Qwen2.5-32B-Instruct": _qwen2(5120, 27648, 64, 40, 8),
    "deepseek-ai/DeepSeek-R1-Distill-Qwen-32B": _qwen2(5120, 27648, 64, 40, 8,
                                                      max_position_embeddings=131072,
                                                      eos_token_id=151643),
    "Qwen/Qwen3-1.7B": _qwen3(2048, 6144, 28, 16, 8),
    "Qwen/Qwen3-4B-Instruct-2507": _qwen3(2560, 9728, 36, 32, 8, rope_theta=5000000.0,
                                          max_position_embeddings=262144),
    "meta-llama/Llama-4-Scout-17B-16E-Instruct": {
        "architectures": ["Llama4ForConditionalGeneration"], "hidden_size": 5120,
        "intermediate_size": 8192, "intermediate_size_mlp": 16384, "num_hidden_layers": 48,
        "num_attention_heads": 40, "num_key_value_heads": 8, "head_dim": 128,
        "vocab_size": 202048, "max_position_embeddings": 10485760, "rms_norm_eps": 1e-5,
        "rope_theta": 500000.0, "num_local_experts": 16, "num_experts_per_tok": 1,
        "attention_chunk_size": 8192, "tie_word_embeddings": False, "bos_token_id": 200000,
        "eos_token_id": [200001, 200007, 200008], "hidden_act": "silu",
        "shared_expert_intermediate_size": 8192,
        "rope_scaling": {"rope_type": "llama3", "factor": 16.0, "low_freq_factor": 1.0,
                         "high_freq_factor": 1.0, "original_max_position_embeddings": 8192}},
    "facebook/opt-125m": {
        "architectures": ["OPTForCausalLM"], "hidden_size": 768, "ffn_dim": 3072,
        "num_hidden_layers": 12, "num_attention_heads": 12, "vocab_size": 50272,
        "max_position_embeddings": 2048, "word_embed_proj_dim": 768,
        "do_layer_norm_before": True, "activation_function": "relu",
        "tie_word_embeddings": True, "pad_token_id": 1, "bos_token_id": 2, "eos_token_id": 2,
        "layer_norm_eps": 1e-5},
    "BAAI/bge-base-en-v1.5": {
        "architectures": ["BertModel"], "hidden_size": 768, "intermediate_size": 3072,
        "num_hidden_layers": 12, "num_attention_heads": 12, "vocab_size": 30522,
        "max_position_embeddings": 512, "type_vocab_size": 2, "layer_norm_eps": 1e-12,
        "hidden_act": "gelu", "pad_token_id": 0},
    "BAAI/bge-reranker-base": {
        "architectures": ["XLMRobertaForSequenceClassification"], "model_type": "xlm-roberta",
        "hidden_size": 768, "intermediate_size": 3072, "num_hidden_layers": 12,
        "num_attention_heads": 12, "vocab_size": 250002, "max_position_embeddings": 514,
        "type_vocab_size": 1, "layer_norm_eps": 1e-5, "hidden_act": "gelu", "pad_token_id": 1,
        "num_labels": 1},
}

# Reference menu names (core/lib/models/model-selection.sh:105-258) -> HF id.
SHORT_NAMES: Dict[str, str] = {
    "llama-8b": "meta-llama/Llama-3.1-8B-Instruct",
    "llama-70b": "meta-llama/Llama-3.1-70B-Instruct",
    "llama3-405b": "meta-llama/Llama-3.1-405B-Instruct",
    "llama-3-3-70b": "meta-llama/Llama-3.3-70B-Instruct",
    "llama-4-scout-17b": "meta-llama/Llama-4-Scout-17B-16E-Instruct",
    "qwen-2-5-32b": "Qwen/Qwen2.5-32B-Instruct",
    "deepseek-r1-distill-qwen-32b": "deepseek-ai/DeepSeek-R1-Distill-Qwen-32B",
    "deepseek-r1-distill-llama8b": "deepseek-ai/DeepSeek-R1-Distill-Llama-8B",
    "mixtral-8x-7b": "mistralai/Mixtral-8x7B-Instruct-v0.1",
    "mistral-7b": "mistralai/Mistral-7B-Instruct-v0.3",
    "tei": "BAAI/bge-base-en-v1.5",
    "rerank": "BAAI/bge-reranker-base",
    "codellama-34b": "codellama/CodeLlama-34b-Instruct-hf",
    "falcon3-7b": "tiiuae/Falcon3-7B-Instruct",
    "cpu-llama-8b": "meta-llama/Llama-3.1-8B-Instruct",
    "cpu-llama-3-2-3b": "meta-llama/Llama-3.2-3B-Instruct",
    "cpu-deepseek-r1-distill-llama8b": "deepseek-ai/DeepSeek-R1-Distill-Llama-8B",
    "cpu-deepseek-r1-distill-qwen-32b": "deepseek-ai/DeepSeek-R1-Distill-Qwen-32B",
    "cpu-qwen3-1-7b": "Qwen/Qwen3-1.7B",
    "cpu-qwen3-4b": "Qwen/Qwen3-4B-Instruct-2507",
    "opt-125m": "facebook/opt-125m",
    "llama-70b-tp8-rank": "eia/Llama-3.3-70B-TP8-rank",
    "llama-405b-tp8-rank": "eia/Llama-3.1-405B-TP8-rank",
    # BASELINE.json config names
    "Llama-3-8B": "meta-llama/Llama-3.1-8B-Instruct",
    "Llama-3-70B": "meta-llama/Llama-3.3-70B-Instruct",
}


def resolve_name(name: str) -> str:
    return SHORT_NAMES.get(name, name)


def get_preset(name: str) -> dict:
    key = resolve_name(name)
    if key not in PRESETS:
        raise KeyError(f"unknown model {name!r} (not a local dir with config.json and not in the "
                       f"built-in catalog: {sorted(PRESETS)})")
    return copy.deepcopy(PRESETS[key])


def tiny_config(arch: str = "LlamaForCausalLM", **kw) -> dict:
    """Small random-init configs for tests and smoke runs."""
    base = {"architectures": [arch], "hidden_size": 256, "intermediate_size": 512,
            "num_hidden_layers": 2, "num_attention_heads": 8, "num_key_value_heads": 2,
            "vocab_size": 512, "max_position_embeddings": 2048, "rms_norm_eps": 1e-5,
            "rope_theta": 10000.0, "tie_word_embeddings": False, "eos_token_id": 2,
            "bos_token_id": 1, "hidden_act": "silu"}
    if arch == "MixtralForCausalLM":
        base.update(num_local_experts=4, num_experts_per_tok=2)
    if arch == "Qwen2ForCausalLM":
        base.update(attention_bias=True)
    if arch == "Qwen3ForCausalLM":
        base.update(head_dim=64)
    if arch == "OPTForCausalLM":
        base = {"architectures": [arch], "hidden_size": 128, "ffn_dim": 256,
                "num_hidden_layers": 2, "num_attention_heads": 4, "vocab_size": 512,
                "max_position_embeddings": 512, "word_embed_proj_dim": 128,
                "do_layer_norm_before": True, "activation_function": "relu",
                "tie_word_embeddings": True, "pad_token_id": 1, "bos_token_id": 2,
                "eos_token_id": 2, "layer_norm_eps": 1e-5}
    base.update(kw)
    return base
