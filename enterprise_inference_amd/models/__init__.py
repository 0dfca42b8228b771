"""Model registry: HF ``architectures[0]`` -> implementation class."""

from __future__ import annotations

from typing import Dict, Type

import torch.nn as nn

_REGISTRY: Dict[str, str] = {
    "LlamaForCausalLM": "llama:LlamaForCausalLM",
    "MistralForCausalLM": "llama:LlamaForCausalLM",
    "Qwen2ForCausalLM": "llama:LlamaForCausalLM",
    "Qwen3ForCausalLM": "llama:LlamaForCausalLM",
    "MixtralForCausalLM": "mixtral:MixtralForCausalLM",
    "Qwen2MoeForCausalLM": "mixtral:MixtralForCausalLM",
    "Qwen3MoeForCausalLM": "mixtral:MixtralForCausalLM",
    "Llama4ForConditionalGeneration": "mixtral:Llama4ForCausalLM",
    "Llama4ForCausalLM": "mixtral:Llama4ForCausalLM",
    "OPTForCausalLM": "opt:OPTForCausalLM",
    "BertModel": "bert:BertEmbeddingModel",
    "XLMRobertaModel": "bert:BertEmbeddingModel",
    "XLMRobertaForSequenceClassification": "bert:CrossEncoderModel",
    "BertForSequenceClassification": "bert:CrossEncoderModel",
}


def supported_architectures():
    return sorted(_REGISTRY)


def get_model_class(arch: str) -> Type[nn.Module]:
    if arch not in _REGISTRY:
        raise ValueError(f"unsupported architecture {arch!r}; supported: {supported_architectures()}")
    mod, cls = _REGISTRY[arch].split(":")
    import importlib
    m = importlib.import_module(f"{__name__}.{mod}")
    return getattr(m, cls)
