"""Weight loading: safetensors (mmap, TP-sharded via per-parameter weight_loader)
or deterministic random init (``--load-format dummy``; the north-star benchmark
mode, no checkpoints are available offline).

Reference behaviour: weights are downloaded into the /data PVC with HF_HOME=/data
(core/helm-charts/vllm/templates/configmap.yaml:20); the download itself is
models/hub.py (run by the CLI before the engine starts), this module reads the
local snapshot and fails loudly when it holds no weights.
"""

from __future__ import annotations

import glob
import json
import os
from typing import Iterator, Optional, Tuple

import logging

import torch
import torch.nn as nn

from ..config import EngineConfig, ModelConfig
from . import get_model_class
from .layers import init_random_

logger = logging.getLogger(__name__)


def iter_safetensors(path: str) -> Iterator[Tuple[str, torch.Tensor]]:
    from safetensors import safe_open

    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors under {path}")
    for f in files:
        with safe_open(f, framework="pt", device="cpu") as sf:
            for k in sf.keys():
                yield k, sf.get_tensor(k)


def iter_torch_bins(path: str) -> Iterator[Tuple[str, torch.Tensor]]:
    for f in sorted(glob.glob(os.path.join(path, "*.bin"))):
        sd = torch.load(f, map_location="cpu", weights_only=True)   # never unpickles code
        yield from sd.items()


def build_model(cfg: EngineConfig, device: torch.device) -> nn.Module:
    cls = get_model_class(cfg.model.architecture)
    from ..parallel import state as pstate
    if pstate.pp_size() > 1 and not getattr(cls, "supports_pp", False):
        raise NotImplementedError(f"{cfg.model.architecture} does not support "
                                  "--pipeline-parallel-size > 1 (Llama/Qwen/Mistral/Mixtral do)")
    model = cls(cfg.model, dtype=cfg.dtype, device=device)
    model.eval()
    fmt = cfg.load_format
    if cfg.model_path is None and fmt != "dummy":
        # never serve random weights by accident: only --load-format dummy asks for them
        raise ValueError("no model_path given and load_format is not 'dummy' (random weights "
                         "must be requested explicitly)")
    if fmt == "dummy":
        logger.info("random-init weights (load_format=%s, no checkpoint)", fmt)
        init_random_(model, seed=cfg.seed)
        post = getattr(model, "post_load", None)
        if post:
            post()
        return model
    if glob.glob(os.path.join(cfg.model_path, "*.safetensors")) and fmt != "pt":
        it = iter_safetensors(cfg.model_path)
    elif glob.glob(os.path.join(cfg.model_path, "*.bin")):
        it = iter_torch_bins(cfg.model_path)
    else:
        raise FileNotFoundError(f"no *.safetensors or *.bin weights under {cfg.model_path} "
                                "(use --load-format dummy for random weights)")
    with torch.no_grad():
        model.load_weights(it)
    post = getattr(model, "post_load", None)
    if post:
        post()
    return model


def resolve_model_config(model: str, hf_overrides: Optional[dict] = None) -> ModelConfig:
    """A local dir with config.json, a catalog HF id, or a catalog short name."""
    from .catalog import get_preset

    if os.path.isdir(model) and os.path.exists(os.path.join(model, "config.json")):
        with open(os.path.join(model, "config.json")) as f:
            d = json.load(f)
    else:
        d = get_preset(model)
    if hf_overrides:
        d = {**d, **hf_overrides}
    return ModelConfig.from_hf_dict(d, name=model)
