"""Model acquisition: a local snapshot, or a Hugging Face Hub download into ``HF_HOME``.

Reference behaviour: the serving pod gets ``HF_HOME=/data`` (a PVC,
core/helm-charts/vllm/templates/configmap.yaml:20), ``HF_TOKEN`` from the
per-release Secret (templates/secret.yaml:11-13) and ``HF_HUB_DISABLE_XET=1``
(gaudi-values.yaml:62); vLLM downloads the checkpoint on first start and reuses
it after restarts.  Same contract here: ``ensure_local_model`` returns the
snapshot directory (found in ``--download-dir`` / ``HF_HOME`` or downloaded with
``huggingface_hub.snapshot_download``) and raises when the model cannot be
obtained.  Random weights happen only with an explicit ``--load-format dummy``;
never as a silent fallback.
"""

from __future__ import annotations

import glob
import logging
import os
from typing import Optional

logger = logging.getLogger(__name__)

# files a serving snapshot needs (weights, configs, tokenizer); skips *.pth / onnx / gguf / etc.
_PATTERNS = ["*.json", "*.safetensors", "*.model", "*.txt", "*.tiktoken", "tokenizer*",
             "*.jinja"]


class ModelNotAvailableError(RuntimeError):
    pass


def has_weights(path: str) -> bool:
    return bool(glob.glob(os.path.join(path, "*.safetensors")) or
                glob.glob(os.path.join(path, "*.bin")))


def _cache_roots(download_dir: Optional[str]):
    roots = []
    if download_dir:
        roots += [download_dir, os.path.join(download_dir, "hub")]
    home = os.environ.get("HF_HOME")
    if home:
        roots.append(os.path.join(home, "hub"))
    hub_cache = os.environ.get("HF_HUB_CACHE") or os.environ.get("HUGGINGFACE_HUB_CACHE")
    if hub_cache:
        roots.append(hub_cache)
    return roots


def find_local(model: str, download_dir: Optional[str] = None) -> Optional[str]:
    """A directory with config.json for ``model``: the path itself, or an HF-cache snapshot."""
    if os.path.isdir(model) and os.path.exists(os.path.join(model, "config.json")):
        return model
    for root in _cache_roots(download_dir):
        snap = os.path.join(root, "models--" + model.replace("/", "--"), "snapshots")
        if os.path.isdir(snap):
            for d in sorted(os.listdir(snap), reverse=True):
                p = os.path.join(snap, d)
                if os.path.exists(os.path.join(p, "config.json")):
                    return p
    return None


def download(model: str, download_dir: Optional[str] = None, revision: Optional[str] = None) -> str:
    """``snapshot_download`` of the serving files; raises ``ModelNotAvailableError``."""
    try:
        from huggingface_hub import snapshot_download
    except ImportError as e:   # pragma: no cover - huggingface_hub ships in the image
        raise ModelNotAvailableError("huggingface_hub is not installed") from e
    token = os.environ.get("HF_TOKEN") or os.environ.get("HUGGING_FACE_HUB_TOKEN") or None
    kw = dict(repo_id=model, revision=revision, token=token, cache_dir=download_dir)
    logger.info("downloading %s into %s (HF_HUB_DISABLE_XET=%s)", model,
                download_dir or os.environ.get("HF_HOME", "~/.cache/huggingface"),
                os.environ.get("HF_HUB_DISABLE_XET", "0"))
    try:
        path = snapshot_download(allow_patterns=_PATTERNS, **kw)
        if not has_weights(path):       # pre-safetensors checkpoints: PyTorch .bin shards
            path = snapshot_download(allow_patterns=_PATTERNS + ["*.bin"], **kw)
    except Exception as e:   # noqa: BLE001 - network / auth / gated repo / missing repo
        raise ModelNotAvailableError(
            f"model {model!r} is not in --download-dir/HF_HOME and could not be downloaded "
            f"({type(e).__name__}: {e}). Provide HF_TOKEN for gated models, pre-populate "
            f"HF_HOME, pass a local directory, or use --load-format dummy for random weights."
        ) from e
    return path


def ensure_local_model(model: str, load_format: str = "auto",
                       download_dir: Optional[str] = None,
                       revision: Optional[str] = None) -> Optional[str]:
    """Local snapshot directory for ``model``.  ``None`` only for ``load_format == "dummy"``
    without a local config (then the catalog preset supplies the architecture)."""
    path = find_local(model, download_dir)
    if load_format == "dummy":
        return path
    if path is None or not has_weights(path):
        path = download(model, download_dir, revision)
    if not has_weights(path):
        raise ModelNotAvailableError(f"no *.safetensors / *.bin weights under {path}")
    return path
