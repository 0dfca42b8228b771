"""Weight acquisition: HF download into HF_HOME, fail-loud loading.

The reference downloads checkpoints into the /data PVC with HF_TOKEN
(core/helm-charts/vllm/templates/configmap.yaml:20, templates/secret.yaml:11-13).
There is no network here, so ``huggingface_hub.snapshot_download`` is replaced by a
fake that materialises a local safetensors checkpoint in the HF cache layout; the
served tokens are checked against transformers on the same weights (parity), and
every way of *not* getting weights must raise instead of serving random ones.
"""

import os
import shutil

import pytest
import torch

from enterprise_inference_amd.entrypoints.cli_args import engine_config_from_args, parse_args
from enterprise_inference_amd.models import hub
from enterprise_inference_amd.models.catalog import tiny_config


def _make_checkpoint(d):
    import transformers
    from tokenizers import Tokenizer, models, pre_tokenizers

    cfg = tiny_config(vocab_size=300)
    hc = transformers.LlamaConfig(**{k: v for k, v in cfg.items() if k != "architectures"})
    hc.architectures = ["LlamaForCausalLM"]
    torch.manual_seed(0)
    hf = transformers.LlamaForCausalLM(hc).float().eval()
    hf.save_pretrained(d, safe_serialization=True)
    vocab = {f"w{i}": i for i in range(300)}
    tk = Tokenizer(models.WordLevel(vocab, unk_token="w0"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    fast = transformers.PreTrainedTokenizerFast(tokenizer_object=tk, unk_token="w0",
                                                bos_token="w1", eos_token="w2")
    fast.save_pretrained(d)
    return hf


@pytest.fixture(scope="module")
def checkpoint(tmp_path_factory):
    d = tmp_path_factory.mktemp("ckpt")
    hf = _make_checkpoint(str(d))
    return str(d), hf


def _fake_download(src, calls):
    def fake(repo_id, revision=None, token=None, cache_dir=None, allow_patterns=None, **_):
        calls.append({"repo_id": repo_id, "token": token, "cache_dir": cache_dir,
                      "patterns": allow_patterns})
        root = cache_dir or os.path.join(os.environ["HF_HOME"], "hub")
        snap = os.path.join(root, "models--" + repo_id.replace("/", "--"), "snapshots", "abc123")
        if not os.path.isdir(snap):
            shutil.copytree(src, snap)
        return snap
    return fake


def test_download_then_serve_matches_transformers(checkpoint, tmp_path, monkeypatch):
    import huggingface_hub

    from enterprise_inference_amd.engine.llm_engine import LLMEngine
    from enterprise_inference_amd.engine.sampling_params import SamplingParams

    src, hf = checkpoint
    calls = []
    monkeypatch.setenv("HF_HOME", str(tmp_path / "data"))
    monkeypatch.setenv("HF_TOKEN", "hf_secret")
    monkeypatch.setattr(huggingface_hub, "snapshot_download", _fake_download(src, calls))
    args = parse_args(["--model", "acme/tiny-llama", "--device", "cpu", "--max-model-len", "256",
                       "--max-num-seqs", "4", "--max-num-batched-tokens", "64",
                       "--block-size", "16"])
    cfg = engine_config_from_args(args)
    assert calls and calls[0]["repo_id"] == "acme/tiny-llama" and calls[0]["token"] == "hf_secret"
    assert cfg.model_path.startswith(str(tmp_path / "data")) and hub.has_weights(cfg.model_path)
    eng = LLMEngine(cfg)
    assert eng.tokenizer.__class__.__name__ != "ByteTokenizer"
    prompt = [5, 9, 17, 33, 60]
    out = eng.generate(prompt_token_ids=[prompt],
                       params=SamplingParams(max_tokens=8, temperature=0, ignore_eos=True))
    ref = hf.generate(torch.tensor([prompt]), max_new_tokens=8, do_sample=False,
                      eos_token_id=None, pad_token_id=0)[0, len(prompt):].tolist()
    assert out[0].outputs[0].token_ids == ref
    # second start: the cached snapshot is reused, no new download
    n = len(calls)
    assert engine_config_from_args(args).model_path == cfg.model_path and len(calls) == n


def test_missing_model_raises(tmp_path, monkeypatch):
    import huggingface_hub

    def offline(**_):
        raise OSError("no route to host")

    monkeypatch.setenv("HF_HOME", str(tmp_path / "empty"))
    monkeypatch.setattr(huggingface_hub, "snapshot_download", offline)
    args = parse_args(["--model", "meta-llama/Llama-3.1-8B-Instruct", "--device", "cpu"])
    with pytest.raises(hub.ModelNotAvailableError, match="could not be downloaded"):
        engine_config_from_args(args)
    # explicit dummy: random weights, no download attempted
    cfg = engine_config_from_args(parse_args(["--model", "meta-llama/Llama-3.1-8B-Instruct",
                                              "--device", "cpu", "--load-format", "dummy"]))
    assert cfg.model_path is None and cfg.load_format == "dummy"


def test_weights_and_tokenizer_required_for_real_checkpoints(checkpoint, tmp_path):
    from enterprise_inference_amd.config import EngineConfig, ModelConfig
    from enterprise_inference_amd.models.loader import build_model
    from enterprise_inference_amd.tokenizer import get_tokenizer

    src, _ = checkpoint
    only_cfg = tmp_path / "cfg_only"
    only_cfg.mkdir()
    shutil.copy(os.path.join(src, "config.json"), only_cfg / "config.json")
    m = ModelConfig.from_pretrained(str(only_cfg))
    cfg = EngineConfig(model=m, device="cpu", dtype=torch.float32, model_path=str(only_cfg))
    with pytest.raises(FileNotFoundError, match="no \\*.safetensors"):
        build_model(cfg, torch.device("cpu"))
    with pytest.raises(RuntimeError, match="no loadable tokenizer"):
        get_tokenizer(str(only_cfg), 300, allow_byte_fallback=False)
    assert get_tokenizer(None, 300).__class__.__name__ == "ByteTokenizer"
