"""Beam search (``use_beam_search`` / ``length_penalty`` / ``early_stopping``, reference
docs/api-spec.yaml:385-408) against a brute-force beam reference that re-runs the fp32 HF
model on every full hypothesis (no KV cache): same candidates, same ranking, same stop rule.
The engine side exercises the KV block-table forks, the copy-on-write block copies of the
shared partial block and the logprobs path of the sampler."""

import json

import pytest
import torch

from enterprise_inference_amd.config import (CacheConfig, EngineConfig, ModelConfig,
                                             ParallelConfig, SchedulerConfig)
from enterprise_inference_amd.engine.llm_engine import LLMEngine
from enterprise_inference_amd.engine.sampling_params import SamplingParams
from enterprise_inference_amd.models.catalog import tiny_config


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    import transformers
    from safetensors.torch import save_file
    d = tiny_config("LlamaForCausalLM", vocab_size=300, initializer_range=0.2)
    hc = transformers.LlamaConfig(**{k: v for k, v in d.items() if k != "architectures"})
    torch.manual_seed(3)
    hf = transformers.LlamaForCausalLM(hc).float().eval()
    p = tmp_path_factory.mktemp("beam")
    save_file({k: v.contiguous() for k, v in hf.state_dict().items()}, str(p / "model.safetensors"))
    (p / "config.json").write_text(json.dumps(d))
    return hf, str(p), d


def _engine(path, d, tp=1, blocks=64):
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d), model_path=path,
                       cache=CacheConfig(block_size=16, num_gpu_blocks=blocks),
                       scheduler=SchedulerConfig(max_num_seqs=16, max_num_batched_tokens=64,
                                                 max_model_len=256),
                       parallel=ParallelConfig(tensor_parallel_size=tp),
                       device="cpu", dtype=torch.float32)
    return LLMEngine(cfg)


@torch.no_grad()
def reference_beam(hf, prompt, W, n, max_tokens, length_penalty, early_stopping, eos):
    def score(cum, out_len, ends_eos):
        return cum / (max(1, len(prompt) + out_len - (1 if ends_eos else 0)) ** length_penalty)

    beams = [([], 0.0)]
    finished = []
    for _ in range(max_tokens):
        cands = []
        for bi, (out, cum) in enumerate(beams):
            lp = torch.log_softmax(hf(torch.tensor([prompt + out])).logits[0, -1].float(), -1)
            v, i = lp.topk(2 * W)
            cands += [(cum + float(a), bi, int(t), out) for a, t in zip(v, i)]
        cands.sort(key=lambda c: (-c[0], c[1], c[2]))
        running = []
        for cum, bi, tok, out in cands[:2 * W]:
            if tok in eos:
                finished.append((score(cum, len(out) + 1, True), out + [tok], cum))
            elif len(out) + 1 >= max_tokens:
                finished.append((score(cum, len(out) + 1, False), out + [tok], cum))
            elif len(running) < W:
                running.append((out + [tok], cum))
        finished.sort(key=lambda f: -f[0])
        finished = finished[:W]
        if not running:
            break
        if len(finished) >= W:
            if early_stopping:
                break
            best = max(score(c, len(o), False) for o, c in running)
            if finished[-1][0] >= best:
                break
        beams = running
    return [f[1] for f in sorted(finished, key=lambda f: -f[0])[:n]], finished


@pytest.mark.parametrize("W,n,lp,early,max_tokens", [(3, 2, 1.0, False, 9), (4, 1, 0.5, True, 12),
                                                    (2, 2, 2.0, False, 20)])
def test_beam_search_matches_bruteforce(ckpt, W, n, lp, early, max_tokens):
    hf, path, d = ckpt
    eos = {d["eos_token_id"]}
    prompts = [list(range(5, 28)), [7, 8, 9, 10, 11]]      # 23 and 5 tokens: partial blocks
    eng = _engine(path, d)
    params = SamplingParams(n=n, best_of=W, use_beam_search=True, temperature=0.0,
                            max_tokens=max_tokens, length_penalty=lp, early_stopping=early)
    outs = eng.generate(prompt_token_ids=prompts, params=params)
    for p, o in zip(prompts, outs):
        want, fin = reference_beam(hf, p, W, n, max_tokens, lp, early, eos)
        got = [c.token_ids for c in o.outputs]
        assert got == want, (got, want)
        for c, f in zip(o.outputs, sorted(fin, key=lambda f: -f[0])):
            assert abs(c.cumulative_logprob - f[2]) < 1e-3
    # every beam's blocks were released (forks + cow included)
    assert eng.scheduler.bm.num_free_blocks() == eng.scheduler.bm.num_blocks
    assert eng.scheduler.bm.check_invariants() == ""


def test_beam_search_tp2_matches_tp1(ckpt):
    """At TP=2 the copy-on-write block copies travel in the step plan to every rank."""
    from enterprise_inference_amd.parallel import state
    hf, path, d = ckpt
    params = SamplingParams(n=2, best_of=3, use_beam_search=True, temperature=0.0, max_tokens=10)
    prompts = [list(range(5, 28))]
    ref = [[c.token_ids for c in o.outputs]
           for o in _engine(path, d).generate(prompt_token_ids=prompts, params=params)]
    eng = _engine(path, d, tp=2)
    try:
        got = [[c.token_ids for c in o.outputs]
               for o in eng.generate(prompt_token_ids=prompts, params=params)]
    finally:
        eng.shutdown()
        state.destroy_distributed()
    assert got == ref


def test_beam_search_params_validation():
    with pytest.raises(ValueError, match="temperature"):
        SamplingParams(use_beam_search=True, temperature=0.7, best_of=2)
    with pytest.raises(ValueError, match="top_p"):
        SamplingParams(use_beam_search=True, temperature=0.0, top_p=0.5, best_of=2)


def test_beam_search_via_openai_api(ckpt, tmp_path):
    from fastapi.testclient import TestClient

    from enterprise_inference_amd.entrypoints.cli_args import parse_args
    from enterprise_inference_amd.entrypoints.openai.api_server import build_from_args
    _, path, _ = ckpt
    args = parse_args(["--model", path, "--served-model-name", "tiny", "--device", "cpu",
                       "--max-model-len", "256", "--max-num-seqs", "8", "--block-size", "16",
                       "--disable-log-requests", "--load-format", "dummy"])
    app, aeng = build_from_args(args, engine_mode="thread", wait_ready=True)
    try:
        with TestClient(app) as c:
            r = c.post("/v1/completions", json={"model": "tiny", "prompt": [5, 6, 7, 8, 9],
                                                "max_tokens": 6, "use_beam_search": True,
                                                "n": 2, "best_of": 3, "length_penalty": 1.0})
            assert r.status_code == 200, r.text
            body = r.json()
            assert len(body["choices"]) == 2
            assert {ch["index"] for ch in body["choices"]} == {0, 1}
            assert all(ch["finish_reason"] in ("stop", "length") for ch in body["choices"])
            assert 0 < body["usage"]["completion_tokens"] <= 12
            bad = c.post("/v1/completions", json={"model": "tiny", "prompt": [5, 6],
                                                  "max_tokens": 3, "use_beam_search": True,
                                                  "temperature": 0.9})
            assert bad.status_code == 400
    finally:
        aeng.shutdown()


def test_beam_search_ignores_sampling_generation_defaults():
    """A model whose generation_config sets min_p / repetition_penalty must still accept a
    beam-search request that sets neither (they are sampling knobs); stop strings are
    rejected up front (beams end on token ids only)."""
    from enterprise_inference_amd.entrypoints.openai.protocol import CompletionRequest
    gd = {"temperature": 0.6, "top_p": 0.9, "min_p": 0.05, "repetition_penalty": 1.1}
    req = CompletionRequest(model="m", prompt=[1, 2], use_beam_search=True, best_of=2)
    sp = req.to_sampling_params(16, None, gd)
    assert sp.use_beam_search and sp.temperature == 0.0 and sp.min_p == 0.0
    assert sp.repetition_penalty == 1.0 and sp.top_p == 1.0
    with pytest.raises(ValueError, match="stop strings"):
        CompletionRequest(model="m", prompt=[1], use_beam_search=True, best_of=2,
                          stop=["\n"]).to_sampling_params(16, None, gd)
    # without beam search the generation defaults still apply
    sp2 = CompletionRequest(model="m", prompt=[1]).to_sampling_params(16, None, gd)
    assert sp2.min_p == 0.05 and sp2.repetition_penalty == 1.1
