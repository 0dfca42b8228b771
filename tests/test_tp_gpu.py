"""Tensor-parallel engine on the MI355X, every rank on the one GPU of the test box.

RCCL refuses two ranks on one device, so ``ParallelConfig(share_device=True)``
(``EIA_TP_SHARE_DEVICE=1``) runs the TP engine with gloo and host-staged collectives, eager
decode and no custom all-reduce -- everything else is the production TP path: the driver +
spawned worker processes, the binary step plan through the native shm ring, column/row
sharded projections, vocab-sharded embedding and LM head with per-shard sampling, and the
HIP kernels at the PER-RANK shapes.  The Llama shapes reproduce Llama-3.3-70B at TP=8 per
rank (8 query heads / 1 KV head, GQA 8, head_dim 128); Mixtral covers both EP forms.

Every generated token is checked by teacher forcing against HF transformers fp32 on the CPU
(same safetensors checkpoint, utils/parity.py), and against the TP=1 engine on the same GPU.
"""

import json

import pytest
import torch

from enterprise_inference_amd.config import (CacheConfig, EngineConfig, ModelConfig,
                                             ParallelConfig, SchedulerConfig)
from enterprise_inference_amd.engine.llm_engine import LLMEngine
from enterprise_inference_amd.engine.sampling_params import SamplingParams
from enterprise_inference_amd.models.catalog import tiny_config
from enterprise_inference_amd.utils.parity import check_greedy, check_logprobs, hf_reference_model

pytestmark = pytest.mark.gpu

# TP2 -> 8 q heads / 1 kv head per rank; TP4 -> same per rank with 32 / 4 heads
SHAPES = {
    2: dict(hidden_size=1024, intermediate_size=2048, num_attention_heads=16,
            num_key_value_heads=2, head_dim=128, vocab_size=2048, num_hidden_layers=2,
            max_position_embeddings=4096, initializer_range=0.05),
    4: dict(hidden_size=2048, intermediate_size=4096, num_attention_heads=32,
            num_key_value_heads=4, head_dim=128, vocab_size=2048, num_hidden_layers=2,
            max_position_embeddings=4096, initializer_range=0.05),
}


def _ckpt(tmp_path, d):
    from safetensors.torch import save_file
    hf = hf_reference_model(d)
    save_file({k: v.contiguous() for k, v in hf.state_dict().items()},
              str(tmp_path / "model.safetensors"))
    (tmp_path / "config.json").write_text(json.dumps(d))
    return hf, str(tmp_path)


# init std 0.05 (2.5x the e2e tests'): logits, and their bf16 rounding, scale with the init
# and sqrt(hidden); a token may trail the oracle's best by 10 % of the row's logit std
TOL, REL = 0.08, 0.1


def _generate(path, d, tp, ep=False, temperature=0.0, logprobs=None):
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d), model_path=path,
                       cache=CacheConfig(block_size=128, num_gpu_blocks=48),
                       scheduler=SchedulerConfig(max_num_seqs=8, max_num_batched_tokens=256,
                                                 max_model_len=1024),
                       parallel=ParallelConfig(tensor_parallel_size=tp, enable_expert_parallel=ep,
                                               share_device=tp > 1),
                       device="cuda", dtype=torch.bfloat16)
    eng = LLMEngine(cfg)
    try:
        if tp > 1:
            r = eng.executor.runner
            assert r.num_heads == d["num_attention_heads"] // tp
            assert r.num_kv_heads == max(1, d["num_key_value_heads"] // tp)
            assert r.sharded_lm, "TP>1 must keep the LM head vocab-sharded"
        g = torch.Generator().manual_seed(7)
        prompts = [torch.randint(3, d["vocab_size"], (n,), generator=g).tolist()
                   for n in (300, 37, 129)]       # chunked prefill (budget 256) + short + 1 block+1
        params = SamplingParams(max_tokens=12, temperature=temperature, ignore_eos=True, seed=5,
                                logprobs=logprobs)
        outs = eng.generate(prompt_token_ids=prompts, params=params)
        toks = [o.outputs[0].token_ids for o in outs]
        if logprobs is not None:
            return prompts, toks, [o.outputs[0].logprobs for o in outs]
        return prompts, toks
    finally:
        eng.shutdown()
        from enterprise_inference_amd.parallel import state
        state.destroy_distributed()


@pytest.mark.parametrize("tp", [2, 4])
def test_tp_llama_70b_rank_layout_matches_oracle(tmp_path, tp):
    d = tiny_config("LlamaForCausalLM", **SHAPES[tp])
    hf, path = _ckpt(tmp_path, d)
    prompts, got = _generate(path, d, tp)
    stats = check_greedy(hf, prompts, got, tol=TOL, rel=REL)
    assert stats["argmax_agreement"] > 0.8, stats
    # logits-level bound on the gathered (vocab-sharded) rows through the logprobs path
    p2, got2, lps = _generate(path, d, tp, logprobs=5)
    check_logprobs(hf, p2, got2, lps, tol=0.25)   # O(1) nats for a real sharding bug
    _, ref = _generate(path, d, 1)
    same = sum(a == b for x, y in zip(got, ref) for a, b in zip(x, y)) / sum(map(len, ref))
    assert same > 0.8, (got, ref)
    assert got[0][0] == ref[0][0] and got[1][0] == ref[1][0]


@pytest.mark.parametrize("dispatch", ["allreduce", "all_to_all"])
def test_tp2_mixtral_expert_parallel_matches_oracle(tmp_path, monkeypatch, dispatch):
    monkeypatch.setenv("EIA_EP_DISPATCH", dispatch)
    d = tiny_config("MixtralForCausalLM", **{**SHAPES[2], "num_local_experts": 4,
                                             "num_experts_per_tok": 2})
    hf, path = _ckpt(tmp_path, d)
    prompts, got = _generate(path, d, 2, ep=True)
    # top-2 routing is discrete: a bf16-level near-tie between two experts' router logits
    # flips the expert set of a token, so MoE rows get a wider logit bound
    stats = check_greedy(hf, prompts, got, tol=TOL, rel=2.5 * REL)
    assert stats["argmax_agreement"] > 0.8, stats


def test_tp2_sharded_sampling_matches_tp1(tmp_path):
    """Seeded temperature sampling: per-shard winners (global-id-keyed RNG) merged over the
    group pick the same tokens as the TP=1 full-row sampler, as long as the logits agree --
    compared on the first token of each request (identical prefill logits up to bf16)."""
    d = tiny_config("LlamaForCausalLM", **SHAPES[2])
    _, path = _ckpt(tmp_path, d)
    _, got = _generate(path, d, 2, temperature=0.8)
    _, ref = _generate(path, d, 1, temperature=0.8)
    assert [g[0] for g in got] == [r[0] for r in ref]
    assert len({t for g in got for t in g}) > 3
