"""MoE model families vs HF transformers on the CPU path (Mixtral, Qwen3-MoE, Llama-4 text)."""

import pytest
import torch

from enterprise_inference_amd.config import CacheConfig, EngineConfig, ModelConfig, SchedulerConfig
from enterprise_inference_amd.engine.llm_engine import LLMEngine
from enterprise_inference_amd.engine.sampling_params import SamplingParams
from enterprise_inference_amd.models.catalog import tiny_config


def _engine(d):
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d),
                       cache=CacheConfig(block_size=16, num_gpu_blocks=64),
                       scheduler=SchedulerConfig(max_num_seqs=4, max_num_batched_tokens=48,
                                                 max_model_len=512),
                       device="cpu", dtype=torch.float32, load_format="dummy")
    return LLMEngine(cfg)


def _check(eng, hf, prompts, n=6):
    outs = eng.generate(prompt_token_ids=prompts,
                        params=SamplingParams(max_tokens=n, temperature=0, ignore_eos=True))
    with torch.no_grad():
        for p, o in zip(prompts, outs):
            ids = torch.tensor([p])
            for _ in range(n):
                nxt = hf(ids).logits[0, -1].argmax()
                ids = torch.cat([ids, nxt.view(1, 1)], 1)
            assert o.outputs[0].token_ids == ids[0, len(p):].tolist()


def test_mixtral_matches_transformers():
    import transformers
    d = tiny_config("MixtralForCausalLM")
    hc = transformers.MixtralConfig(**{k: v for k, v in d.items() if k != "architectures"})
    torch.manual_seed(0)
    hf = transformers.MixtralForCausalLM(hc).eval()
    eng = _engine(d)
    eng.executor.runner.model.load_weights(hf.state_dict().items())
    _check(eng, hf, [[3, 4, 5, 6, 7, 8, 9] * 9, [11, 12]])


def test_qwen3_moe_matches_transformers():
    import transformers
    d = tiny_config("Qwen3MoeForCausalLM", num_local_experts=4, num_experts=4,
                    num_experts_per_tok=2, moe_intermediate_size=128, head_dim=64,
                    norm_topk_prob=True, decoder_sparse_step=1, mlp_only_layers=[])
    hc = transformers.Qwen3MoeConfig(**{k: v for k, v in d.items() if k != "architectures"})
    torch.manual_seed(0)
    hf = transformers.Qwen3MoeForCausalLM(hc).eval()
    eng = _engine(d)
    eng.executor.runner.model.load_weights(hf.state_dict().items())
    _check(eng, hf, [[5, 6, 7, 8] * 12, [9, 10, 11]])


@pytest.mark.parametrize("moe_layers", [[0, 1, 2, 3], [1, 3]])   # [1, 3]: Maverick-style dense/MoE
def test_llama4_text_matches_transformers(moe_layers):
    import transformers
    d = tiny_config("Llama4ForCausalLM", num_local_experts=4, num_experts_per_tok=1,
                    intermediate_size=128, intermediate_size_mlp=256, head_dim=32,
                    num_hidden_layers=4, attention_chunk_size=32, no_rope_layers=[1, 1, 1, 0],
                    use_qk_norm=True, attn_temperature_tuning=True, floor_scale=8, attn_scale=0.1,
                    interleave_moe_layer_step=1, moe_layers=moe_layers)
    hcfg = {k: v for k, v in d.items() if k not in ("architectures",)}
    hc = transformers.Llama4TextConfig(**hcfg)
    hc._attn_implementation = "eager"
    torch.manual_seed(0)
    hf = transformers.Llama4ForCausalLM(hc).eval()
    eng = _engine(d)
    eng.executor.runner.model.load_weights(hf.state_dict().items())
    # 50-token prompt crosses the 32-token attention chunk and the temperature floor
    _check(eng, hf, [list(range(20, 70)), [7, 8, 9]], n=5)


def test_rope_cache_accepts_splitk_on_cpu():
    """The split-K hand-off into K4 (ops/rotary.py) also works on the CPU reference path."""
    import torch
    from enterprise_inference_amd.ops import gemm
    from enterprise_inference_amd.ops.rotary import RotaryCache, rope_qkv_cache
    Hq, Hkv, D, M = 4, 2, 64, 3
    N = (Hq + 2 * Hkv) * D
    part = torch.randn(2, M, N)
    bias = torch.randn(N).to(torch.bfloat16)
    rot = RotaryCache(D, 128, 10000.0, None, torch.device("cpu"))
    pos = torch.tensor([0, 5, 9], dtype=torch.int32)
    slots = torch.tensor([0, 1, 2], dtype=torch.int32)
    outs = []
    for split in (True, False):
        kc = torch.zeros(2, Hkv, 16, D, dtype=torch.bfloat16)
        vc = torch.zeros(2, Hkv, D, 16, dtype=torch.bfloat16)
        s = gemm.SplitK(part, 2, M, N, bias)
        qkv = s if split else s.materialize()
        q = rope_qkv_cache(qkv, pos, rot, slots, kc, vc, Hq, Hkv, D,
                           bias=None)
        outs.append((q, kc, vc))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_grouped_moe_cfgs():
    """ops/moe.py moe_cfgs: 4-wave forms where the shape divides, overrides masked to the four
    grouped forms the kernel builds (cfg 0-3)."""
    from enterprise_inference_amd.ops.moe import moe_cfgs
    assert moe_cfgs(14336, 4096) == (3, 2)
    assert moe_cfgs(100, 100) == (1, 0)
    assert moe_cfgs(14336, 4096, 7, 6) == (3, 2)
    assert moe_cfgs(14336, 4096, 1, 0) == (1, 0)
