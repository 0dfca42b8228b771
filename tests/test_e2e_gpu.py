"""End-to-end GPU parity: the whole bf16 engine on an MI355X against an fp32 oracle.

Each decoder family runs through the production path -- HIP kernels, decode HIP graphs with
the device-side partition count (p_dyn), overlapped scheduling (in-flight token ids read on
device), chunked prefill, a prefix-cache hit and split-K skinny GEMMs -- and every generated
token is checked by teacher forcing against HF transformers fp32 on the CPU with identical
weights (utils/parity.py).  The TEI encoders are compared with the same CPU models.
"""

import pytest
import torch

from enterprise_inference_amd.config import CacheConfig, EngineConfig, ModelConfig, SchedulerConfig
from enterprise_inference_amd.engine.llm_engine import LLMEngine
from enterprise_inference_amd.engine.sampling_params import SamplingParams
from enterprise_inference_amd.models.catalog import tiny_config
from enterprise_inference_amd.utils.parity import check_greedy, check_logprobs, hf_reference_model

pytestmark = pytest.mark.gpu

SHAPE = dict(hidden_size=1024, intermediate_size=2048, num_attention_heads=8,
             num_key_value_heads=2, head_dim=128, vocab_size=1024, num_hidden_layers=2,
             max_position_embeddings=4096)


def _engine(d, mbt=256):
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d),
                       cache=CacheConfig(block_size=128, num_gpu_blocks=64),
                       scheduler=SchedulerConfig(max_num_seqs=16, max_num_batched_tokens=mbt,
                                                 max_model_len=2048),
                       device="cuda", dtype=torch.bfloat16, load_format="dummy")
    return LLMEngine(cfg)


@pytest.mark.parametrize("arch", ["LlamaForCausalLM", "Qwen2ForCausalLM", "Qwen3ForCausalLM",
                                  "MixtralForCausalLM"])
def test_engine_greedy_matches_fp32_oracle(arch):
    extra = {"num_local_experts": 4, "num_experts_per_tok": 2} if arch.startswith("Mixtral") else {}
    d = tiny_config(arch, **SHAPE, **extra)
    hf = hf_reference_model(d)
    eng = _engine(d)
    r = eng.executor.runner
    assert r.graphs, "decode graphs must be captured"
    r.model.load_weights(hf.state_dict().items())
    gen = torch.Generator().manual_seed(5)
    long_prompt = torch.randint(3, 1000, (700,), generator=gen).tolist()    # > 512: P > 1
    params = SamplingParams(max_tokens=24, temperature=0, ignore_eos=True)
    # 1) a long prompt alone: chunked prefill (budget 256), then graph decode with p_dyn > 1
    first = eng.generate(prompt_token_ids=[long_prompt], params=params)
    # 2) shared 640-token prefix (5 cached blocks) + a short prompt + a mid one, together
    shared = long_prompt[:640] + torch.randint(3, 1000, (30,), generator=gen).tolist()
    short = torch.randint(3, 1000, (37,), generator=gen).tolist()
    mid = torch.randint(3, 1000, (300,), generator=gen).tolist()
    outs = eng.generate(prompt_token_ids=[shared, short, mid], params=params)
    assert outs[0].num_cached_tokens >= 512, "prefix cache must hit"
    prompts = [long_prompt, shared, short, mid]
    toks = [first[0].outputs[0].token_ids] + [o.outputs[0].token_ids for o in outs]
    assert all(len(t) == 24 for t in toks)
    stats = check_greedy(hf, prompts, toks, tol=0.08)
    print(arch, stats)
    assert stats["argmax_agreement"] > 0.8
    # logits-level bound (graph decode + logprobs path): top-5 + chosen log-probs vs fp32
    lp_prompts = [short, mid]
    lp_outs = eng.generate(prompt_token_ids=lp_prompts,
                           params=SamplingParams(max_tokens=8, temperature=0, ignore_eos=True,
                                                 logprobs=5))
    lstats = check_logprobs(hf, lp_prompts, [o.outputs[0].token_ids for o in lp_outs],
                            [o.outputs[0].logprobs for o in lp_outs], tol=0.1)
    print(arch, lstats)


def test_engine_sampled_run_is_reproducible():
    """Seeded temperature sampling through graphs + overlap: identical tokens across runs."""
    d = tiny_config("LlamaForCausalLM", **SHAPE)
    eng = _engine(d)
    p = [list(range(5, 70)), list(range(200, 233))]
    sp = SamplingParams(max_tokens=16, temperature=0.9, top_p=0.95, seed=3, ignore_eos=True)
    a = [o.outputs[0].token_ids for o in eng.generate(prompt_token_ids=p, params=sp)]
    b = [o.outputs[0].token_ids for o in eng.generate(prompt_token_ids=p, params=sp)]
    assert a == b


BERT = {"architectures": ["BertModel"], "hidden_size": 768, "intermediate_size": 1536,
        "num_hidden_layers": 2, "num_attention_heads": 12, "vocab_size": 1000,
        "max_position_embeddings": 512, "type_vocab_size": 2, "layer_norm_eps": 1e-12,
        "hidden_act": "gelu", "pad_token_id": 0}
XLMR = {"architectures": ["XLMRobertaForSequenceClassification"], "model_type": "xlm-roberta",
        "hidden_size": 768, "intermediate_size": 1536, "num_hidden_layers": 2,
        "num_attention_heads": 12, "vocab_size": 1000, "max_position_embeddings": 514,
        "type_vocab_size": 1, "layer_norm_eps": 1e-5, "hidden_act": "gelu", "pad_token_id": 1,
        "num_labels": 1}


@pytest.mark.parametrize("cfgd", [BERT, XLMR])
def test_tei_encoders_gpu_match_cpu(cfgd):
    """BGE-style embeddings (CLS, normalised) and the XLM-R reranker score on the GPU path
    (HIP LayerNorm + non-causal prefill attention) vs the fp32 CPU model, same weights."""
    from enterprise_inference_amd.entrypoints.tei.server import EmbeddingEngine

    def eng(dev):
        cfg = EngineConfig(model=ModelConfig.from_hf_dict(cfgd, name="m"), device=dev,
                           dtype=torch.bfloat16 if dev == "cuda" else torch.float32,
                           served_model_name="m", load_format="dummy")
        return EmbeddingEngine(cfg, max_batch_tokens=4096)

    import transformers
    if cfgd is BERT:
        hc = transformers.BertConfig(**{k: v for k, v in cfgd.items() if k != "architectures"})
        torch.manual_seed(0)
        hf = transformers.BertModel(hc, add_pooling_layer=False).eval()
    else:
        hc = transformers.XLMRobertaConfig(**{k: v for k, v in cfgd.items()
                                              if k not in ("architectures", "model_type")})
        torch.manual_seed(1)
        hf = transformers.XLMRobertaForSequenceClassification(hc).eval()
    cpu, gpu = eng("cpu"), eng("cuda")
    for e in (cpu, gpu):           # HF checkpoint names -> both engines' loaders
        e.model.load_weights(hf.state_dict().items())
    gen = torch.Generator().manual_seed(1)
    seqs = [torch.randint(5, 900, (n,), generator=gen).tolist() for n in (7, 130, 64, 300)]
    encs = [(s, None) for s in seqs]
    if cfgd is BERT:
        fn = lambda e: e._run(encs, "embed_norm")                          # noqa: E731
        a, b = torch.stack(fn(gpu)), torch.stack(fn(cpu))
        cos = torch.nn.functional.cosine_similarity(a, b, dim=-1)
        assert cos.min().item() > 0.995, cos
    else:
        fn = lambda e: e._run(encs, "rerank")                              # noqa: E731
        a, b = torch.stack(fn(gpu)), torch.stack(fn(cpu))
        assert (a - b).abs().max().item() < 0.03 * (1 + b.abs().max().item()), (a, b)


def test_kv_swap_under_pressure_matches_fp32_oracle():
    """K14 on the GPU path (HIP graphs, overlap): pinned-host swap-out/in of KV blocks.  Batch
    compositions differ from an unpressured run (other GEMM buckets, other bf16 rounding), so
    the check is teacher-forced against the fp32 oracle, which catches a corrupted block."""
    d = tiny_config("LlamaForCausalLM", **SHAPE)
    hf = hf_reference_model(d)
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d),
                       cache=CacheConfig(block_size=128, num_gpu_blocks=12, swap_space_gb=1.0,
                                         enable_prefix_caching=False),
                       scheduler=SchedulerConfig(max_num_seqs=16, max_num_batched_tokens=512,
                                                 max_model_len=2048),
                       device="cuda", dtype=torch.bfloat16, load_format="dummy")
    eng = LLMEngine(cfg)
    eng.executor.runner.model.load_weights(hf.state_dict().items())
    gen = torch.Generator().manual_seed(4)
    prompts = [torch.randint(3, 1000, (200 + 37 * i,), generator=gen).tolist() for i in range(6)]
    params = SamplingParams(max_tokens=100, temperature=0, ignore_eos=True)
    outs = eng.generate(prompt_token_ids=prompts, params=params)   # ~18 blocks needed, 12 here
    assert eng.scheduler.num_swapouts > 0
    toks = [o.outputs[0].token_ids for o in outs]
    stats = check_greedy(hf, prompts, toks, tol=0.08)
    assert stats["argmax_agreement"] > 0.8, stats


def test_llama4_vision_gpu_matches_fp32_oracle():
    """Llama-4 on the GPU path (interleaved RoPE + NoPE layer, qk L2-norm, chunked local
    attention, a top-1 MoE layer with a shared expert) with an image: the vision tower runs
    bf16 on the GPU, its embeddings replace the placeholder tokens inside a chunked prefill,
    and every generated token is teacher-forced against HF Llama4ForConditionalGeneration fp32
    on the CPU with the same weights and pixels."""
    import transformers

    IMG = 1000
    text = tiny_config("Llama4ForCausalLM", **SHAPE, num_local_experts=4,
                       num_experts_per_tok=1, intermediate_size_mlp=2048,
                       attention_chunk_size=256, no_rope_layers=[1, 0], use_qk_norm=True,
                       interleave_moe_layer_step=1, moe_layers=[1])
    text = {k: v for k, v in text.items() if k != "architectures"}
    vision = {"hidden_size": 256, "intermediate_size": 1024, "num_hidden_layers": 2,
              "num_attention_heads": 4, "image_size": 112, "patch_size": 14,
              "pixel_shuffle_ratio": 0.5, "projector_input_dim": 512,
              "projector_output_dim": 512, "vision_output_dim": 512, "rope_theta": 10000.0,
              "num_channels": 3}
    d = {"architectures": ["Llama4ForConditionalGeneration"], "text_config": text,
         "vision_config": vision, "image_token_index": IMG}
    vc = transformers.Llama4VisionConfig(**{k: v for k, v in vision.items() if k != "rope_theta"},
                                         rope_parameters={"rope_theta": 10000.0,
                                                          "rope_type": "default"})
    hc = transformers.Llama4Config(text_config=transformers.Llama4TextConfig(**text).to_dict(),
                                   vision_config=vc.to_dict(), image_token_index=IMG)
    for c in (hc, hc.text_config, hc.vision_config):
        c._attn_implementation = "eager"
    torch.manual_seed(0)
    hf = transformers.Llama4ForConditionalGeneration(hc).float().eval()
    eng = _engine(d)
    model = eng.executor.runner.model
    assert model.vision is not None and model.vision.tokens_per_tile == 16
    model.load_weights(hf.state_dict().items())
    gen = torch.Generator().manual_seed(2)
    pv = torch.randn(3, 3, 112, 112, generator=gen)                   # 3 tiles -> 48 tokens
    prompt = (torch.randint(3, 990, (230,), generator=gen).tolist() + [IMG] * 48 +
              torch.randint(3, 990, (120,), generator=gen).tolist())    # spans prefill chunks
    n = 16
    out = eng.generate(prompt_token_ids=[prompt],
                       params=SamplingParams(max_tokens=n, temperature=0, ignore_eos=True),
                       multi_modal_data=[{"image": [pv]}])[0]
    toks = out.outputs[0].token_ids
    assert len(toks) == n
    with torch.no_grad():
        lg = hf(input_ids=torch.tensor([prompt + toks]), pixel_values=pv).logits[0].float()
    rows = lg[len(prompt) - 1:len(prompt) - 1 + n]
    margins = rows.max(-1).values - rows.gather(1, torch.tensor(toks)[:, None])[:, 0]
    assert float(margins.max()) < 0.08, margins
    assert float((margins == 0).float().mean()) > 0.8, margins
