"""CPU path: engine end-to-end, parity with HF transformers as an independent oracle."""

import pytest
import torch

from enterprise_inference_amd.config import CacheConfig, EngineConfig, ModelConfig, SchedulerConfig
from enterprise_inference_amd.engine.llm_engine import LLMEngine
from enterprise_inference_amd.engine.sampling_params import SamplingParams
from enterprise_inference_amd.models.catalog import tiny_config


def _engine(d, mbt=64, bs=16, nblocks=64, prefix=True, max_seqs=8):
    m = ModelConfig.from_hf_dict(d)
    cfg = EngineConfig(model=m, cache=CacheConfig(block_size=bs, num_gpu_blocks=nblocks,
                                                  enable_prefix_caching=prefix),
                       scheduler=SchedulerConfig(max_num_seqs=max_seqs, max_num_batched_tokens=mbt,
                                                 max_model_len=512),
                       device="cpu", dtype=torch.float32, load_format="dummy")
    return LLMEngine(cfg)


def _hf_model(d, arch):
    import transformers

    cls_cfg = {"LlamaForCausalLM": "LlamaConfig", "Qwen2ForCausalLM": "Qwen2Config",
               "Qwen3ForCausalLM": "Qwen3Config", "MistralForCausalLM": "MistralConfig",
               "MixtralForCausalLM": "MixtralConfig", "OPTForCausalLM": "OPTConfig"}[arch]
    hc = getattr(transformers, cls_cfg)(**{k: v for k, v in d.items() if k != "architectures"})
    torch.manual_seed(0)
    return getattr(transformers, arch)(hc).float().eval()


@pytest.mark.parametrize("arch", ["LlamaForCausalLM", "Qwen2ForCausalLM", "Qwen3ForCausalLM",
                                  "MistralForCausalLM"])
def test_parity_with_transformers(arch):
    d = tiny_config(arch)
    if arch == "LlamaForCausalLM":
        d["rope_scaling"] = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                             "high_freq_factor": 4.0, "original_max_position_embeddings": 256}
    hf = _hf_model(d, arch)
    eng = _engine(d, mbt=32)     # forces chunked prefill of the longer prompts
    eng.executor.runner.model.load_weights(hf.state_dict().items())
    cap = []
    r = eng.executor.runner
    orig = r._sample_tokens      # every sampling path (sync and overlapped) goes through it
    r._sample_tokens = lambda logits, items, plan, **kw: (cap.append(logits.clone()),
                                                          orig(logits, items, plan, **kw))[1]
    prompts = [[5, 6, 7, 8, 9] * 10, [3, 4, 5], list(range(10, 100))]
    eng.generate(prompt_token_ids=prompts, params=SamplingParams(max_tokens=1, temperature=0))
    with torch.no_grad():
        for i, p in enumerate(prompts):
            ref = hf(torch.tensor([p])).logits[0, -1]
            # find our row for this prompt: rows are emitted in scheduling order
            got = [c for c in cap if c.shape[-1] == ref.shape[-1]]
            assert any((g - ref).abs().max(-1).values.min() < 1e-4 for g in got), i


def test_greedy_generation_matches_transformers():
    d = tiny_config()
    hf = _hf_model(d, "LlamaForCausalLM")
    eng = _engine(d, mbt=48)
    eng.executor.runner.model.load_weights(hf.state_dict().items())
    prompts = [[3, 4, 5], list(range(10, 70))]
    outs = eng.generate(prompt_token_ids=prompts,
                        params=SamplingParams(max_tokens=10, temperature=0, ignore_eos=True))
    for p, o in zip(prompts, outs):
        g = hf.generate(torch.tensor([p]), max_new_tokens=10, do_sample=False, eos_token_id=None,
                        pad_token_id=0)[0, len(p):].tolist()
        assert o.outputs[0].token_ids == g


def test_prefix_cache_hit_and_same_output():
    d = tiny_config()
    eng = _engine(d, mbt=256)
    p = list(range(20, 120))
    sp = SamplingParams(max_tokens=5, temperature=0, ignore_eos=True)
    a = eng.generate(prompt_token_ids=[p], params=sp)[0]
    b = eng.generate(prompt_token_ids=[p], params=sp)[0]
    assert b.num_cached_tokens == 96          # 6 full blocks of 16 reused
    assert a.outputs[0].token_ids == b.outputs[0].token_ids
    assert eng.scheduler.bm.check_invariants() == ""


def test_preemption_recompute_keeps_output():
    d = tiny_config()
    sp = SamplingParams(max_tokens=40, temperature=0, ignore_eos=True)
    prompts = [list(range(10 + i, 40 + i)) for i in range(4)]
    ref = _engine(d, nblocks=64).generate(prompt_token_ids=prompts, params=sp)
    small = _engine(d, nblocks=12, prefix=False)     # 4 seqs x 70 tok needs 20 blocks
    out = small.generate(prompt_token_ids=prompts, params=sp)
    assert small.scheduler.num_preemptions > 0
    for a, b in zip(ref, out):
        assert a.outputs[0].token_ids == b.outputs[0].token_ids
    assert small.scheduler.bm.check_invariants() == ""


def test_stop_conditions_and_n():
    d = tiny_config()
    eng = _engine(d)
    o = eng.generate(prompt_token_ids=[[5, 6, 7]],
                     params=SamplingParams(max_tokens=7, temperature=0.8, seed=1, n=3))[0]
    assert len(o.outputs) == 3
    assert all(len(c.token_ids) <= 7 for c in o.outputs)
    first = o.outputs[0].token_ids
    o2 = eng.generate(prompt_token_ids=[[5, 6, 7]],
                      params=SamplingParams(max_tokens=7, temperature=0.8, seed=1, n=3))[0]
    assert o2.outputs[0].token_ids == first            # seeded sampling is reproducible
    stop_tok = first[2]
    o3 = eng.generate(prompt_token_ids=[[5, 6, 7]],
                      params=SamplingParams(max_tokens=7, temperature=0.8, seed=1,
                                            stop_token_ids=[stop_tok]))[0]
    c = o3.outputs[0]
    assert c.finish_reason == "stop" and c.stop_reason == stop_tok
    assert c.token_ids[-1] == stop_tok


def test_logprobs_and_penalties_run():
    d = tiny_config()
    eng = _engine(d)
    o = eng.generate(prompt_token_ids=[[5, 6, 7, 8]],
                     params=SamplingParams(max_tokens=4, temperature=0, logprobs=3,
                                           repetition_penalty=1.3, presence_penalty=0.5,
                                           frequency_penalty=0.5, logit_bias={7: 5.0}))[0]
    c = o.outputs[0]
    assert len(c.logprobs) == 4
    assert all(tok in lp for tok, lp in zip(c.token_ids, c.logprobs))
    assert all(len(lp) >= 3 for lp in c.logprobs)


def _mixed_requests():
    sp = [SamplingParams(max_tokens=12, temperature=0, ignore_eos=True),
          SamplingParams(max_tokens=9, temperature=0.9, seed=7, ignore_eos=True),
          SamplingParams(max_tokens=15, temperature=1.1, top_k=20, seed=3, ignore_eos=True),
          SamplingParams(max_tokens=6, temperature=0.7, seed=11, n=2, ignore_eos=True),
          SamplingParams(max_tokens=10, temperature=0.8, seed=5, ignore_eos=True,
                         repetition_penalty=1.2, presence_penalty=0.3)]
    prompts = [list(range(10 + 3 * i, 40 + 5 * i)) for i in range(len(sp))]
    return prompts, sp


@pytest.mark.parametrize("nblocks,prefix", [(64, True), (12, False)])
def test_overlapped_scheduling_matches_sync(nblocks, prefix):
    """Overlapped scheduling (step k+1 planned before step k's tokens are read back, inputs
    taken from the device) produces exactly the tokens of the synchronous engine, including
    under preemption and with penalty rows that force a read-back."""
    d = tiny_config()
    prompts, sp = _mixed_requests()
    outs = {}
    for overlap in (False, True):
        eng = _engine(d, nblocks=nblocks, prefix=prefix, mbt=48)
        eng._overlap = overlap
        outs[overlap] = eng.generate(prompt_token_ids=prompts, params=sp)
        assert eng._pending is None and not eng.has_unfinished_requests()
        assert eng.scheduler.bm.check_invariants() == ""
    for a, b in zip(outs[False], outs[True]):
        assert [c.token_ids for c in a.outputs] == [c.token_ids for c in b.outputs]
        assert [c.finish_reason for c in a.outputs] == [c.finish_reason for c in b.outputs]


def test_overlapped_scheduling_stops_and_streams():
    d = tiny_config()
    eng = _engine(d)
    assert eng._overlap
    p = [5, 6, 7, 8, 9]
    ref = eng.generate(prompt_token_ids=[p], params=SamplingParams(max_tokens=8, temperature=0))[0]
    stop_tok = ref.outputs[0].token_ids[3]
    eng.add_request("s", prompt_token_ids=p,
                    params=SamplingParams(max_tokens=8, temperature=0, stop_token_ids=[stop_tok]))
    streamed = []
    final = None
    while eng.has_unfinished_requests():
        for o in eng.step():
            streamed += o.outputs[0].new_token_ids
            if o.finished:
                final = o
    assert final.outputs[0].finish_reason == "stop"
    assert final.outputs[0].token_ids == ref.outputs[0].token_ids[:4]
    assert streamed == final.outputs[0].token_ids       # no token lost or duplicated


def test_overlap_decision_pinned():
    """The headline workload (temperature sampling, ignore_eos, no logprobs / penalties / stop
    strings) launches EVERY step ahead of the previous step's token read-back; a row that needs
    host-side processing (logprobs) makes exactly its steps synchronous."""
    d = tiny_config()
    eng = _engine(d)
    assert eng._overlap
    prompts = [list(range(10 + i, 30 + i)) for i in range(4)]
    eng.generate(prompt_token_ids=prompts,
                 params=SamplingParams(max_tokens=12, temperature=1.0, ignore_eos=True, seed=3))
    st = eng.stats
    assert st.num_sync_steps == 0 and st.num_overlapped_steps == st.num_steps > 0
    # a row with logprobs: its steps read the tokens back before the next launch
    eng.generate(prompt_token_ids=prompts[:1],
                 params=SamplingParams(max_tokens=5, temperature=1.0, ignore_eos=True, seed=3,
                                       logprobs=1))
    assert st.num_sync_steps >= 5
    assert st.num_overlapped_steps + st.num_sync_steps == st.num_steps
