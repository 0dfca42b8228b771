"""K14 KV swap: under KV pressure, preempted sequences park their blocks in the host swap
space and resume from them; greedy tokens equal an unpressured run (and the recompute
path), the swap metrics move, and aborting a swapped request frees its host blocks."""

import torch

from enterprise_inference_amd.config import CacheConfig, EngineConfig, ModelConfig, SchedulerConfig
from enterprise_inference_amd.engine.llm_engine import LLMEngine
from enterprise_inference_amd.engine.sampling_params import SamplingParams
from enterprise_inference_amd.models.catalog import tiny_config


def _engine(blocks, swap_gb):
    d = tiny_config("LlamaForCausalLM", vocab_size=320)
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d),
                       cache=CacheConfig(block_size=16, num_gpu_blocks=blocks,
                                         swap_space_gb=swap_gb, enable_prefix_caching=False),
                       scheduler=SchedulerConfig(max_num_seqs=8, max_num_batched_tokens=64,
                                                 max_model_len=256),
                       device="cpu", dtype=torch.float32, load_format="dummy")
    return LLMEngine(cfg)


PROMPTS = [list(range(3 + i, 40 + i)) for i in range(6)]
PARAMS = SamplingParams(max_tokens=40, temperature=0, ignore_eos=True)


def test_swap_preemption_matches_unpressured_run():
    ref = [o.outputs[0].token_ids for o in
           _engine(256, 0).generate(prompt_token_ids=PROMPTS, params=PARAMS)]
    eng = _engine(24, 0.01)          # 6 x (37 + 40) tokens need ~30 blocks of 16
    assert eng.scheduler.swap is not None and eng.scheduler.swap.num_blocks > 0
    got = [o.outputs[0].token_ids for o in eng.generate(prompt_token_ids=PROMPTS, params=PARAMS)]
    assert eng.scheduler.num_swapouts > 0, "the pressured run must swap"
    assert got == ref
    assert eng.scheduler.swap.usage() == 0.0 and not eng.scheduler.swapped


def test_recompute_fallback_without_swap_space():
    ref = [o.outputs[0].token_ids for o in
           _engine(256, 0).generate(prompt_token_ids=PROMPTS, params=PARAMS)]
    eng = _engine(24, 0)
    assert eng.scheduler.swap is None
    got = [o.outputs[0].token_ids for o in eng.generate(prompt_token_ids=PROMPTS, params=PARAMS)]
    assert eng.scheduler.num_preemptions > 0 and got == ref


def test_abort_swapped_request_frees_host_blocks():
    eng = _engine(24, 0.01)
    for i, p in enumerate(PROMPTS):
        eng.add_request(f"r{i}", prompt_token_ids=p, params=PARAMS)
    for _ in range(200):
        eng.step()
        if eng.scheduler.swapped:
            break
    assert eng.scheduler.swapped, "expected a swapped sequence"
    victim = eng.scheduler.swapped[0].request_id
    used = eng.scheduler.swap.usage()
    eng.abort_request(victim)
    assert eng.scheduler.swap.usage() < used
    while eng.has_unfinished_requests():
        eng.step()
    assert eng.scheduler.swap.usage() == 0.0
