"""BERT / XLM-R encoders (TEI embed + rerank) and OPT vs HF transformers on the CPU path."""

import json

import pytest
import torch
from fastapi.testclient import TestClient

from enterprise_inference_amd.config import CacheConfig, EngineConfig, ModelConfig, SchedulerConfig
from enterprise_inference_amd.models.bert import BertEmbeddingModel, CrossEncoderModel, EncoderBatch

BERT = {"architectures": ["BertModel"], "hidden_size": 64, "intermediate_size": 128,
        "num_hidden_layers": 2, "num_attention_heads": 4, "vocab_size": 300,
        "max_position_embeddings": 128, "type_vocab_size": 2, "layer_norm_eps": 1e-12,
        "hidden_act": "gelu", "pad_token_id": 0}
XLMR = {"architectures": ["XLMRobertaForSequenceClassification"], "model_type": "xlm-roberta",
        "hidden_size": 64, "intermediate_size": 128, "num_hidden_layers": 2,
        "num_attention_heads": 4, "vocab_size": 300, "max_position_embeddings": 130,
        "type_vocab_size": 1, "layer_norm_eps": 1e-5, "hidden_act": "gelu", "pad_token_id": 1,
        "num_labels": 1}


def test_bert_matches_transformers():
    import transformers
    hc = transformers.BertConfig(**{k: v for k, v in BERT.items() if k != "architectures"})
    torch.manual_seed(0)
    hf = transformers.BertModel(hc, add_pooling_layer=False).eval()
    m = BertEmbeddingModel(ModelConfig.from_hf_dict(BERT), dtype=torch.float32)
    m.load_weights(hf.state_dict().items())
    seqs = [[2, 5, 9, 11, 3], [2, 7, 3]]
    b = EncoderBatch(seqs, None, "cpu")
    got = m(b, normalize=False)
    with torch.no_grad():
        for i, s in enumerate(seqs):
            ref = hf(torch.tensor([s])).last_hidden_state[0, 0]
            assert torch.allclose(got[i], ref, atol=1e-4), (got[i] - ref).abs().max()


def test_xlmr_reranker_matches_transformers():
    import transformers
    hc = transformers.XLMRobertaConfig(**{k: v for k, v in XLMR.items()
                                          if k not in ("architectures", "model_type")})
    torch.manual_seed(1)
    hf = transformers.XLMRobertaForSequenceClassification(hc).eval()
    cfg = ModelConfig.from_hf_dict(XLMR)
    m = CrossEncoderModel(cfg, dtype=torch.float32)
    m.load_weights(hf.state_dict().items())
    seqs = [[0, 5, 9, 2, 2, 17, 2], [0, 8, 2]]
    b = EncoderBatch(seqs, None, "cpu", cfg.position_offset)
    got = m(b)
    with torch.no_grad():
        for i, s in enumerate(seqs):
            ref = hf(torch.tensor([s])).logits[0]
            assert torch.allclose(got[i], ref, atol=1e-4), (got[i], ref)


@pytest.mark.parametrize("cfgd", [BERT, XLMR])
def test_tei_server(tmp_path, cfgd):
    from enterprise_inference_amd.entrypoints.tei.server import EmbeddingEngine, build_tei_app
    (tmp_path / "config.json").write_text(json.dumps(cfgd))
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(cfgd, name="m"), device="cpu",
                       dtype=torch.float32, served_model_name="m", load_format="dummy")
    emb = EmbeddingEngine(cfg, max_batch_tokens=64)
    c = TestClient(build_tei_app(emb))
    assert c.get("/health").status_code == 200
    info = c.get("/info").json()
    if cfgd is BERT:
        v = c.post("/embed", json={"inputs": ["hello", "a longer sentence here"]}).json()
        assert len(v) == 2 and abs(sum(x * x for x in v[0]) - 1.0) < 1e-3
        o = c.post("/v1/embeddings", json={"input": ["hi", "yo"], "model": "m"}).json()
        assert o["object"] == "list" and len(o["data"]) == 2 and o["usage"]["prompt_tokens"] > 0
        assert c.post("/rerank", json={"query": "q", "texts": ["a"]}).status_code == 422
        assert info["model_type"] == "embedding"
    else:
        r = c.post("/rerank", json={"query": "what", "texts": ["a", "bb", "ccc"],
                                    "return_text": True}).json()
        assert sorted(x["index"] for x in r) == [0, 1, 2]
        assert all(0.0 <= x["score"] <= 1.0 for x in r) and r[0]["score"] >= r[-1]["score"]
        assert info["model_type"] == "reranker"


def test_opt_matches_transformers():
    import transformers
    from enterprise_inference_amd.engine.llm_engine import LLMEngine
    from enterprise_inference_amd.engine.sampling_params import SamplingParams
    from enterprise_inference_amd.models.catalog import tiny_config

    d = tiny_config("OPTForCausalLM")
    hc = transformers.OPTConfig(**{k: v for k, v in d.items() if k != "architectures"})
    torch.manual_seed(0)
    hf = transformers.OPTForCausalLM(hc).eval()
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d),
                       cache=CacheConfig(block_size=16, num_gpu_blocks=32),
                       scheduler=SchedulerConfig(max_num_seqs=4, max_num_batched_tokens=32,
                                                 max_model_len=256),
                       device="cpu", dtype=torch.float32, load_format="dummy")
    eng = LLMEngine(cfg)
    eng.executor.runner.model.load_weights(hf.state_dict().items())
    prompt = [2, 11, 45, 7, 99, 100, 3, 5, 8, 13, 21, 34, 55, 89, 144, 233, 17, 18, 19, 20]
    out = eng.generate(prompt_token_ids=[prompt],
                       params=SamplingParams(max_tokens=8, temperature=0, ignore_eos=True))
    with torch.no_grad():
        ids = torch.tensor([prompt])
        ref = hf.generate(ids, max_new_tokens=8, do_sample=False)[0, len(prompt):].tolist()
    assert out[0].outputs[0].token_ids == ref


def test_tei_dynamic_batching_across_requests():
    """Concurrent single-document requests share forwards (TEI-style dynamic batching): the
    batcher packs what is waiting into one varlen batch up to max_batch_tokens, kinds never
    mix, and every request gets exactly its own rows back."""
    import threading

    import torch

    from enterprise_inference_amd.config import EngineConfig, ModelConfig
    from enterprise_inference_amd.entrypoints.tei.server import EmbeddingEngine
    from enterprise_inference_amd.models import catalog

    d = catalog.get_preset("BAAI/bge-base-en-v1.5")
    d.update(num_hidden_layers=2, hidden_size=64, intermediate_size=128, num_attention_heads=4)
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d, name="m"), device="cpu",
                       dtype=torch.float32, served_model_name="m", load_format="dummy")
    eng = EmbeddingEngine(cfg, max_batch_tokens=256)
    texts = [f"document number {i} " * (1 + i % 5) for i in range(24)]
    solo = [eng.embed([t])[0] for t in texts]             # one request at a time
    b0 = eng.stats["batches"]
    gate = threading.Event()
    res = [None] * len(texts)
    orig = eng._forward

    def slow_forward(batch, key):                           # first forward holds the worker
        gate.wait(5)
        orig(batch, key)
    eng._forward = slow_forward

    def one(i):
        res[i] = eng.embed([texts[i]], normalize=(i % 3 != 0))[0]
    th = [threading.Thread(target=one, args=(i,)) for i in range(len(texts))]
    for t in th:
        t.start()
    import time
    time.sleep(0.3)
    gate.set()
    for t in th:
        t.join(30)
    nb = eng.stats["batches"] - b0
    assert nb < len(texts) // 2, nb                         # requests shared forwards
    for i, t in enumerate(texts):
        want = torch.tensor(solo[i])
        got = torch.tensor(res[i])
        if i % 3 == 0:                                      # the unnormalised kind
            got = torch.nn.functional.normalize(got, dim=-1)
        assert torch.allclose(got, want, atol=1e-4), i
