"""OpenAI server on the CPU path: schema, SSE framing, include_usage, tools, metrics, health.

Mirrors the reference's manual API checks (Postman collection
core/catalog/AI-Inference-as-Service-postman-collection.json, curl recipes in
docs/accessing-deployed-models.md:137-203) as automated tests.
"""

import json

import pytest
from fastapi.testclient import TestClient

from enterprise_inference_amd.entrypoints.cli_args import parse_args


@pytest.fixture(scope="module")
def server(tmp_path_factory):
    import os
    from enterprise_inference_amd.models import catalog

    d = tmp_path_factory.mktemp("tiny")
    cfg = catalog.tiny_config(vocab_size=300, max_position_embeddings=2048)
    (d / "config.json").write_text(json.dumps(cfg))
    from enterprise_inference_amd.entrypoints.openai.api_server import build_from_args
    args = parse_args(["--model", str(d), "--served-model-name", "tiny-llama", "--device", "cpu",
                       "--load_format", "dummy", "--max-model-len", "1024", "--max-num-seqs", "8",
                       "--max_num_batched_tokens", "128", "--block-size", "16",
                       "--tool-call-parser", "llama3_json", "--enable-auto-tool-choice",
                       "--chat-template",
                       "/workspace/vllm/examples/tool_chat_template_llama3.1_json.jinja",
                       "--gpu-memory-util", "0.5", "--num_scheduler_steps", "1",
                       "--use-padding-aware-scheduling", "--disable-log-requests"])
    app, aeng = build_from_args(args, wait_ready=True)
    with TestClient(app) as c:
        yield c
    aeng.shutdown()


def test_health_models_version(server):
    assert server.get("/health").status_code == 200
    m = server.get("/v1/models").json()
    assert m["data"][0]["id"] == "tiny-llama" and m["data"][0]["max_model_len"] == 1024
    assert "version" in server.get("/version").json()


def test_completion_basic(server):
    r = server.post("/v1/completions", json={"model": "tiny-llama", "prompt": "hello world",
                                              "max_tokens": 5, "temperature": 0,
                                              "ignore_eos": True})
    assert r.status_code == 200, r.text
    j = r.json()
    assert j["object"] == "text_completion"
    assert j["usage"]["completion_tokens"] == 5
    assert j["choices"][0]["finish_reason"] == "length"


def test_completion_batch_n_logprobs_echo(server):
    r = server.post("/v1/completions", json={"prompt": ["ab", "cd"], "max_tokens": 3, "n": 2,
                                              "logprobs": 2, "echo": True, "ignore_eos": True,
                                              "seed": 7})
    j = r.json()
    assert len(j["choices"]) == 4
    for c in j["choices"]:
        assert c["text"].startswith(("ab", "cd"))
        lp = c["logprobs"]
        assert len(lp["tokens"]) == 3 and len(lp["top_logprobs"]) == 3


def test_greedy_is_deterministic(server):
    body = {"prompt": [5, 6, 7, 8], "max_tokens": 6, "temperature": 0, "ignore_eos": True}
    a = server.post("/v1/completions", json=body).json()["choices"][0]["text"]
    b = server.post("/v1/completions", json=body).json()["choices"][0]["text"]
    assert a == b


def _sse(resp):
    frames = [l for l in resp.iter_lines() if l]
    assert frames[-1] == "data: [DONE]"
    return [json.loads(f[len("data: "):]) for f in frames[:-1]]


def test_completion_stream_include_usage(server):
    with server.stream("POST", "/v1/completions",
                       json={"prompt": "xyz", "max_tokens": 4, "stream": True, "ignore_eos": True,
                             "stream_options": {"include_usage": True}}) as r:
        chunks = _sse(r)
    assert chunks[-1]["choices"] == [] and chunks[-1]["usage"]["completion_tokens"] == 4
    assert any(c["choices"] and c["choices"][0].get("finish_reason") == "length" for c in chunks)


def test_chat_and_stream(server):
    msgs = [{"role": "system", "content": "be brief"}, {"role": "user", "content": "hi"}]
    r = server.post("/v1/chat/completions", json={"model": "tiny-llama", "messages": msgs,
                                                   "max_tokens": 4, "ignore_eos": True,
                                                   "logprobs": True, "top_logprobs": 2})
    j = r.json()
    assert j["object"] == "chat.completion" and j["choices"][0]["message"]["role"] == "assistant"
    assert len(j["choices"][0]["logprobs"]["content"]) == 4
    with server.stream("POST", "/v1/chat/completions",
                       json={"messages": msgs, "max_tokens": 3, "stream": True, "ignore_eos": True,
                             "stream_options": {"include_usage": True}}) as r:
        chunks = _sse(r)
    assert chunks[0]["choices"][0]["delta"]["role"] == "assistant"
    assert chunks[-1]["usage"]["completion_tokens"] == 3


def test_chat_forced_tool_and_guided_choice(server):
    tools = [{"type": "function", "function": {"name": "get_weather", "parameters": {
        "type": "object", "properties": {"city": {"type": "string", "enum": ["Paris", "Oslo"]}},
        "required": ["city"]}}}]
    r = server.post("/v1/chat/completions", json={
        "messages": [{"role": "user", "content": "weather?"}], "tools": tools,
        "tool_choice": {"type": "function", "function": {"name": "get_weather"}},
        "max_tokens": 40})
    j = r.json()
    call = j["choices"][0]["message"]["tool_calls"][0]["function"]
    assert call["name"] == "get_weather"
    assert json.loads(call["arguments"])["city"] in ("Paris", "Oslo")
    r = server.post("/v1/completions", json={"prompt": "pick", "max_tokens": 10,
                                              "guided_choice": ["yes", "no"]})
    assert r.json()["choices"][0]["text"] in ("yes", "no")


def test_errors(server):
    assert server.post("/v1/completions", json={"model": "other", "prompt": "x"}).status_code == 404
    assert server.post("/v1/completions", json={"prompt": "x" * 1100}).status_code == 400
    assert server.post("/v1/completions", json={"prompt": "x", "top_p": 2}).status_code == 400
    r = server.post("/v1/embeddings", json={"input": "x"})
    assert r.status_code == 400


def test_metrics_contract(server):
    server.post("/v1/completions", json={"prompt": "m", "max_tokens": 2, "ignore_eos": True})
    text = server.get("/metrics").text
    for name in ["vllm:e2e_request_latency_seconds_bucket", "vllm:prompt_tokens_total",
                 "vllm:generation_tokens_total", "vllm:time_per_output_token_seconds_bucket",
                 "vllm:num_requests_running", "vllm:num_requests_swapped",
                 "vllm:num_requests_waiting", "vllm:time_to_first_token_seconds_bucket",
                 "vllm:gpu_cache_usage_perc", "vllm:cpu_cache_usage_perc",
                 "vllm:request_prompt_tokens_bucket", "vllm:request_generation_tokens_bucket",
                 "vllm:request_success_total"]:
        assert name in text, name
    assert 'model_name="tiny-llama"' in text


def test_tokenize_roundtrip(server):
    t = server.post("/tokenize", json={"prompt": "abc"}).json()
    assert t["count"] == len(t["tokens"])
    assert "abc" in server.post("/detokenize", json={"tokens": t["tokens"]}).json()["prompt"]


@pytest.mark.parametrize("text,finish,stop", [("hi", None, None), ('a "q" \\ é\n日本', "stop", None),
                                              ("", "length", None), ("x", "stop", 128009),
                                              ("y", "stop", "</s>")])
def test_fast_sse_chunks_match_pydantic(text, finish, stop):
    """The hand-framed SSE hot path is JSON-equal to the pydantic models it replaces."""
    from enterprise_inference_amd.entrypoints.openai import serving as sv
    from enterprise_inference_amd.entrypoints.openai.protocol import (
        ChatCompletionResponseStreamChoice, ChatCompletionStreamResponse, CompletionStreamChoice,
        CompletionStreamResponse, DeltaMessage)

    def body(frame):
        assert frame.startswith("data: ") and frame.endswith("\n\n")
        return json.loads(frame[6:-2])

    ref = sv._sse(CompletionStreamResponse(
        id="cmpl-1", created=7, model="m/x", choices=[CompletionStreamChoice(
            index=3, text=text, finish_reason=finish, stop_reason=stop)]))
    got = sv.fast_completion_chunk(sv.completion_chunk_head("cmpl-1", 7, "m/x"), 3, text,
                                   finish, stop)
    assert body(got) == body(ref)
    ref = sv._sse(ChatCompletionStreamResponse(
        id="chatcmpl-1", created=7, model="m/x", choices=[ChatCompletionResponseStreamChoice(
            index=0, delta=DeltaMessage(content=text or None, tool_calls=[]),
            finish_reason=finish, stop_reason=stop)]))
    got = sv.fast_chat_chunk(sv.chat_chunk_head("chatcmpl-1", 7, "m/x"), 0, text, finish, stop)
    assert body(got) == body(ref)


def test_openapi_spec_in_sync():
    """docs/api-spec.yaml is generated from the apps (scripts/gen_openapi.py) and current."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "gen_openapi.py"), "--check"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    import yaml
    with open(os.path.join(root, "docs", "api-spec.yaml")) as f:
        doc = yaml.safe_load(f)
    for p in ("/v1/chat/completions", "/v1/completions", "/v1/embeddings", "/embed", "/rerank"):
        assert p in doc["paths"], p


def test_requests_reach_engine_before_stream_iterates(monkeypatch):
    """Handlers hand a request to the engine while they run (engine.submit), not when the
    streaming response first advances its iterator -- a burst of concurrent requests then
    reaches the engine core together; engines without submit keep the lazy generate."""
    from enterprise_inference_amd.entrypoints.openai import serving

    calls = []

    class Eager:
        can_submit = True

        def submit(self, rid, prompt, params, **kw):
            calls.append(("submit", rid, kw.get("prompt_token_ids")))

            async def it():
                yield "out"
            return it()

    class Lazy:
        def generate(self, rid, prompt, params, **kw):
            calls.append(("generate-created", rid))

            async def it():
                calls.append(("generate-started", rid))
                yield "out"
            return it()

    serving._start(Eager(), "r1", None, None, prompt_token_ids=[1, 2])
    assert calls == [("submit", "r1", [1, 2])]
    calls.clear()
    g = serving._start(Lazy(), "r2", None, None)
    assert calls == [("generate-created", "r2")]
    monkeypatch.setattr(serving, "EAGER_SUBMIT", False)
    calls.clear()

    class Both(Eager, Lazy):
        pass
    serving._start(Both(), "r3", None, None)
    assert calls == [("generate-created", "r3")]
    del g


def test_submitted_request_released_when_stream_never_iterates():
    """Eager submit registers the request before its output generator starts; a stream that
    is dropped unstarted (client gone before the response body, a later prompt of the same
    completion failing) must still abort the request in the core and forget it, and a stream
    iterated to completion must not send an abort."""
    import asyncio
    import gc

    from enterprise_inference_amd.engine.core_proc import MPEngineClient

    class Out:
        def __init__(self, finished):
            self.finished = finished

    async def scenario():
        c = MPEngineClient.__new__(MPEngineClient)
        c._reqs, c.dead, c.ready, c._last_msg = {}, None, False, 0.0
        sent = []
        c._send = sent.append

        class W:
            def is_closing(self):
                return False
        c._writer = W()
        s = c.submit("a", None, None, prompt_token_ids=[1, 2])
        assert "a" in c._reqs and sent[-1][0] == "add"
        del s
        gc.collect()
        assert "a" not in c._reqs and sent[-1] == ("abort", "a")
        s = c.submit("b", None, None, prompt_token_ids=[3])
        c._reqs["b"].queue.put_nowait(Out(False))
        c._reqs["b"].queue.put_nowait(Out(True))
        got = [o.finished async for o in s]
        assert got == [False, True] and "b" not in c._reqs
        del s
        gc.collect()
        assert [f for f in sent if f[0] == "abort"] == [("abort", "a")]
        s = c.submit("c", None, None, prompt_token_ids=[4])   # closed mid-stream
        c._reqs["c"].queue.put_nowait(Out(False))
        assert (await s.__anext__()).finished is False
        await s.aclose()
        assert "c" not in c._reqs and sent[-1] == ("abort", "c")
        assert [f for f in sent if f == ("abort", "c")] == [("abort", "c")]

    asyncio.run(scenario())
