"""Llama-4 vision path (models/llama4_vision.py) vs HF Llama4ForConditionalGeneration on the
CPU: tiny text + vision configs, the HF checkpoint's weights loaded into our engine, image
placeholders replaced by our tower's embeddings, greedy tokens equal HF's multimodal greedy
decode.  Also: tile preprocessing geometry, prompt expansion, and the engine's errors."""

import base64
import io

import numpy as np
import pytest
import torch

from enterprise_inference_amd.config import CacheConfig, EngineConfig, ModelConfig, SchedulerConfig
from enterprise_inference_amd.engine.llm_engine import LLMEngine
from enterprise_inference_amd.engine.sampling_params import SamplingParams
from enterprise_inference_amd.models.catalog import tiny_config
from enterprise_inference_amd.models.llama4_vision import (best_fit_canvas, expand_image_prompt,
                                                           preprocess)

IMG_TOK = 299


def _configs():
    text = tiny_config("Llama4ForCausalLM", num_local_experts=4, num_experts_per_tok=1,
                       intermediate_size=128, intermediate_size_mlp=256, head_dim=32,
                       num_hidden_layers=2, attention_chunk_size=64, no_rope_layers=[1, 0],
                       use_qk_norm=True, interleave_moe_layer_step=1, moe_layers=[],
                       vocab_size=300)
    # dense MLP layers: top-1 expert routing flips on near-tied router logits between any two
    # fp32 implementations and would blur what this test isolates (the image path)
    text = {k: v for k, v in text.items() if k != "architectures"}
    vision = {"hidden_size": 32, "intermediate_size": 128, "num_hidden_layers": 2,
              "num_attention_heads": 2, "image_size": 56, "patch_size": 14,
              "pixel_shuffle_ratio": 0.5, "projector_input_dim": 64, "projector_output_dim": 64,
              "vision_output_dim": 64, "rope_theta": 10000.0, "num_channels": 3}
    d = {"architectures": ["Llama4ForConditionalGeneration"], "text_config": text,
         "vision_config": vision, "image_token_index": IMG_TOK}
    return d, text, vision


def _hf(d, text, vision):
    import transformers
    tc = transformers.Llama4TextConfig(**text)
    vc = transformers.Llama4VisionConfig(**{k: v for k, v in vision.items() if k != "rope_theta"},
                                         rope_parameters={"rope_theta": 10000.0,
                                                          "rope_type": "default"})
    cfg = transformers.Llama4Config(text_config=tc.to_dict(), vision_config=vc.to_dict(),
                                    image_token_index=IMG_TOK)
    cfg._attn_implementation = "eager"
    cfg.text_config._attn_implementation = "eager"
    cfg.vision_config._attn_implementation = "eager"
    torch.manual_seed(0)
    return transformers.Llama4ForConditionalGeneration(cfg).eval()


@pytest.mark.parametrize("lead", [15, 44])      # 44: the 8 image tokens straddle the 48-token chunk
def test_vision_greedy_matches_transformers(lead):
    d, text, vision = _configs()
    hf = _hf(d, text, vision)
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d),
                       cache=CacheConfig(block_size=16, num_gpu_blocks=64),
                       scheduler=SchedulerConfig(max_num_seqs=4, max_num_batched_tokens=48,
                                                 max_model_len=512),
                       device="cpu", dtype=torch.float32, load_format="dummy")
    eng = LLMEngine(cfg)
    model = eng.executor.runner.model
    assert model.vision is not None and model.vision.tokens_per_tile == 4
    loaded = model.load_weights(hf.state_dict().items())
    assert any(n.startswith(("vision_model", "model.vision_model")) for n in loaded)
    torch.manual_seed(1)
    pv = torch.randn(2, 3, 56, 56)                       # 2 tiles -> 8 placeholder tokens
    prompt = list(range(10, 10 + lead)) + [IMG_TOK] * 8 + list(range(100, 130))   # chunked
    n = 5
    out = eng.generate(prompt_token_ids=[prompt],
                       params=SamplingParams(max_tokens=n, temperature=0, ignore_eos=True),
                       multi_modal_data=[{"image": [pv]}])[0]
    # teacher forcing: every token of ours is the fp32 oracle's argmax up to near-ties
    toks = out.outputs[0].token_ids
    with torch.no_grad():
        lg = hf(input_ids=torch.tensor([prompt + toks]), pixel_values=pv).logits[0]
    rows = lg[len(prompt) - 1:len(prompt) - 1 + n]
    margins = (rows.max(-1).values - rows.gather(1, torch.tensor(toks)[:, None])[:, 0])
    assert float(margins.max()) < 1e-2, margins
    # and without the image the oracle disagrees somewhere (the embeddings were used)
    with torch.no_grad():
        lg_txt = hf(input_ids=torch.tensor([prompt + toks])).logits[0]
    assert not torch.allclose(lg_txt[len(prompt) - 1], lg[len(prompt) - 1])
    # the image changes the continuation vs the same prompt without it
    plain = eng.generate(prompt_token_ids=[prompt],
                         params=SamplingParams(max_tokens=n, temperature=0, ignore_eos=True))[0]
    assert plain.outputs[0].token_ids != out.outputs[0].token_ids


def test_image_count_mismatch_is_a_client_error():
    d, _, _ = _configs()
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d), cache=CacheConfig(block_size=16,
                       num_gpu_blocks=16), device="cpu", dtype=torch.float32, load_format="dummy")
    eng = LLMEngine(cfg)
    with pytest.raises(ValueError, match="placeholder"):
        eng.add_request("r", prompt_token_ids=[5, 6, IMG_TOK, 7],
                        params=SamplingParams(max_tokens=2),
                        multi_modal_data={"image": [torch.randn(1, 3, 56, 56)]})


def test_preprocess_tiles_and_prompt_expansion():
    from PIL import Image
    img = Image.fromarray((np.random.rand(500, 900, 3) * 255).astype("uint8"))
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    url = "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()
    pv, (th, tw) = preprocess(url, max_tiles=16)
    assert best_fit_canvas(500, 900, 16) == (th * 336, tw * 336)
    assert pv.shape == (th * tw + (1 if th * tw > 1 else 0), 3, 336, 336)
    assert pv.min() >= -1.0 and pv.max() <= 1.0
    s = expand_image_prompt((th, tw), 144)
    assert s.count("<|patch|>") == 144 * (th * tw + (1 if th * tw > 1 else 0))
    assert s.startswith("<|image_start|>") and s.endswith("<|image_end|>")
    assert best_fit_canvas(300, 300, 16) == (336, 336)


def _png_data_url(h=70, w=130):
    from PIL import Image
    rng = np.random.default_rng(0)
    img = Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8))
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    return "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()


def test_openai_chat_image_parts(tmp_path):
    """/v1/chat/completions with an image_url content part on a (dummy-weight) Llama-4 vision
    checkpoint: the image becomes its tile/patch placeholder block, the engine runs the tower,
    and the response counts the placeholder tokens as prompt tokens."""
    import json

    from fastapi.testclient import TestClient

    from enterprise_inference_amd.entrypoints.cli_args import parse_args
    from enterprise_inference_amd.entrypoints.openai.api_server import build_from_args

    d, _, _ = _configs()
    d["text_config"]["max_position_embeddings"] = 2048
    (tmp_path / "config.json").write_text(json.dumps(d))
    args = parse_args(["--model", str(tmp_path), "--served-model-name", "tiny-l4v", "--device",
                       "cpu", "--load_format", "dummy", "--max-model-len", "1024",
                       "--max-num-seqs", "4", "--max_num_batched_tokens", "256",
                       "--block-size", "16", "--gpu-memory-util", "0.5",
                       "--disable-log-requests"])
    app, aeng = build_from_args(args, wait_ready=True)
    try:
        with TestClient(app) as c:
            def chat(content, **kw):
                return c.post("/v1/chat/completions", json={
                    "messages": [{"role": "user", "content": content}], "max_tokens": 3,
                    "temperature": 0, "ignore_eos": True, **kw})

            url = _png_data_url()
            _, (th, tw) = preprocess(url, tile=56)
            assert th * tw > 1
            r0 = chat([{"type": "text", "text": "describe"}])
            r1 = chat([{"type": "text", "text": "describe"},
                       {"type": "image_url", "image_url": {"url": url}}])
            assert r0.status_code == 200 and r1.status_code == 200, r1.text
            extra = r1.json()["usage"]["prompt_tokens"] - r0.json()["usage"]["prompt_tokens"]
            assert extra == (th * tw + 1) * 4     # tiles + global tile, 4 patches each
            assert r1.json()["usage"]["completion_tokens"] == 3
            two = chat([{"type": "image_url", "image_url": {"url": url}},
                        {"type": "text", "text": "and"},
                        {"type": "image_url", "image_url": {"url": url}}])
            assert two.status_code == 200, two.text
            bad = chat([{"type": "image_url", "image_url": {"url": "/etc/hostname"}}])
            assert bad.status_code == 400
            junk = chat([{"type": "image_url", "image_url": {"url": "data:image/png;base64,AAAA"}}])
            assert junk.status_code == 400
    finally:
        aeng.shutdown()


def _serve_bytes(payload: bytes, delay: float = 0.0):
    """Local HTTP server returning `payload` for every GET; returns (url, stop)."""
    import http.server
    import threading
    import time as _t

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            _t.sleep(delay)
            self.send_response(200)
            self.send_header("Content-Type", "image/png")
            self.end_headers()
            self.wfile.write(payload)

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return f"http://127.0.0.1:{srv.server_address[1]}/img.png", srv.shutdown


def test_remote_image_policy(monkeypatch):
    """http(s) image URLs: private/loopback targets refused by default (no SSRF into the
    cluster), domain allowlist, a streamed byte cap, and an off switch."""
    import base64

    from enterprise_inference_amd.models import llama4_vision as lv
    png = base64.b64decode(_png_data_url().split(",", 1)[1])
    url, stop = _serve_bytes(png)
    try:
        with pytest.raises(ValueError, match="non-public"):
            lv.fetch_image_bytes(url)
        monkeypatch.setenv("EIA_ALLOW_PRIVATE_MEDIA", "1")
        assert lv.fetch_image_bytes(url) == png
        assert lv.load_image(url).size[0] > 0
        with pytest.raises(ValueError, match="exceeds"):
            lv.fetch_image_bytes(url, max_bytes=len(png) // 2)
        monkeypatch.setenv("EIA_ALLOWED_MEDIA_DOMAINS", "images.example.com")
        with pytest.raises(ValueError, match="allowed media domains"):
            lv.fetch_image_bytes(url)
        monkeypatch.setenv("EIA_DISABLE_REMOTE_MEDIA", "1")
        with pytest.raises(ValueError, match="disabled"):
            lv.fetch_image_bytes(url)
    finally:
        stop()


def test_remote_image_dns_rebinding_pinned(monkeypatch):
    """A resolver that answers a public address for the policy check and the metadata
    address afterwards must not steer the fetch: the request dials the address the check
    validated (Host header and SNI keep the name), and the name is resolved once."""
    import contextlib
    import socket

    from enterprise_inference_amd.models import llama4_vision as lv
    answers = iter(["93.184.216.34", "169.254.169.254", "169.254.169.254"])
    lookups = []

    def fake_getaddrinfo(host, port, *a, **k):
        lookups.append(host)
        return [(socket.AF_INET, socket.SOCK_STREAM, 6, "", (next(answers), port))]

    seen = {}

    class _Resp:
        is_redirect = False
        headers = {"content-length": "3"}
        extensions = {}

        def raise_for_status(self):
            pass

        def iter_bytes(self):
            yield b"abc"

    @contextlib.contextmanager
    def fake_stream(url, headers, extensions, timeout, trust_env=False):
        seen.update(url=url, headers=headers, ext=extensions, trust_env=trust_env)
        yield _Resp()

    for k in ("HTTPS_PROXY", "https_proxy", "HTTP_PROXY", "http_proxy", "ALL_PROXY",
              "all_proxy"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(socket, "getaddrinfo", fake_getaddrinfo)
    monkeypatch.setattr(lv, "_open_stream", fake_stream)
    assert lv.fetch_image_bytes("https://img.example.com:8443/a.png") == b"abc"
    assert lookups == ["img.example.com"]
    assert seen["url"] == "https://93.184.216.34:8443/a.png"
    assert seen["headers"] == {"Host": "img.example.com:8443"}
    assert seen["ext"] == {"sni_hostname": "img.example.com"}
    assert seen["trust_env"] is False         # the pinned dial ignores proxy settings

    # a peer address other than the validated one is refused before the body is read
    class _Stream:
        def get_extra_info(self, k):
            return ("10.0.0.5", 443) if k == "server_addr" else None

    _Resp.extensions = {"network_stream": _Stream()}
    answers = iter(["93.184.216.34"])
    with pytest.raises(ValueError, match="unexpected address"):
        lv.fetch_image_bytes("https://img.example.com/a.png")


def test_remote_image_through_egress_proxy(monkeypatch):
    """With HTTPS_PROXY set (enterprise egress), the policy check still resolves and vets the
    name, and the PINNED target (the validated address, SNI / Host = the name) goes through
    the proxy, so the proxy never resolves the name itself; the peer check (which would see
    the proxy's address) is skipped; NO_PROXY matches the name."""
    import contextlib
    import socket

    from enterprise_inference_amd.models import llama4_vision as lv
    seen = {}

    class _Stream:
        def get_extra_info(self, k):
            return ("10.1.2.3", 3128) if k == "server_addr" else None   # the proxy

    class _Resp:
        is_redirect = False
        headers = {"content-length": "3"}
        extensions = {"network_stream": _Stream()}

        def raise_for_status(self):
            pass

        def iter_bytes(self):
            yield b"abc"

    @contextlib.contextmanager
    def fake_stream(url, headers, extensions, timeout, trust_env=False):
        seen.update(url=url, headers=headers, ext=extensions, trust_env=trust_env)
        yield _Resp()

    def fake_getaddrinfo(host, port, *a, **k):
        return [(socket.AF_INET, socket.SOCK_STREAM, 6, "", ("93.184.216.34", port))]

    @contextlib.contextmanager
    def fake_proxied(url, headers, extensions, timeout, proxy):
        seen.update(url=url, headers=headers, ext=extensions, proxy=proxy, trust_env=None)
        yield _Resp()

    monkeypatch.setattr(socket, "getaddrinfo", fake_getaddrinfo)
    monkeypatch.setattr(lv, "_open_stream", fake_stream)
    monkeypatch.setattr(lv, "_open_proxied_stream", fake_proxied)
    monkeypatch.setenv("HTTPS_PROXY", "http://proxy.corp:3128")
    monkeypatch.delenv("NO_PROXY", raising=False)
    monkeypatch.delenv("no_proxy", raising=False)
    assert lv.fetch_image_bytes("https://img.example.com/a.png") == b"abc"
    assert seen["url"] == "https://93.184.216.34/a.png"
    assert seen["ext"] == {"sni_hostname": "img.example.com"}
    assert seen["headers"] == {"Host": "img.example.com"}
    assert seen["proxy"] == "http://proxy.corp:3128"
    # the host is exempted by NO_PROXY: back to the pinned direct dial
    monkeypatch.setenv("NO_PROXY", "img.example.com")
    _Resp.extensions = {}
    assert lv.fetch_image_bytes("https://img.example.com/a.png") == b"abc"
    assert seen["url"] == "https://93.184.216.34/a.png" and seen["trust_env"] is False


def test_slow_image_url_does_not_block_event_loop(monkeypatch):
    """The image download runs on a worker thread: while one request waits 1.5 s on a slow
    image URL, the event loop keeps serving other coroutines."""
    import asyncio
    import time as _t

    from enterprise_inference_amd.entrypoints.openai import serving

    calls = []

    def slow_expand(ctx, prompt, images, add_special):
        _t.sleep(1.5)
        calls.append(1)
        raise serving.RequestError("done")

    monkeypatch.setattr(serving, "_expand_images", slow_expand)

    class Ctx:
        model = "m"
        chat_template = None
        tokenizer = None

        def check_model(self, m):
            pass

    monkeypatch.setattr(serving, "apply_chat_template", lambda *a, **k: "prompt")
    req = serving.ChatCompletionRequest(model="m", messages=[{"role": "user", "content": [
        {"type": "image_url", "image_url": {"url": "http://slow.example.com/x.png"}}]}])

    async def main():
        ticks = 0

        async def ticker():
            nonlocal ticks
            while not calls:
                await asyncio.sleep(0.05)
                ticks += 1

        t = asyncio.create_task(ticker())
        with pytest.raises(serving.RequestError):
            await serving.create_chat_completion(req, Ctx())
        await t
        return ticks

    assert asyncio.run(main()) >= 10


def test_http_image_via_local_proxy_dials_pinned_address(monkeypatch):
    """End to end over a real socket: a forward proxy on 127.0.0.1 receives the absolute-form
    request for the VALIDATED address (not the name, which it would resolve again) with the
    name in Host, through _open_proxied_stream / http.client."""
    import socket
    import threading

    from enterprise_inference_amd.models import llama4_vision as lv

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    got = {}

    def serve():
        c, _ = srv.accept()
        data = b""
        while b"\r\n\r\n" not in data:
            data += c.recv(4096)
        got["head"] = data.decode()
        c.sendall(b"HTTP/1.1 200 OK\r\nContent-Length: 3\r\nConnection: close\r\n\r\nxyz")
        c.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    real = socket.getaddrinfo

    def fake_getaddrinfo(host, port, *a, **k):
        if host == "img.example.com":
            return [(socket.AF_INET, socket.SOCK_STREAM, 6, "", ("93.184.216.34", port))]
        return real(host, port, *a, **k)

    monkeypatch.setattr(socket, "getaddrinfo", fake_getaddrinfo)
    for k in ("NO_PROXY", "no_proxy", "ALL_PROXY", "all_proxy", "http_proxy"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("HTTP_PROXY", f"http://user:pw@127.0.0.1:{srv.getsockname()[1]}")
    assert lv.fetch_image_bytes("http://img.example.com/a.png?x=1") == b"xyz"
    t.join(5)
    srv.close()
    line, *hdrs = got["head"].split("\r\n")
    assert line == "GET http://93.184.216.34/a.png?x=1 HTTP/1.1", line
    assert "Host: img.example.com" in hdrs
    assert any(h.startswith("Proxy-Authorization: Basic ") for h in hdrs)
