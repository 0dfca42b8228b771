"""TEI-compatible embedding / rerank server (§2.14).

Drop-in for the text-embeddings-inference container the reference's ``tei`` and
``teirerank`` charts run: configuration from env ``MODEL_ID`` / ``PORT``
(core/helm-charts/tei/templates/configmap.yaml:10-11, 2081 embed / 2082 rerank),
argv ``--auto-truncate`` (core/helm-charts/tei/templates/deployment.yaml:53),
``MAX_WARMUP_SEQUENCE_LENGTH`` warmup (core/helm-charts/tei/gaudi-values.yaml:11).

Routes: ``POST /embed``, ``POST /rerank {query, texts}`` (Postman collection
core/catalog/AI-Inference-as-Service-postman-collection.json:518-541),
``POST /v1/embeddings`` (OpenAI form, docs/api-spec.yaml:50), ``GET /health``,
``GET /info``, ``GET /metrics``.

  python -m enterprise_inference_amd.entrypoints.tei.server --model-id BAAI/bge-base-en-v1.5
"""

from __future__ import annotations

import argparse
import asyncio
import base64
import collections
import concurrent.futures
import logging
import os
import queue
import struct
import sys
import threading
import time
from typing import List, Optional, Union

import torch
from fastapi import FastAPI
from fastapi.responses import JSONResponse, Response
from pydantic import BaseModel, ConfigDict

from ..openai.protocol import (EmbeddingRequest, EmbeddingResponse, EmbeddingResponseData,
                               UsageInfo)

logger = logging.getLogger(__name__)


class EmbeddingEngine:
    """Batched encoder inference on one GPU (or the CPU path).

    Dynamic batching across requests (what TEI's router does): every request's sequences go
    into one queue, and a single worker thread packs whatever is waiting -- from any number of
    concurrent requests -- into varlen batches of up to ``max_batch_tokens`` (one forward
    each), so many single-document calls share a forward instead of running one by one.  A
    batch holds one kind of work (embedding with / without normalisation, or rerank)."""

    def __init__(self, cfg, max_batch_tokens: int = 16384, auto_truncate: bool = True):
        from ...models.loader import build_model
        from ...tokenizer import get_tokenizer

        self.cfg = cfg
        dev = torch.device("cuda", torch.cuda.current_device()) \
            if cfg.device == "cuda" and torch.cuda.is_available() else torch.device("cpu")
        self.device = dev
        if dev.type == "cuda":
            from ... import _native
            _native.kernels()
        self.model = build_model(cfg, dev)
        m = cfg.model
        self.model_name = cfg.served_model_name or m.name
        self.tokenizer = get_tokenizer(cfg.tokenizer or cfg.model_path, m.vocab_size,
                                       m.eos_token_id, m.bos_token_id, cfg.trust_remote_code,
                                       allow_byte_fallback=not cfg.strict_tokenizer)
        self.max_len = m.max_position_embeddings - m.position_offset
        self.max_batch_tokens = max_batch_tokens
        self.auto_truncate = auto_truncate
        self.is_reranker = m.architecture.endswith("SequenceClassification")
        self.stats = {"requests": 0, "tokens": 0, "batches": 0, "batch_seqs": 0}
        self._q: "queue.Queue" = queue.Queue()
        self._worker: Optional[threading.Thread] = None
        self._worker_lock = threading.Lock()

    # ------------------------------------------------------------------ tokenise
    def _encode(self, text: str, pair: Optional[str] = None, truncate: bool = True):
        tok = self.tokenizer
        if pair is not None and hasattr(tok, "__call__") and tok.__class__.__name__ != "ByteTokenizer":
            enc = tok(text, pair, truncation=truncate, max_length=self.max_len)
            ids = enc["input_ids"]
            tt = enc.get("token_type_ids")
        else:
            ids = tok.encode(text if pair is None else f"{text} {pair}")
            tt = None
        if len(ids) > self.max_len:
            if not (truncate or self.auto_truncate):
                raise ValueError(f"input of {len(ids)} tokens exceeds the maximum of {self.max_len}")
            ids = ids[:self.max_len]
            tt = tt[:self.max_len] if tt else None
        return ids, tt

    def _batches(self, encs):
        batch, tok = [], 0
        for i, e in enumerate(encs):
            n = len(e[0])
            if batch and tok + n > self.max_batch_tokens:
                yield batch
                batch, tok = [], 0
            batch.append(i)
            tok += n
        if batch:
            yield batch

    def _fn(self, key):
        if key == "rerank":
            return lambda b: self.model(b)
        return lambda b: self.model(b, normalize=key == "embed_norm")

    def _ensure_worker(self) -> None:
        with self._worker_lock:
            if self._worker is None or not self._worker.is_alive():
                self._worker = threading.Thread(target=self._loop, name="tei-batcher",
                                                daemon=True)
                self._worker.start()

    def _loop(self) -> None:
        carry: collections.deque = collections.deque()   # left for the next batch, in order
        while True:
            pending = list(carry)
            carry.clear()
            if not pending:
                pending.append(self._q.get())
            while True:                     # everything already waiting
                try:
                    pending.append(self._q.get_nowait())
                except queue.Empty:
                    break
            key = pending[0][2]
            batch, tok = [], 0
            for item in pending:            # FIFO: one kind, up to the token budget
                if item[2] == key and (not batch or tok + len(item[0]) <= self.max_batch_tokens):
                    batch.append(item)
                    tok += len(item[0])
                else:
                    carry.append(item)
            self._forward(batch, key)

    @torch.no_grad()
    def _forward(self, batch, key) -> None:
        from ...models.bert import EncoderBatch
        try:
            seqs = [it[0] for it in batch]
            tts = [it[1] or [0] * len(it[0]) for it in batch]
            b = EncoderBatch(seqs, tts, self.device, self.cfg.model.position_offset)
            res = self._fn(key)(b).float().cpu()
            self.stats["tokens"] += sum(len(x) for x in seqs)
            self.stats["batches"] += 1
            self.stats["batch_seqs"] += len(seqs)
            for j, it in enumerate(batch):
                it[3].set_result(res[j])
        except Exception as e:   # noqa: BLE001 - delivered to every waiting request
            for it in batch:
                if not it[3].done():
                    it[3].set_exception(e)

    def _run(self, encs, key):
        """Queue this request's sequences for the batcher and wait for their outputs."""
        self._ensure_worker()
        futs = []
        for ids, tt in encs:
            f: concurrent.futures.Future = concurrent.futures.Future()
            self._q.put((ids, tt, key, f))
            futs.append(f)
        out = [f.result() for f in futs]
        self.stats["requests"] += 1
        return out

    def embed(self, texts: List[str], normalize: bool = True, truncate: bool = True,
              dimensions: Optional[int] = None) -> List[List[float]]:
        if self.is_reranker:
            raise ValueError("this model is a reranker; use /rerank")
        encs = [self._encode(t, truncate=truncate) for t in texts]
        vecs = self._run(encs, "embed_norm" if normalize and not dimensions else "embed")
        if dimensions:
            vecs = [torch.nn.functional.normalize(v[:dimensions], dim=-1) if normalize else
                    v[:dimensions] for v in vecs]
        return [v.tolist() for v in vecs]

    def rerank(self, query: str, texts: List[str], raw_scores: bool = False,
               truncate: bool = True) -> List[float]:
        if not self.is_reranker:
            raise ValueError("this model is an embedding model; use /embed")
        encs = [self._encode(query, t, truncate=truncate) for t in texts]
        logits = self._run(encs, "rerank")
        out = []
        for l in logits:
            s = float(l[0]) if l.numel() == 1 else float(torch.softmax(l, -1)[-1])
            out.append(s if raw_scores or l.numel() > 1 else 1.0 / (1.0 + pow(2.718281828459045, -s)))
        return out

    def count_tokens(self, texts: List[str]) -> int:
        return sum(len(self._encode(t)[0]) for t in texts)

    def warmup(self, seq_len: int = 512) -> None:
        n = min(seq_len, self.max_len)
        encs = [([self.tokenizer.bos_token_id or 0] * n, None)]
        self._run(encs, "rerank" if self.is_reranker else "embed_norm")


class EmbedRequest(BaseModel):
    model_config = ConfigDict(extra="allow")
    inputs: Union[str, List[str]]
    normalize: bool = True
    truncate: Optional[bool] = None
    prompt_name: Optional[str] = None


class RerankRequest(BaseModel):
    model_config = ConfigDict(extra="allow")
    query: str
    texts: List[str]
    raw_scores: bool = False
    return_text: bool = False
    truncate: Optional[bool] = None


def _err(msg: str, code: int = 422, kind: str = "validation"):
    return JSONResponse({"error": msg, "error_type": kind}, status_code=code)


def register_openai_embeddings(app: FastAPI, emb: EmbeddingEngine, model_name: str) -> None:
    @app.post("/v1/embeddings")
    async def v1_embeddings(req: EmbeddingRequest):
        if req.model and req.model != model_name:
            return JSONResponse({"object": "error", "message": f"The model `{req.model}` does not "
                                 "exist.", "type": "NotFoundError", "code": 404}, status_code=404)
        inp = req.input
        if isinstance(inp, str):
            texts = [inp]
        elif inp and isinstance(inp[0], int):
            texts = [emb.tokenizer.decode(inp)]
        elif inp and isinstance(inp[0], list):
            texts = [emb.tokenizer.decode(x) for x in inp]
        else:
            texts = list(inp)
        try:
            vecs = await asyncio.to_thread(emb.embed, texts, True, True, req.dimensions)
        except ValueError as e:
            return JSONResponse({"object": "error", "message": str(e), "type": "BadRequestError",
                                 "code": 400}, status_code=400)
        data = []
        for i, v in enumerate(vecs):
            if req.encoding_format == "base64":
                v = base64.b64encode(struct.pack(f"<{len(v)}f", *v)).decode()
            data.append(EmbeddingResponseData(index=i, embedding=v))
        ntok = emb.count_tokens(texts)
        return JSONResponse(EmbeddingResponse(model=model_name, data=data,
                                              usage=UsageInfo(prompt_tokens=ntok,
                                                              total_tokens=ntok)).model_dump())


def build_tei_app(emb: EmbeddingEngine) -> FastAPI:
    from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest

    app = FastAPI(title="enterprise-inference-amd TEI")
    reg = CollectorRegistry()
    req_count = Counter("te_request_count", "Requests", ["method"], registry=reg)
    req_lat = Histogram("te_request_duration", "Request duration (s)", ["method"], registry=reg)
    name = emb.model_name

    @app.get("/health")
    async def health():
        return Response(status_code=200)

    @app.get("/info")
    async def info():
        return {"model_id": name, "model_type": "reranker" if emb.is_reranker else "embedding",
                "max_input_length": emb.max_len, "max_batch_tokens": emb.max_batch_tokens,
                "auto_truncate": emb.auto_truncate, "version": "enterprise-inference-amd"}

    @app.get("/metrics")
    async def metrics():
        return Response(generate_latest(reg), media_type="text/plain; version=0.0.4")

    @app.post("/embed")
    async def embed(req: EmbedRequest):
        t0 = time.time()
        texts = [req.inputs] if isinstance(req.inputs, str) else req.inputs
        try:
            vecs = await asyncio.to_thread(emb.embed, texts, req.normalize,
                                           req.truncate if req.truncate is not None else True)
        except ValueError as e:
            return _err(str(e))
        req_count.labels(method="embed").inc()
        req_lat.labels(method="embed").observe(time.time() - t0)
        return vecs

    @app.post("/rerank")
    async def rerank(req: RerankRequest):
        t0 = time.time()
        try:
            scores = await asyncio.to_thread(emb.rerank, req.query, req.texts, req.raw_scores,
                                             req.truncate if req.truncate is not None else True)
        except ValueError as e:
            return _err(str(e))
        out = [{"index": i, "score": s} for i, s in enumerate(scores)]
        if req.return_text:
            for o in out:
                o["text"] = req.texts[o["index"]]
        out.sort(key=lambda o: -o["score"])
        req_count.labels(method="rerank").inc()
        req_lat.labels(method="rerank").observe(time.time() - t0)
        return out

    register_openai_embeddings(app, emb, name)
    return app


def main(argv=None) -> int:
    import uvicorn

    from ...config import CacheConfig, EngineConfig
    from ...models.loader import resolve_model_config
    from ..cli_args import normalise_argv, resolve_model_source

    logging.basicConfig(level=os.environ.get("EIA_LOG_LEVEL", "INFO"))
    ap = argparse.ArgumentParser(description="TEI-compatible embedding/rerank server (MI355X)")
    ap.add_argument("--model-id", default=os.environ.get("MODEL_ID", "BAAI/bge-base-en-v1.5"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("PORT", 2081)))
    ap.add_argument("--hostname", default=os.environ.get("HOSTNAME_BIND", "0.0.0.0"))
    ap.add_argument("--auto-truncate", action="store_true")
    ap.add_argument("--max-batch-tokens", type=int,
                    default=int(os.environ.get("MAX_BATCH_TOKENS", 16384)))
    ap.add_argument("--dtype", default=os.environ.get("DTYPE", "bfloat16"))
    ap.add_argument("--pooling", default=os.environ.get("POOLING", "cls"))
    ap.add_argument("--load-format", default=os.environ.get("LOAD_FORMAT", "auto"),
                    choices=["auto", "safetensors", "pt", "dummy"],
                    help="dummy: random weights (benchmarks); otherwise download / load")
    ap.add_argument("--huggingface-hub-cache", default=os.environ.get("HF_HUB_CACHE"))
    ap.add_argument("--root-path", default=os.environ.get("ROOT_PATH"),
                    help="URL prefix stripped from request paths (EKS ALB without APISIX)")
    args, unknown = ap.parse_known_args(normalise_argv(list(sys.argv[1:] if argv is None else argv)))
    if unknown:
        logger.warning("ignoring unsupported arguments: %s", unknown)
    path, cfg_id = resolve_model_source(args.model_id, args.huggingface_hub_cache,
                                        args.load_format)
    mcfg = resolve_model_config(cfg_id)
    gpu = torch.cuda.is_available()
    cfg = EngineConfig(model=mcfg, cache=CacheConfig(), device="cuda" if gpu else "cpu",
                       dtype=torch.bfloat16 if gpu else torch.float32,
                       model_path=path if args.load_format != "dummy" else None,
                       served_model_name=args.model_id, tokenizer=path,
                       load_format=args.load_format,
                       strict_tokenizer=args.load_format != "dummy")
    emb = EmbeddingEngine(cfg, args.max_batch_tokens, args.auto_truncate)
    if hasattr(emb.model, "pooling"):
        emb.model.pooling = args.pooling
    emb.warmup(int(os.environ.get("MAX_WARMUP_SEQUENCE_LENGTH", 512)))
    app = build_tei_app(emb)
    if args.root_path and args.root_path.strip("/"):
        from ..openai.api_server import _StripPrefix
        app.add_middleware(_StripPrefix, prefix=args.root_path)
    from ...utils.gc_tuning import tune_after_startup
    tune_after_startup()
    uvicorn.run(app, host=args.hostname, port=args.port)
    return 0


if __name__ == "__main__":
    sys.exit(main())
