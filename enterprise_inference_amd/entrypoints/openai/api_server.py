"""OpenAI-compatible HTTP server.

Replaces the vLLM serving container the reference's ``vllm`` chart launches:
same port 2080 (core/helm-charts/vllm/values.yaml:21), same argv contract
(core/helm-charts/vllm/templates/deployment.yaml:66-87), ``GET /health`` for the
readiness probe (values.yaml:135-141), ``GET /metrics`` for the ServiceMonitor
(templates/servicemonitor.yaml:15-19), OpenAI ``/v1/completions``,
``/v1/chat/completions``, ``/v1/embeddings``, ``/v1/models``
(docs/api-spec.yaml:6-72), plus ``/tokenize``, ``/detokenize``, ``/version``.

  python -m enterprise_inference_amd.entrypoints.openai.api_server \\
      --model meta-llama/Llama-3.1-8B-Instruct --port 2080 --tensor-parallel-size 1 ...
"""

from __future__ import annotations

import logging
import os
import sys
from typing import Optional

from fastapi import FastAPI, Request
from fastapi.exceptions import RequestValidationError
from fastapi.responses import JSONResponse, Response, StreamingResponse

from ...engine.async_engine import AsyncLLMEngine, EngineDeadError
from ...version import __version__
from ..cli_args import engine_config_from_args, make_parser, parse_args
from .chat_utils import resolve_chat_template
from .protocol import (ChatCompletionRequest, CompletionRequest, EmbeddingRequest,
                       ErrorResponse, ModelCard, ModelList)
from .serving import RequestError, ServingContext, create_chat_completion, create_completion

logger = logging.getLogger(__name__)


def _error(msg: str, code: int, kind: str) -> JSONResponse:
    return JSONResponse(ErrorResponse(message=msg, type=kind, code=code).model_dump(),
                        status_code=code)


def build_app(ctx: ServingContext, metrics=None, embedder=None, api_key: Optional[str] = None,
              served_model_name: Optional[str] = None) -> FastAPI:
    """FastAPI app over a ServingContext (LLM) and/or an embedding engine (TEI-style)."""
    app = FastAPI(title="enterprise-inference-amd", version=__version__)
    model_name = served_model_name or (ctx.model if ctx else embedder.model_name)

    @app.middleware("http")
    async def auth(request: Request, call_next):
        if api_key and request.url.path.startswith("/v1"):
            if request.headers.get("Authorization") != f"Bearer {api_key}":
                return _error("Unauthorized", 401, "AuthenticationError")
        return await call_next(request)

    @app.exception_handler(RequestValidationError)
    async def validation_error(_, exc):
        return _error(str(exc), 400, "BadRequestError")

    @app.exception_handler(RequestError)
    async def request_error(_, exc: RequestError):
        return _error(str(exc), exc.code, exc.kind)

    @app.exception_handler(EngineDeadError)
    async def engine_dead(_, exc):
        return _error(str(exc), 500, "InternalServerError")

    @app.exception_handler(ValueError)
    async def value_error(_, exc):
        return _error(str(exc), 400, "BadRequestError")

    @app.get("/health")
    async def health():
        if ctx is not None:
            eng = ctx.engine
            if eng.dead is not None:
                return Response(status_code=500)
            if not eng.healthy:
                return Response(status_code=503)
        return Response(status_code=200)

    @app.get("/ping")
    async def ping():
        return await health()

    @app.get("/version")
    async def version():
        return {"version": __version__}

    @app.get("/metrics")
    async def metrics_route():
        from ...metrics import CONTENT_TYPE_LATEST
        body = metrics.render() if metrics is not None else b""
        return Response(body, media_type=CONTENT_TYPE_LATEST)

    @app.get("/v1/models")
    async def models():
        mml = ctx.max_model_len if ctx else None
        return ModelList(data=[ModelCard(id=model_name, root=model_name, max_model_len=mml)])

    if ctx is not None:
        @app.post("/v1/completions")
        async def completions(req: CompletionRequest, raw: Request):
            res = await create_completion(req, ctx)
            if req.stream:
                return StreamingResponse(res, media_type="text/event-stream")
            return JSONResponse(res.model_dump(exclude_none=True))

        @app.post("/v1/chat/completions")
        async def chat(req: ChatCompletionRequest, raw: Request):
            res = await create_chat_completion(req, ctx)
            if req.stream:
                return StreamingResponse(res, media_type="text/event-stream")
            return JSONResponse(res.model_dump(exclude_none=True))

        @app.post("/tokenize")
        async def tokenize(body: dict):
            if "messages" in body:
                from .chat_utils import apply_chat_template
                text = apply_chat_template(ctx.tokenizer, body["messages"], ctx.chat_template,
                                           add_generation_prompt=body.get(
                                               "add_generation_prompt", True))
                ids = ctx.tokenizer.encode(text, add_special_tokens=False)
            else:
                ids = ctx.tokenizer.encode(body.get("prompt", ""),
                                           add_special_tokens=body.get("add_special_tokens", True))
            return {"tokens": ids, "count": len(ids), "max_model_len": ctx.max_model_len}

        @app.post("/detokenize")
        async def detokenize(body: dict):
            return {"prompt": ctx.tokenizer.decode(body.get("tokens", []))}

        from ...utils.profiling import profiler_dir
        if profiler_dir():
            # vLLM-compatible profiler control (only with EIA/VLLM_TORCH_PROFILER_DIR set)
            import asyncio as _asyncio

            @app.post("/start_profile")
            async def start_profile():
                eng = ctx.engine
                await _asyncio.wrap_future(eng.call_in_engine_thread(eng.engine.profiler.start))
                return Response(status_code=200)

            @app.post("/stop_profile")
            async def stop_profile():
                eng = ctx.engine
                path = await _asyncio.wrap_future(
                    eng.call_in_engine_thread(eng.engine.profiler.stop))
                return JSONResponse({"trace": path})

    if embedder is not None:
        from ..tei.server import register_openai_embeddings
        register_openai_embeddings(app, embedder, model_name)
    else:
        @app.post("/v1/embeddings")
        async def embeddings_unsupported(req: EmbeddingRequest):
            raise RequestError(f"The model `{model_name}` does not support embeddings; deploy it "
                               "with the tei chart (BERT / XLM-R encoders).", 400)

    return app


def build_from_args(args):
    """Engine + app for parsed CLI args (used by ``main`` and the in-process tests)."""
    from ...engine.llm_engine import LLMEngine
    from ...metrics import EngineMetrics

    cfg = engine_config_from_args(args)
    if cfg.model.is_encoder:
        from ..tei.server import EmbeddingEngine
        emb = EmbeddingEngine(cfg)
        metrics = EngineMetrics(cfg.served_model_name)
        return build_app(None, metrics, embedder=emb, api_key=args.api_key,
                         served_model_name=cfg.served_model_name), None
    if cfg.parallel.world_size > 1 or os.environ.get("WORLD_SIZE"):
        from ...parallel import state as pstate
        if os.environ.get("WORLD_SIZE"):
            pstate.init_distributed(cfg.parallel.tensor_parallel_size,
                                    enable_expert_parallel=cfg.parallel.enable_expert_parallel,
                                    pp_size=cfg.parallel.pipeline_parallel_size)
    engine = LLMEngine(cfg)
    metrics = EngineMetrics(cfg.served_model_name)
    aengine = AsyncLLMEngine(engine, metrics, log_requests=not args.disable_log_requests)
    gen_defaults = dict(args.override_generation_config or {})
    ctx = ServingContext(aengine, cfg.served_model_name, cfg.scheduler.max_model_len,
                         chat_template=resolve_chat_template(args.chat_template),
                         tool_parser=args.tool_call_parser,
                         enable_auto_tool_choice=args.enable_auto_tool_choice,
                         generation_defaults=gen_defaults)
    return build_app(ctx, metrics, api_key=args.api_key), aengine


def main(argv=None) -> int:
    import uvicorn

    logging.basicConfig(level=os.environ.get("EIA_LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    args = parse_args(argv, make_parser())
    app, aengine = build_from_args(args)
    logger.info("serving %s on %s:%d", (args.served_model_name or [args.model])[0], args.host,
                args.port)
    try:
        uvicorn.run(app, host=args.host, port=args.port, log_level=args.uvicorn_log_level,
                    timeout_keep_alive=5)
    finally:
        if aengine is not None:
            aengine.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
