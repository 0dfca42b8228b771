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


class _BearerAuth:
    """``Authorization: Bearer <api_key>`` on ``/v1/*`` (vLLM ``--api-key`` semantics)."""

    def __init__(self, app, api_key: str):
        self.app = app
        self.expected = f"Bearer {api_key}".encode()

    async def __call__(self, scope, receive, send):
        if scope["type"] == "http" and scope["path"].startswith("/v1"):
            auth = dict(scope.get("headers") or []).get(b"authorization")
            if auth != self.expected:
                await _error("Unauthorized", 401, "AuthenticationError")(scope, receive, send)
                return
        await self.app(scope, receive, send)


class _StripPrefix:
    """``--root-path /<prefix>``: requests arrive as /<prefix>/v1/... (EKS ALB paths cannot
    be rewritten) and are served as /v1/...; unprefixed paths (kubelet probes) pass as is."""

    def __init__(self, app, prefix: str):
        self.app = app
        self.prefix = "/" + prefix.strip("/")

    async def __call__(self, scope, receive, send):
        if scope["type"] == "http":
            path = scope["path"]
            if path == self.prefix or path.startswith(self.prefix + "/"):
                scope = dict(scope, path=path[len(self.prefix):] or "/",
                             raw_path=(path[len(self.prefix):] or "/").encode())
        await self.app(scope, receive, send)


def bench_endpoints_enabled() -> bool:
    return os.environ.get("EIA_BENCH_ENDPOINTS", "0") not in ("0", "", "false")


def build_app(ctx: ServingContext, metrics=None, embedder=None, api_key: Optional[str] = None,
              served_model_name: Optional[str] = None, wait_ready: bool = False,
              root_path: Optional[str] = None) -> FastAPI:
    """FastAPI app over a ServingContext (LLM) and/or an embedding engine (TEI-style)."""
    app = FastAPI(title="enterprise-inference-amd", version=__version__)
    model_name = served_model_name or (ctx.model if ctx else embedder.model_name)

    if api_key:
        # Pure ASGI middleware (Starlette's BaseHTTPMiddleware re-streams every SSE chunk
        # through anyio memory streams: ~25 us/chunk of API-process CPU at 13k chunks/s).
        app.add_middleware(_BearerAuth, api_key=api_key)
    if root_path and root_path.strip("/"):
        # added last = outermost: the auth check above sees the stripped /v1/... path
        app.add_middleware(_StripPrefix, prefix=root_path)

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
                # still loading / capturing graphs, or a step exceeded the watchdog
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

        if bench_endpoints_enabled():
            # benchmark control, opt-in (EIA_BENCH_ENDPOINTS=1, set by bench.py for the servers
            # it starts): a device sync between steps defeats overlapped scheduling, so a
            # production pod never exposes it
            @app.post("/eia/sync")
            async def engine_sync():
                """Barrier with the device: returns once the engine drained its GPU queue
                (bench.py brackets its timed region with it)."""
                await ctx.engine.run_op("sync")
                return {"ok": True}

            @app.get("/eia/stats")
            async def engine_stats():
                return await ctx.engine.run_op("stats")

        from ...utils.profiling import profiler_dir
        if profiler_dir():
            # vLLM-compatible profiler control (only with EIA/VLLM_TORCH_PROFILER_DIR set)
            @app.post("/start_profile")
            async def start_profile():
                await ctx.engine.run_op("profile_start")
                return Response(status_code=200)

            @app.post("/stop_profile")
            async def stop_profile():
                return JSONResponse({"trace": await ctx.engine.run_op("profile_stop")})

        async def _start_engine():
            await ctx.engine.start()
            if wait_ready:      # tests: serve only once the engine core reported ready
                await ctx.engine.wait_ready()

        app.router.on_startup.append(_start_engine)

    if embedder is not None:
        from ..tei.server import register_openai_embeddings
        register_openai_embeddings(app, embedder, model_name)
    else:
        @app.post("/v1/embeddings")
        async def embeddings_unsupported(req: EmbeddingRequest):
            raise RequestError(f"The model `{model_name}` does not support embeddings; deploy it "
                               "with the tei chart (BERT / XLM-R encoders).", 400)

    return app


def build_from_args(args, engine_mode: Optional[str] = None, wait_ready: bool = False):
    """Engine + app for parsed CLI args (used by ``main`` and the in-process tests).

    ``engine_mode``: ``process`` (default for the server: the step loop runs in an
    engine-core process, engine/core_proc.py, and this process never touches the GPU) or
    ``thread`` (step loop on a thread of this process; tests, torchrun-launched TP ranks)."""
    from ...engine.llm_engine import LLMEngine
    from ...metrics import EngineMetrics

    cfg = engine_config_from_args(args)
    mode = engine_mode or getattr(args, "engine_mode", None) or \
        os.environ.get("EIA_ENGINE_MODE", "process")
    if cfg.model.is_encoder:
        from ..tei.server import EmbeddingEngine
        emb = EmbeddingEngine(cfg)
        metrics = EngineMetrics(cfg.served_model_name)
        return build_app(None, metrics, embedder=emb, api_key=args.api_key,
                         served_model_name=cfg.served_model_name,
                         root_path=getattr(args, "root_path", None)), None
    metrics = EngineMetrics(cfg.served_model_name)
    if os.environ.get("WORLD_SIZE"):
        mode = "thread"          # torchrun-launched TP rank 0: this process is the driver
    if mode == "process":
        from ...engine.core_proc import MPEngineClient
        env = {k: v for k, v in os.environ.items()
               if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
               and not k.startswith("TORCHELASTIC_")}
        aengine = MPEngineClient(cfg, metrics, log_requests=not args.disable_log_requests,
                                 env=env)
    else:
        if os.environ.get("WORLD_SIZE"):
            from ...parallel import state as pstate
            pstate.init_distributed(cfg.parallel.tensor_parallel_size,
                                    backend=cfg.parallel.dist_backend,
                                    enable_expert_parallel=cfg.parallel.enable_expert_parallel,
                                    pp_size=cfg.parallel.pipeline_parallel_size)
        engine = LLMEngine(cfg)
        aengine = AsyncLLMEngine(engine, metrics, log_requests=not args.disable_log_requests)
    gen_defaults = dict(args.override_generation_config or {})
    ctx = ServingContext(aengine, cfg.served_model_name, cfg.scheduler.max_model_len,
                         chat_template=resolve_chat_template(args.chat_template),
                         tool_parser=args.tool_call_parser,
                         enable_auto_tool_choice=args.enable_auto_tool_choice,
                         generation_defaults=gen_defaults)
    return build_app(ctx, metrics, api_key=args.api_key, wait_ready=wait_ready,
                     root_path=getattr(args, "root_path", None)), aengine


def main(argv=None) -> int:
    import uvicorn

    logging.basicConfig(level=os.environ.get("EIA_LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    args = parse_args(argv, make_parser())
    app, aengine = build_from_args(args)
    logger.info("serving %s on %s:%d", (args.served_model_name or [args.model])[0], args.host,
                args.port)
    if os.environ.get("EIA_API_CPROFILE"):      # host-side profile of the API process
        import cProfile
        import pstats
        prof = cProfile.Profile()
        prof.enable()

        async def _dump_profile():
            prof.disable()
            with open(os.environ["EIA_API_CPROFILE"], "w") as f:
                pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(60)

        app.router.on_shutdown.append(_dump_profile)
    from ...utils.gc_tuning import tune_after_startup
    tune_after_startup()
    if aengine is not None:
        _exit_on_engine_death(aengine)
    try:
        uvicorn.run(app, host=args.host, port=args.port, log_level=args.uvicorn_log_level,
                    timeout_keep_alive=5)
    finally:
        if aengine is not None:
            aengine.shutdown()
    return 1 if aengine is not None and aengine.dead is not None else 0


def _exit_on_engine_death(aengine, grace_s: Optional[float] = None) -> None:
    """A dead engine (step exception, custom all-reduce error, lost TP worker) keeps answering
    ``/health`` with 500 for ``EIA_ENGINE_DEATH_GRACE_S`` (default 10 s: probes and clients see
    the failure), then the server shuts down and ``main`` exits non-zero so the pod restarts."""
    import signal
    import threading
    import time

    grace = float(os.environ.get("EIA_ENGINE_DEATH_GRACE_S", 10)) if grace_s is None else grace_s

    def watch():
        while aengine.dead is None:
            time.sleep(0.5)
        logger.critical("engine is dead (%s); shutting the server down in %.0f s",
                        aengine.dead, grace)
        time.sleep(grace)
        os.kill(os.getpid(), signal.SIGTERM)

    threading.Thread(target=watch, name="eia-death-watch", daemon=True).start()


if __name__ == "__main__":
    sys.exit(main())
