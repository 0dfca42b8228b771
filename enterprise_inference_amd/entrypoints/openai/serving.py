"""Request handlers for ``/v1/completions`` and ``/v1/chat/completions``.

Streaming follows the OpenAI SSE framing the reference documents
(docs/api-spec.md:29-47, :73-87): ``data: {chunk}\\n\\n`` frames, a final chunk
carrying ``finish_reason``, an optional usage-only chunk when
``stream_options.include_usage`` is set (:113-122), then ``data: [DONE]``.
"""

from __future__ import annotations

import asyncio
import json
import os
import time
from typing import AsyncIterator, Dict, List, Optional, Tuple

from ...engine.async_engine import AsyncLLMEngine
from .chat_utils import apply_chat_template
from .protocol import (ChatCompletionRequest, ChatCompletionResponse,
                       ChatCompletionResponseChoice, ChatCompletionResponseStreamChoice,
                       ChatCompletionStreamResponse, ChatLogprobContent, ChatLogprobs,
                       ChatMessage, CompletionLogprobs, CompletionRequest, CompletionResponse,
                       CompletionResponseChoice, CompletionStreamChoice,
                       CompletionStreamResponse, DeltaFunctionCall, DeltaMessage, DeltaToolCall,
                       Logprob, UsageInfo, random_id)
from .tool_parsers import StreamingToolState, get_parser


class RequestError(ValueError):
    def __init__(self, msg: str, code: int = 400, kind: str = "BadRequestError"):
        super().__init__(msg)
        self.code = code
        self.kind = kind


def _sse(obj) -> str:
    data = obj if isinstance(obj, str) else obj.model_dump_json(exclude_none=True)
    return f"data: {data}\n\n"


# Hot-path SSE framing.  At the chatbot sizing row (65 streams x ~200 tok/s) the server frames
# ~13k chunks/s; building + validating + dumping a pydantic model per token costs ~25 us of
# API-process CPU each, string templates ~2 us.  Output is JSON-equal to
# ``_sse(CompletionStreamResponse(...))`` / ``_sse(ChatCompletionStreamResponse(...))`` for the
# plain-text case (no logprobs / tools / echo / continuous usage), which tests pin.
_dumps = json.JSONEncoder(ensure_ascii=False, separators=(",", ":")).encode


def _chunk_tail(finish_reason, stop_reason) -> str:
    t = ""
    if finish_reason is not None:
        t += ',"finish_reason":' + _dumps(finish_reason)
    if stop_reason is not None:
        t += ',"stop_reason":' + _dumps(stop_reason)
    return t + "}]}\n\n"


def completion_chunk_head(rid: str, created: int, model: str) -> str:
    return ('data: {"id":' + _dumps(rid) + ',"object":"text_completion","created":'
            + str(created) + ',"model":' + _dumps(model) + ',"choices":[{"index":')


def fast_completion_chunk(head: str, index: int, text: str, finish_reason=None,
                          stop_reason=None) -> str:
    return (head + str(index) + ',"text":' + _dumps(text)
            + _chunk_tail(finish_reason, stop_reason))


def chat_chunk_head(rid: str, created: int, model: str) -> str:
    return ('data: {"id":' + _dumps(rid) + ',"object":"chat.completion.chunk","created":'
            + str(created) + ',"model":' + _dumps(model) + ',"choices":[{"index":')


def fast_chat_chunk(head: str, index: int, content: Optional[str], finish_reason=None,
                    stop_reason=None) -> str:
    delta = ('{"content":' + _dumps(content) + ',"tool_calls":[]}') if content \
        else '{"tool_calls":[]}'
    return head + str(index) + ',"delta":' + delta + _chunk_tail(finish_reason, stop_reason)


EAGER_SUBMIT = os.environ.get("EIA_EAGER_SUBMIT", "1") != "0"


def _start(engine, request_id, prompt, params, **kw) -> AsyncIterator:
    """The request's output iterator, with the request already handed to the engine when the
    engine supports it (``submit``): a burst of concurrent requests then reaches the engine
    as their handlers run instead of when each streaming response first iterates."""
    if EAGER_SUBMIT and getattr(engine, "can_submit", False):
        return engine.submit(request_id, prompt, params, **kw)
    return engine.generate(request_id, prompt, params, **kw)


async def _merge(gens: List[AsyncIterator]) -> AsyncIterator[Tuple[int, object]]:
    """Interleave several async generators: yields (generator index, item)."""
    if len(gens) == 1:
        async for x in gens[0]:
            yield 0, x
        return
    q: asyncio.Queue = asyncio.Queue()
    done = object()

    async def pump(i, g):
        try:
            async for x in g:
                await q.put((i, x))
        except BaseException as e:   # noqa: BLE001
            await q.put((i, e))
        finally:
            await q.put((i, done))

    tasks = [asyncio.create_task(pump(i, g)) for i, g in enumerate(gens)]
    remaining = len(gens)
    try:
        while remaining:
            i, x = await q.get()
            if x is done:
                remaining -= 1
                continue
            if isinstance(x, BaseException):
                raise x
            yield i, x
    finally:
        for t in tasks:
            t.cancel()


class ServingContext:
    """State shared by the handlers (engine, tokenizer, model name, tool config)."""

    def __init__(self, engine: AsyncLLMEngine, served_model_name: str, max_model_len: int,
                 chat_template: Optional[str] = None, tool_parser: Optional[str] = None,
                 enable_auto_tool_choice: bool = False,
                 generation_defaults: Optional[Dict] = None):
        self.engine = engine
        self.tokenizer = engine.tokenizer
        self.model = served_model_name
        self.max_model_len = max_model_len
        self.chat_template = chat_template
        self.tool_parser = tool_parser
        if tool_parser:
            get_parser(tool_parser)
        self.enable_auto_tool_choice = enable_auto_tool_choice
        self.generation_defaults = generation_defaults or {}

    # ---------------------------------------------------------------- helpers
    def check_model(self, name: Optional[str]) -> None:
        if name and name != self.model:
            raise RequestError(f"The model `{name}` does not exist.", 404, "NotFoundError")

    def tokenize_prompt(self, prompt, add_special_tokens: bool = True,
                        truncate: Optional[int] = None) -> Tuple[Optional[str], List[int]]:
        if isinstance(prompt, str):
            ids = self.tokenizer.encode(prompt, add_special_tokens=add_special_tokens)
            text = prompt
        else:
            ids, text = list(prompt), None
        if truncate:
            ids = ids[-truncate:]
        if not ids:
            raise RequestError("prompt is empty")
        if len(ids) >= self.max_model_len:
            raise RequestError(
                f"This model's maximum context length is {self.max_model_len} tokens. However, "
                f"you requested {len(ids)} tokens in the prompt.")
        return text, ids

    def _tok_str(self, tid: int) -> str:
        try:
            return self.tokenizer.decode([tid], skip_special_tokens=False)
        except Exception:   # noqa: BLE001
            return ""

    def default_max_tokens(self, n_prompt: int) -> int:
        return max(1, self.max_model_len - n_prompt)


# ----------------------------------------------------------------------------- completions

def _prompts(req: CompletionRequest) -> List:
    p = req.prompt
    if isinstance(p, str):
        return [p]
    if isinstance(p, list) and p and isinstance(p[0], int):
        return [p]
    if isinstance(p, list) and p and isinstance(p[0], list):
        return p
    if isinstance(p, list) and p and isinstance(p[0], str):
        return p
    raise RequestError("prompt must be a string, a list of strings or token ids")


def _completion_logprobs(ctx: ServingContext, token_ids: List[int], lps, offset0: int,
                         nlog: int) -> CompletionLogprobs:
    out = CompletionLogprobs()
    off = offset0
    for tid, lp in zip(token_ids, lps or []):
        s = ctx._tok_str(tid)
        out.tokens.append(s)
        out.token_logprobs.append(None if lp is None else lp.get(tid))
        out.text_offset.append(off)
        off += len(s)
        if lp is None or nlog == 0:
            out.top_logprobs.append(None)
        else:
            top = sorted(lp.items(), key=lambda kv: -kv[1])[:nlog]
            out.top_logprobs.append({ctx._tok_str(k): v for k, v in top})
    return out


async def create_completion(req: CompletionRequest, ctx: ServingContext):
    ctx.check_model(req.model)
    if req.suffix:
        raise RequestError("suffix is not supported")
    prompts = _prompts(req)
    rid = random_id("cmpl")
    created = int(time.time())
    enc = [ctx.tokenize_prompt(p, req.add_special_tokens is not False, req.truncate_prompt_tokens)
           for p in prompts]
    params = [req.to_sampling_params(ctx.default_max_tokens(len(ids)), req.logprobs,
                                     ctx.generation_defaults) for _, ids in enc]
    gens = [_start(ctx.engine, f"{rid}-{i}", text, params[i], prompt_token_ids=ids,
                   priority=req.priority)
            for i, (text, ids) in enumerate(enc)]
    n = params[0].n

    if not req.stream:
        finals = {}
        async for i, out in _merge(gens):
            if out.finished:
                finals[i] = out
        choices, ptok, ctok = [], 0, 0
        for i, (text, ids) in enumerate(enc):
            out = finals[i]
            ptok += len(ids)
            for c in out.outputs:
                ctok += len(c.token_ids)
                body = c.text
                prefix = ""
                if req.echo:
                    prefix = text if text is not None else ctx.tokenizer.decode(ids)
                lp = None
                if req.logprobs is not None and c.logprobs is not None:
                    lp = _completion_logprobs(ctx, c.token_ids, c.logprobs, len(prefix), req.logprobs)
                choices.append(CompletionResponseChoice(index=i * n + c.index, text=prefix + body,
                                                        logprobs=lp, finish_reason=c.finish_reason,
                                                        stop_reason=c.stop_reason))
        return CompletionResponse(id=rid, created=created, model=ctx.model, choices=choices,
                                  usage=UsageInfo(prompt_tokens=ptok, completion_tokens=ctok,
                                                  total_tokens=ptok + ctok))

    include_usage = bool(req.stream_options and req.stream_options.include_usage)
    continuous = bool(req.stream_options and req.stream_options.continuous_usage_stats)

    fast = req.logprobs is None and not req.echo and not continuous

    async def stream() -> AsyncIterator[str]:
        ptok = sum(len(ids) for _, ids in enc)
        ctok = 0
        echoed = set()
        offsets: Dict[int, int] = {}
        head = completion_chunk_head(rid, created, ctx.model)
        try:
            async for i, out in _merge(gens):
                for c in out.outputs:
                    idx = i * n + c.index
                    text = c.new_text
                    if fast:
                        ctok += len(c.new_token_ids)
                        if text or c.finish_reason or c.new_token_ids:
                            yield fast_completion_chunk(head, idx, text, c.finish_reason,
                                                        c.stop_reason)
                        continue
                    if req.echo and idx not in echoed:
                        echoed.add(idx)
                        pt, pids = enc[i]
                        text = (pt if pt is not None else ctx.tokenizer.decode(pids)) + text
                    ctok += len(c.new_token_ids)
                    if not text and not c.finish_reason and not c.new_token_ids:
                        continue
                    lp = None
                    if req.logprobs is not None and c.new_logprobs:
                        lp = _completion_logprobs(ctx, c.new_token_ids, c.new_logprobs,
                                                  offsets.get(idx, 0), req.logprobs)
                    offsets[idx] = offsets.get(idx, 0) + len(text)
                    chunk = CompletionStreamResponse(
                        id=rid, created=created, model=ctx.model,
                        choices=[CompletionStreamChoice(index=idx, text=text, logprobs=lp,
                                                        finish_reason=c.finish_reason,
                                                        stop_reason=c.stop_reason)])
                    if continuous:
                        chunk.usage = UsageInfo(prompt_tokens=ptok, completion_tokens=ctok,
                                                total_tokens=ptok + ctok)
                    yield _sse(chunk)
            if include_usage:
                yield _sse(CompletionStreamResponse(
                    id=rid, created=created, model=ctx.model, choices=[],
                    usage=UsageInfo(prompt_tokens=ptok, completion_tokens=ctok,
                                    total_tokens=ptok + ctok)))
        except Exception as e:   # noqa: BLE001 - report inside the stream
            yield _sse(json.dumps({"error": {"message": str(e), "type": "InternalServerError",
                                             "code": 500}}))
        yield "data: [DONE]\n\n"

    return stream()


# ----------------------------------------------------------------------------- chat

def _chat_logprobs(ctx: ServingContext, token_ids, lps, top_n: int) -> ChatLogprobs:
    content = []
    for tid, lp in zip(token_ids, lps or []):
        if lp is None:
            continue
        top = sorted(lp.items(), key=lambda kv: -kv[1])[:top_n] if top_n else []
        s = ctx._tok_str(tid)
        content.append(ChatLogprobContent(
            token=s, logprob=lp.get(tid, float("-inf")), bytes=list(s.encode()),
            top_logprobs=[Logprob(token=ctx._tok_str(k), logprob=v,
                                  bytes=list(ctx._tok_str(k).encode())) for k, v in top]))
    return ChatLogprobs(content=content)


def _tools_for_request(req: ChatCompletionRequest, ctx: ServingContext):
    """(tools passed to the template, parse tool calls?, forced function name)."""
    tools = req.tools
    if not tools or req.tool_choice == "none":
        return (tools if req.tool_choice == "none" else None), False, None
    if isinstance(req.tool_choice, dict):
        name = req.tool_choice.get("function", {}).get("name")
        if not any(t.function.name == name for t in tools):
            raise RequestError(f"tool_choice names unknown function {name!r}")
        return tools, False, name
    if not ctx.tool_parser:
        raise RequestError('"auto" tool choice requires --enable-auto-tool-choice and '
                           '--tool-call-parser to be set')
    if req.tool_choice == "auto" and not ctx.enable_auto_tool_choice:
        raise RequestError('"auto" tool choice requires --enable-auto-tool-choice and '
                           '--tool-call-parser to be set')
    return tools, True, None


def _vision_config(ctx) -> Optional[Dict]:
    cfg = getattr(ctx.engine, "cfg", None) or getattr(getattr(ctx.engine, "engine", None),
                                                       "cfg", None)
    return None if cfg is None else cfg.model.extra.get("vision_config")


def _special_id(tok, name: str) -> Optional[int]:
    try:
        i = tok.convert_tokens_to_ids(name)
    except Exception:   # noqa: BLE001 - tokenizers without that vocabulary entry
        return None
    return i if isinstance(i, int) and i != getattr(tok, "unk_token_id", None) else None


def _expand_images(ctx, prompt: str, images: List[str], add_special: bool):
    """Chat prompt with image markers -> (text, token ids, multi_modal_data).  Every marker
    becomes the Llama-4 image block for that image's tile grid (<|image_start|>, per-tile patch
    runs with tile separators, the global tile, <|image_end|>); the patch token is the model's
    image_token_id, so the ids are built here rather than by re-tokenising the expanded text.
    The image bytes travel to the engine, which runs the vision tower at admission."""
    from ...models.llama4_vision import expand_image_prompt, load_image, preprocess
    from .chat_utils import IMAGE_MARK
    vc = _vision_config(ctx)
    if vc is None:
        raise RequestError(f"model `{ctx.model}` does not accept image inputs")
    cfg = getattr(ctx.engine, "cfg", None) or ctx.engine.engine.cfg
    patch_id = int(cfg.model.extra["image_token_id"])
    tile = vc.get("image_size", 336)
    per_tile = int((tile // vc.get("patch_size", 14)) ** 2 * vc.get("pixel_shuffle_ratio", 0.5) ** 2)
    tok = ctx.tokenizer
    sp = {n: _special_id(tok, f"<|{n}|>") for n in ("image_start", "image_end", "image",
                                                    "tile_x_separator", "tile_y_separator")}

    def block(th: int, tw: int) -> List[int]:
        out = [sp["image_start"]]
        if th * tw > 1:
            for _ in range(th):
                for x in range(tw):
                    out += [patch_id] * per_tile
                    if x < tw - 1:
                        out.append(sp["tile_x_separator"])
                out.append(sp["tile_y_separator"])
        out += [sp["image"]] + [patch_id] * per_tile + [sp["image_end"]]
        return [i for i in out if i is not None]

    segs = prompt.split(IMAGE_MARK)
    if len(segs) != len(images) + 1:
        raise RequestError("image marker mismatch in the rendered chat prompt")
    ids = tok.encode(segs[0], add_special_tokens=add_special) if segs[0] or add_special else []
    text, blobs = segs[0], []
    for src, seg in zip(images, segs[1:]):
        if not isinstance(src, str) or not src.startswith(("data:", "http://", "https://")):
            raise RequestError("image_url must be a data: URL or an http(s) URL")
        try:
            img = load_image(src)
            buf = __import__("io").BytesIO()
            img.save(buf, format="PNG")
            data = buf.getvalue()
            _, (th, tw) = preprocess(data, tile=tile)
        except Exception as e:   # noqa: BLE001 - unreadable image: client error
            raise RequestError(f"could not load image: {e}") from e
        ids += block(th, tw)
        if seg:
            ids += tok.encode(seg, add_special_tokens=False)
        text += expand_image_prompt((th, tw), per_tile) + seg
        blobs.append(data)
    return text, ids, {"image": blobs}


async def create_chat_completion(req: ChatCompletionRequest, ctx: ServingContext):
    ctx.check_model(req.model)
    tools, parse_tools, forced = _tools_for_request(req, ctx)
    template = None
    if req.chat_template:
        from .chat_utils import resolve_chat_template
        template = resolve_chat_template(req.chat_template)
    elif ctx.chat_template:
        template = ctx.chat_template
    from .chat_utils import extract_images
    messages, images = extract_images(req.messages)
    try:
        prompt = apply_chat_template(ctx.tokenizer, messages, template, tools,
                                     req.add_generation_prompt, req.continue_final_message,
                                     req.documents, **(req.chat_template_kwargs or {}))
    except RequestError:
        raise
    except Exception as e:   # noqa: BLE001 - template errors are client errors
        raise RequestError(f"chat template error: {e}") from e
    mm = None
    add_special = req.add_special_tokens if req.add_special_tokens is not None else False
    if images:
        if req.truncate_prompt_tokens:
            raise RequestError("truncate_prompt_tokens cannot be combined with image inputs")
        # download / decode / tile on a worker thread: a slow image URL must not stall the
        # event loop that feeds every other SSE stream and /health
        import asyncio
        text, ids, mm = await asyncio.to_thread(_expand_images, ctx, prompt, images, add_special)
        _, ids = ctx.tokenize_prompt(ids)
    else:
        text, ids = ctx.tokenize_prompt(prompt, add_special, req.truncate_prompt_tokens)
    top_n = (req.top_logprobs or 0) if req.logprobs else None
    max_tokens = req.max_completion_tokens or req.max_tokens
    if max_tokens is not None:
        req.max_tokens = max_tokens
    params = req.to_sampling_params(ctx.default_max_tokens(len(ids)), top_n,
                                    ctx.generation_defaults)
    if forced is not None:
        fn = next(t.function for t in tools if t.function.name == forced)
        params.guided_json = fn.parameters or {}
    rid = random_id("chatcmpl")
    created = int(time.time())
    gen = _start(ctx.engine, rid, text, params, prompt_token_ids=ids, priority=req.priority,
                 **({"multi_modal_data": mm} if mm else {}))
    n = params.n

    if not req.stream:
        final = None
        async for out in gen:
            if out.finished:
                final = out
        choices, ctok = [], 0
        for c in final.outputs:
            ctok += len(c.token_ids)
            msg = ChatMessage(role="assistant", content=c.text)
            finish = c.finish_reason
            if forced is not None:
                from .protocol import FunctionCall, ToolCall
                msg = ChatMessage(role="assistant", content="", tool_calls=[
                    ToolCall(function=FunctionCall(name=forced, arguments=c.text))])
                finish = "tool_calls" if finish == "stop" else finish
            elif parse_tools:
                content, calls = get_parser(ctx.tool_parser)(c.text)
                if calls:
                    msg = ChatMessage(role="assistant", content=content, tool_calls=calls)
                    finish = "tool_calls" if finish == "stop" else finish
            lp = _chat_logprobs(ctx, c.token_ids, c.logprobs, top_n or 0) \
                if top_n is not None and c.logprobs else None
            choices.append(ChatCompletionResponseChoice(index=c.index, message=msg, logprobs=lp,
                                                        finish_reason=finish,
                                                        stop_reason=c.stop_reason))
        return ChatCompletionResponse(id=rid, created=created, model=ctx.model, choices=choices,
                                      usage=UsageInfo(prompt_tokens=len(ids),
                                                      completion_tokens=ctok,
                                                      total_tokens=len(ids) + ctok))

    include_usage = bool(req.stream_options and req.stream_options.include_usage)
    continuous = bool(req.stream_options and req.stream_options.continuous_usage_stats)

    fast = not parse_tools and forced is None and top_n is None and not continuous

    async def stream() -> AsyncIterator[str]:
        ctok = 0
        states = {i: StreamingToolState(ctx.tool_parser) for i in range(n)} if parse_tools else {}
        started = set()
        head = chat_chunk_head(rid, created, ctx.model)
        try:
            for i in range(n):
                yield _sse(ChatCompletionStreamResponse(
                    id=rid, created=created, model=ctx.model,
                    choices=[ChatCompletionResponseStreamChoice(
                        index=i, delta=DeltaMessage(role="assistant", content=""))]))
            async for out in gen:
                for c in out.outputs:
                    ctok += len(c.new_token_ids)
                    delta_text = c.new_text
                    finish = c.finish_reason
                    if fast:
                        if delta_text or finish:
                            yield fast_chat_chunk(head, c.index, delta_text, finish,
                                                  c.stop_reason)
                        continue
                    tool_deltas = []
                    if forced is not None:
                        if delta_text:
                            first = c.index not in started
                            started.add(c.index)
                            tool_deltas = [DeltaToolCall(
                                index=0, id=random_id("chatcmpl-tool") if first else None,
                                type="function" if first else None,
                                function=DeltaFunctionCall(name=forced if first else None,
                                                           arguments=delta_text))]
                        delta_text = ""
                        if finish == "stop":
                            finish = "tool_calls"
                    elif parse_tools:
                        st = states[c.index]
                        delta_text = st.feed(delta_text)
                        if finish:
                            rest, calls = st.finish()
                            delta_text += rest
                            tool_deltas = [DeltaToolCall(index=j, id=tc.id, type="function",
                                                         function=DeltaFunctionCall(
                                                             name=tc.function.name,
                                                             arguments=tc.function.arguments))
                                           for j, tc in enumerate(calls)]
                            if calls and finish == "stop":
                                finish = "tool_calls"
                    if not delta_text and not tool_deltas and not finish:
                        continue
                    lp = _chat_logprobs(ctx, c.new_token_ids, c.new_logprobs, top_n or 0) \
                        if top_n is not None and c.new_logprobs else None
                    chunk = ChatCompletionStreamResponse(
                        id=rid, created=created, model=ctx.model,
                        choices=[ChatCompletionResponseStreamChoice(
                            index=c.index, delta=DeltaMessage(content=delta_text or None,
                                                              tool_calls=tool_deltas),
                            logprobs=lp, finish_reason=finish, stop_reason=c.stop_reason)])
                    if continuous:
                        chunk.usage = UsageInfo(prompt_tokens=len(ids), completion_tokens=ctok,
                                                total_tokens=len(ids) + ctok)
                    yield _sse(chunk)
            if include_usage:
                yield _sse(ChatCompletionStreamResponse(
                    id=rid, created=created, model=ctx.model, choices=[],
                    usage=UsageInfo(prompt_tokens=len(ids), completion_tokens=ctok,
                                    total_tokens=len(ids) + ctok)))
        except Exception as e:   # noqa: BLE001
            yield _sse(json.dumps({"error": {"message": str(e), "type": "InternalServerError",
                                             "code": 500}}))
        yield "data: [DONE]\n\n"

    return stream()
