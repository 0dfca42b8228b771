"""Tool-call parsers for ``--tool-call-parser``.

The reference enables four formats through its per-model ``extraCmdArgs``
(core/helm-charts/vllm/gaudi-values.yaml:65 hermes, :160 llama3_json,
:277 llama4_json, :301 mistral):

* ``llama3_json``  ``{"name": f, "parameters": {...}}`` (optionally after
  ``<|python_tag|>``, several calls separated by ``;``)
* ``llama4_json``  the same JSON objects, optionally inside
  ``<|python_start|> ... <|python_end|>``; a pythonic ``[f(a=1), g(b="x")]``
  list is also accepted
* ``hermes``       ``<tool_call>{"name": f, "arguments": {...}}</tool_call>`` blocks
* ``mistral``      ``[TOOL_CALLS] [{"name": f, "arguments": {...}}, ...]``

Each parser returns (remaining content, [ToolCall]).  Streaming uses
``StreamingToolState``: text is passed through until the output can no longer
be plain content, then buffered and emitted as tool-call deltas at the end.
"""

from __future__ import annotations

import ast
import json
from typing import Callable, Dict, List, Optional, Tuple

from .protocol import FunctionCall, ToolCall

ParseResult = Tuple[Optional[str], List[ToolCall]]


def _call(name: str, args) -> ToolCall:
    if not isinstance(args, str):
        args = json.dumps(args if args is not None else {}, ensure_ascii=False)
    return ToolCall(function=FunctionCall(name=name, arguments=args))


def _json_objects(text: str) -> List[Tuple[int, int, object]]:
    """All top-level JSON values (objects or arrays) embedded in text: (start, end, value)."""
    dec = json.JSONDecoder()
    out, i = [], 0
    while i < len(text):
        j = min([p for p in (text.find("{", i), text.find("[", i)) if p >= 0], default=-1)
        if j < 0:
            break
        try:
            val, end = dec.raw_decode(text, j)
            out.append((j, end, val))
            i = end
        except ValueError:
            i = j + 1
    return out


def _from_dict(d) -> Optional[ToolCall]:
    if not isinstance(d, dict) or "name" not in d:
        return None
    args = d.get("arguments", d.get("parameters", {}))
    return _call(str(d["name"]), args)


def parse_llama3_json(text: str) -> ParseResult:
    body = text.replace("<|python_tag|>", "").strip()
    if not body.startswith("{"):
        return text, []
    calls = []
    for _, _, v in _json_objects(body):
        c = _from_dict(v)
        if c is not None:
            calls.append(c)
    return (None, calls) if calls else (text, [])


def _parse_pythonic(body: str) -> List[ToolCall]:
    try:
        tree = ast.parse(body.strip(), mode="eval")
    except SyntaxError:
        return []
    node = tree.body
    items = node.elts if isinstance(node, ast.List) else [node]
    calls = []
    for it in items:
        if not isinstance(it, ast.Call) or not isinstance(it.func, ast.Name):
            return []
        try:
            kwargs = {k.arg: ast.literal_eval(k.value) for k in it.keywords}
        except ValueError:
            return []
        calls.append(_call(it.func.id, kwargs))
    return calls


def parse_llama4_json(text: str) -> ParseResult:
    body = text
    if "<|python_start|>" in body:
        body = body.split("<|python_start|>", 1)[1].split("<|python_end|>", 1)[0]
    stripped = body.strip()
    if stripped.startswith("[") and "(" in stripped:
        calls = _parse_pythonic(stripped)
        if calls:
            return None, calls
    content, calls = parse_llama3_json(stripped)
    return (None, calls) if calls else (text, [])


def parse_hermes(text: str) -> ParseResult:
    if "<tool_call>" not in text:
        return text, []
    calls, content_parts, rest = [], [], text
    while "<tool_call>" in rest:
        before, after = rest.split("<tool_call>", 1)
        content_parts.append(before)
        inner, _, rest = after.partition("</tool_call>")
        for _, _, v in _json_objects(inner):
            c = _from_dict(v)
            if c is not None:
                calls.append(c)
    content_parts.append(rest)
    content = "".join(content_parts).strip()
    return (content or None), calls


def parse_mistral(text: str) -> ParseResult:
    if "[TOOL_CALLS]" not in text:
        return text, []
    before, after = text.split("[TOOL_CALLS]", 1)
    calls = []
    for _, _, v in _json_objects(after):
        for d in (v if isinstance(v, list) else [v]):
            c = _from_dict(d)
            if c is not None:
                calls.append(c)
    content = before.strip()
    return (content or None), calls


PARSERS: Dict[str, Callable[[str], ParseResult]] = {
    "llama3_json": parse_llama3_json,
    "llama4_json": parse_llama4_json,
    "llama4_pythonic": parse_llama4_json,
    "pythonic": parse_llama4_json,
    "hermes": parse_hermes,
    "mistral": parse_mistral,
}

# prefixes after which an output can no longer be plain content (streaming hold-back)
_STARTS = {
    "llama3_json": ("{", "<|python_tag|>"),
    "llama4_json": ("{", "[", "<|python_start|>"),
    "llama4_pythonic": ("[", "<|python_start|>"),
    "pythonic": ("[",),
    "hermes": ("<tool_call>",),
    "mistral": ("[TOOL_CALLS]",),
}


def get_parser(name: str) -> Callable[[str], ParseResult]:
    if name not in PARSERS:
        raise ValueError(f"unknown --tool-call-parser {name!r}; choose from {sorted(PARSERS)}")
    return PARSERS[name]


class StreamingToolState:
    """Per-choice streaming state: decide whether the output is content or a tool call."""

    def __init__(self, name: str):
        self.name = name
        self.parse = get_parser(name)
        self.starts = _STARTS[name]
        self.text = ""
        self.mode: Optional[str] = None   # None (undecided) | "content" | "tool"
        self.emitted = 0

    def feed(self, delta: str) -> str:
        """Returns the content delta that may be streamed now."""
        self.text += delta
        if self.mode == "content":
            return delta
        if self.mode == "tool":
            return ""
        s = self.text.lstrip()
        if not s:
            return ""
        if any(s.startswith(p) or p.startswith(s) for p in self.starts):
            if any(s.startswith(p) for p in self.starts):
                self.mode = "tool"
            return ""
        if self.name in ("hermes", "mistral"):
            # markers may also appear after some content: stream up to a partial marker
            marker = self.starts[0]
            cut = self.text.find(marker)
            if cut >= 0:
                self.mode = "tool"
                out = self.text[self.emitted:cut]
                self.emitted = cut
                return out
            hold = max((k for k in range(1, len(marker)) if self.text.endswith(marker[:k])),
                       default=0)
            out = self.text[self.emitted:len(self.text) - hold]
            self.emitted = len(self.text) - hold
            return out
        self.mode = "content"
        return self.text

    def finish(self) -> Tuple[str, List[ToolCall]]:
        """At end of stream: (unsent content, tool calls)."""
        if self.mode == "content":
            return "", []
        content, calls = self.parse(self.text)
        if not calls:
            return self.text[self.emitted:], []
        rest = "" if content is None else content[self.emitted:] if self.mode != "tool" else ""
        return rest, calls
