"""Chat-template rendering (``--chat-template``).

Precedence: request ``chat_template`` > server ``--chat-template`` > the
tokenizer's own template > a built-in minimal template.  The reference points
``--chat-template`` at vLLM example files inside its image
(``/workspace/vllm/examples/tool_chat_template_*.jinja``,
core/helm-charts/vllm/gaudi-values.yaml:65,160,277,301); such paths resolve to
the equally named templates shipped in ``chat_templates/`` when absent.
"""

from __future__ import annotations

import functools
import json
import os
from typing import Tuple, Any, Dict, List, Optional

import jinja2
from jinja2.sandbox import ImmutableSandboxedEnvironment

TEMPLATE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "chat_templates")


def resolve_chat_template(value: Optional[str]) -> Optional[str]:
    """A template string, a path, or a reference-image path -> template text."""
    if not value:
        return None
    if os.path.exists(value):
        with open(value) as f:
            return f.read()
    shipped = os.path.join(TEMPLATE_DIR, os.path.basename(value))
    if value.endswith(".jinja") and os.path.exists(shipped):
        with open(shipped) as f:
            return f.read()
    if value.endswith(".jinja") and "/" in value and "{" not in value:
        raise ValueError(f"chat template file {value!r} not found")
    return value


@functools.lru_cache(maxsize=32)
def _compile(template: str) -> jinja2.Template:
    env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True,
                                        extensions=["jinja2.ext.loopcontrols"])
    env.filters["tojson"] = lambda v, indent=None: json.dumps(v, ensure_ascii=False, indent=indent)

    def raise_exception(msg):
        raise jinja2.TemplateError(msg)

    env.globals["raise_exception"] = raise_exception
    return env.from_string(template)


IMAGE_MARK = "\x00eia-image\x00"


def extract_images(messages: List[Any]) -> Tuple[List[Dict[str, Any]], List[str]]:
    """Replace image content parts (``image_url`` / ``image``) by a text marker, in order, and
    return the image sources (data: URL, http(s) URL or path)."""
    out, images = [], []
    for m in messages:
        m = dict(m) if isinstance(m, dict) else m.model_dump()
        c = m.get("content")
        if isinstance(c, list):
            parts = []
            for p in c:
                p = p if isinstance(p, dict) else p.model_dump()
                t = p.get("type", "text")
                if t in ("image_url", "image"):
                    iu = p.get("image_url") or p.get("image")
                    images.append(iu.get("url") if isinstance(iu, dict) else iu)
                    parts.append({"type": "text", "text": IMAGE_MARK})
                else:
                    parts.append(p)
            m["content"] = parts
        out.append(m)
    return out, images


def _normalise(messages: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    out = []
    for m in messages:
        m = dict(m)
        c = m.get("content")
        if isinstance(c, list):   # content parts: text (image parts became markers, extract_images)
            m["content"] = "".join(p.get("text", "") for p in c
                                   if isinstance(p, dict) and p.get("type", "text") == "text")
        if m.get("content") is None:
            m["content"] = ""
        tcs = m.get("tool_calls")
        if tcs:
            m["tool_calls"] = [t if isinstance(t, dict) else t.model_dump() for t in tcs]
        out.append(m)
    return out


def apply_chat_template(tokenizer, messages: List[Dict[str, Any]], template: Optional[str] = None,
                        tools: Optional[List[Dict[str, Any]]] = None,
                        add_generation_prompt: bool = True,
                        continue_final_message: bool = False,
                        documents=None, **kwargs) -> str:
    msgs = _normalise(messages)
    tools_d = [t if isinstance(t, dict) else t.model_dump() for t in (tools or [])] or None
    if template is None and getattr(tokenizer, "chat_template", None) and \
            hasattr(tokenizer, "apply_chat_template") and \
            tokenizer.__class__.__name__ != "ByteTokenizer":
        return tokenizer.apply_chat_template(msgs, tools=tools_d, documents=documents,
                                             add_generation_prompt=add_generation_prompt,
                                             continue_final_message=continue_final_message,
                                             tokenize=False, **kwargs)
    if template is None:
        template = getattr(tokenizer, "chat_template", None)
    if template is None:
        return tokenizer.apply_chat_template(msgs, tools=tools_d,
                                             add_generation_prompt=add_generation_prompt,
                                             tokenize=False)
    bos = getattr(tokenizer, "bos_token", None) or ""
    eos = getattr(tokenizer, "eos_token", None) or ""
    text = _compile(template).render(messages=msgs, tools=tools_d, documents=documents,
                                     add_generation_prompt=add_generation_prompt,
                                     bos_token=bos, eos_token=eos, **kwargs)
    if continue_final_message and msgs and msgs[-1]["role"] == "assistant":
        last = msgs[-1]["content"]
        idx = text.rfind(last)
        if idx >= 0:
            text = text[:idx + len(last)]
    return text
