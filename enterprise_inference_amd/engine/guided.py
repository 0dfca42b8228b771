"""Guided decoding: ``guided_choice`` / ``guided_regex`` / ``guided_json`` request fields
(docs/api-spec.yaml:479 onward; vLLM extras the reference exposes through its
OpenAI surface) and chat ``response_format``.

Each sequence carries a ``GuidedState`` that yields the allowed next tokens as a device
bool mask (K13: applied with one masked_fill before the sampler kernel,
engine/logits_process.py):

* choice  -> token trie over the tokenised choices (exact, O(#choices));
* regex   -> token-level FSM (engine/fsm.py): the pattern is compiled once into an NFA,
  determinised lazily, and each DFA state's allowed-token set / mask is computed once per
  process by walking the vocabulary trie -- shared by every request with the same pattern;
* json    -> a JSON-schema subset compiled to a regex (objects with typed properties,
  enums, arrays, nested objects), then as regex; free-form objects (``{}``, json_object mode)
  and ``$ref`` schemas (recursive definitions) compile to a grammar instead
  (``schema_to_grammar``) and run on the pushdown matcher at any nesting depth;
* grammar -> GBNF / Lark EBNF (``guided_grammar``): a regular grammar compiles to a regex
  (engine/fsm.py grammar_to_regex) and runs as regex; a recursive one runs on the native
  pushdown matcher (engine/grammar.py, csrc/runtime/grammar.cpp).
"""

from __future__ import annotations

import json
from typing import Dict, List, Optional

try:
    import regex as _re
except ImportError:  # pragma: no cover - regex ships in the image
    import re as _re

# Whitespace between JSON tokens is capped: with an unbounded run a weakly-conditioned model
# can spend its whole max_tokens budget on indentation and never close the document.
_WS = r"[ \t\n]{0,2}"
_STR = r'"(?:[^"\\\x00-\x1f]|\\["\\/bfnrt]|\\u[0-9a-fA-F]{4})*"'
_NUM = r"-?(?:0|[1-9][0-9]*)(?:\.[0-9]+)?(?:[eE][+-]?[0-9]+)?"
_INT = r"-?(?:0|[1-9][0-9]*)"
_BOOL = r"(?:true|false)"
_NULL = r"null"
_SCALAR = f"(?:{_STR}|{_NUM}|{_BOOL}|{_NULL})"


def schema_to_regex(schema, depth: int = 0) -> str:
    """Compile a JSON-schema subset into a regex matching its JSON serialisations."""
    if schema is None or schema == {} or schema is True:
        if depth > 2:
            return _SCALAR
        val = f"(?:{_SCALAR}|{schema_to_regex({'type': 'array'}, depth + 1)})"
        pair = f"{_STR}{_WS}:{_WS}{val}"
        return r"\{" + _WS + f"(?:{pair}(?:{_WS},{_WS}{pair})*)?" + _WS + r"\}"
    if isinstance(schema, str):
        schema = json.loads(schema)
    if "enum" in schema:
        return "(?:" + "|".join(_re.escape(json.dumps(v)) for v in schema["enum"]) + ")"
    if "const" in schema:
        return _re.escape(json.dumps(schema["const"]))
    for key in ("anyOf", "oneOf"):
        if key in schema:
            return "(?:" + "|".join(schema_to_regex(s, depth + 1) for s in schema[key]) + ")"
    t = schema.get("type")
    if isinstance(t, list):
        return "(?:" + "|".join(schema_to_regex({**schema, "type": x}, depth) for x in t) + ")"
    if t == "string":
        if "pattern" in schema:
            return '"' + schema["pattern"].lstrip("^").rstrip("$") + '"'
        return _STR
    if t == "number":
        return _NUM
    if t == "integer":
        return _INT
    if t == "boolean":
        return _BOOL
    if t == "null":
        return _NULL
    if t == "array":
        item = schema_to_regex(schema.get("items", {"type": "string"}), depth + 1) \
            if depth < 4 else _SCALAR
        return r"\[" + _WS + f"(?:{item}(?:{_WS},{_WS}{item})*)?" + _WS + r"\]"
    if t == "object" or "properties" in schema:
        props: Dict = schema.get("properties", {})
        if not props:
            return schema_to_regex({}, depth + 1)
        required = set(schema.get("required", list(props)))
        parts = []
        for i, (name, sub) in enumerate(props.items()):
            kv = _re.escape(json.dumps(name)) + _WS + ":" + _WS + schema_to_regex(sub, depth + 1)
            sep = "" if i == 0 else f"{_WS},{_WS}"
            parts.append(f"{sep}{kv}" if name in required else f"(?:{sep}{kv})?")
        return r"\{" + _WS + "".join(parts) + _WS + r"\}"
    return _SCALAR


_G_COMMON = r"""
ws ::= [ \t\n]? [ \t\n]?
string ::= /"(?:[^"\\\x00-\x1f]|\\["\\bfnrt\x2f]|\\u[0-9a-fA-F]{4})*"/
number ::= /-?(?:0|[1-9][0-9]*)(?:\.[0-9]+)?(?:[eE][+-]?[0-9]+)?/
integer ::= /-?(?:0|[1-9][0-9]*)/
boolean ::= "true" | "false"
null ::= "null"
value ::= object | array | string | number | boolean | null
object ::= "{" ws (string ws ":" ws value (ws "," ws string ws ":" ws value)*)? ws "}"
array ::= "[" ws (value (ws "," ws value)*)? ws "]"
"""


def _walk_schema(schema):
    if isinstance(schema, dict):
        yield schema
        for v in schema.values():
            yield from _walk_schema(v)
    elif isinstance(schema, list):
        for v in schema:
            yield from _walk_schema(v)


def schema_needs_grammar(schema) -> bool:
    """A schema the bounded regex cannot express: ``$ref`` (possibly recursive definitions)
    or a free-form object / value (any nesting depth)."""
    if isinstance(schema, str):
        schema = json.loads(schema)
    if schema is None or schema is True or schema == {}:
        return True
    for d in _walk_schema(schema):
        if "$ref" in d:
            return True
        if d.get("type") == "object" and not d.get("properties"):
            return True
    return False


def schema_to_grammar(schema) -> str:
    """JSON schema -> GBNF over the JSON token rules above; ``$ref`` to ``#/$defs/X`` /
    ``#/definitions/X`` becomes a rule reference, so recursive schemas stay exact.  Property
    order / required / enum / const / anyOf / type-list semantics match ``schema_to_regex``."""
    if isinstance(schema, str):
        schema = json.loads(schema)
    root = schema if isinstance(schema, dict) else {}
    defs = {**root.get("definitions", {}), **root.get("$defs", {})}
    rules: List[str] = []
    named: Dict[str, str] = {}

    def lit(v) -> str:
        return json.dumps(json.dumps(v, ensure_ascii=False), ensure_ascii=False)

    def ref(path: str) -> str:
        name = path.rsplit("/", 1)[-1]
        if path in ("#", "#/"):
            key, sub = "root_schema", root
        elif name in defs:
            key, sub = "def_" + "".join(c if c.isalnum() else "_" for c in name), defs[name]
        else:
            raise ValueError(f"guided_json: unresolvable $ref {path!r}")
        if key not in named:
            named[key] = ""                        # reserve before recursing
            named[key] = emit(sub)
            rules.append(f"{key} ::= {named[key]}")
        return key

    def emit(sc) -> str:
        if sc is None or sc is True or sc == {}:
            return "value"
        if "$ref" in sc:
            return ref(sc["$ref"])
        if "enum" in sc:
            return "(" + " | ".join(lit(v) for v in sc["enum"]) + ")"
        if "const" in sc:
            return lit(sc["const"])
        for key in ("anyOf", "oneOf"):
            if key in sc:
                return "(" + " | ".join(emit(x) for x in sc[key]) + ")"
        t = sc.get("type")
        if isinstance(t, list):
            return "(" + " | ".join(emit({**sc, "type": x}) for x in t) + ")"
        if t == "string":
            if "pattern" in sc:
                pat = sc["pattern"].lstrip("^").rstrip("$").replace("/", "\\x2f")
                return '"\\"" /' + pat + '/ "\\""'
            return "string"
        if t in ("number", "integer", "boolean", "null"):
            return t
        if t == "array":
            item = emit(sc.get("items", {}))
            return f'"[" ws ({item} (ws "," ws {item})*)? ws "]"'
        if t == "object" or "properties" in sc:
            props = sc.get("properties", {})
            if not props:
                return "object"
            required = set(sc.get("required", list(props)))
            parts = []
            for i, (name, sub) in enumerate(props.items()):
                kv = f'{lit(name)} ws ":" ws {emit(sub)}'
                sep = "" if i == 0 else 'ws "," ws '
                parts.append(f"{sep}{kv}" if name in required else f"({sep}{kv})?")
            return '"{" ws ' + " ".join(parts) + ' ws "}"'
        return "value"

    body = emit(schema)
    return "\n".join([f"root ::= {body}"] + rules) + _G_COMMON


class GuidedState:
    def allowed_tokens(self) -> Optional[List[int]]:
        raise NotImplementedError

    def allowed_mask(self, device, vocab: int):
        """bool [vocab] on `device` (True = allowed)."""
        import torch

        m = torch.zeros(vocab, dtype=torch.bool)
        ids = [t for t in (self.allowed_tokens() or []) if 0 <= t < vocab]
        if ids:
            m[torch.tensor(ids, dtype=torch.long)] = True
        return m.to(device)

    def advance(self, token: int) -> None:
        raise NotImplementedError

    def is_done(self) -> bool:
        return False


class ChoiceState(GuidedState):
    def __init__(self, choices: List[str], tokenizer, eos_ids: List[int]):
        self.seqs = [tokenizer.encode(c, add_special_tokens=False) for c in choices]
        self.pos = 0
        self.alive = list(range(len(self.seqs)))
        self.eos = list(eos_ids)
        self.done = False

    def allowed_tokens(self):
        nxt = {self.seqs[i][self.pos] for i in self.alive if self.pos < len(self.seqs[i])}
        if any(self.pos == len(self.seqs[i]) for i in self.alive):
            nxt.update(self.eos)
        return sorted(nxt) if nxt else list(self.eos)

    def advance(self, token):
        self.alive = [i for i in self.alive
                      if self.pos < len(self.seqs[i]) and self.seqs[i][self.pos] == token]
        self.pos += 1
        if any(self.pos == len(self.seqs[i]) for i in self.alive) and \
                all(self.pos >= len(self.seqs[i]) for i in self.alive):
            self.done = True

    def is_done(self):
        return self.done or not self.alive


class RegexState(GuidedState):
    """Token-level constrained decoding on a cached token FSM (engine/fsm.py)."""

    def __init__(self, pattern: str, tokenizer, vocab_size: int, eos_ids: List[int]):
        from .fsm import token_fsm

        self.fsm = token_fsm(pattern, tokenizer, vocab_size, eos_ids)
        self.eos = set(self.fsm.eos)
        self.sid = self.fsm.start
        self.done = False

    def allowed_tokens(self):
        return self.fsm.allowed_ids(self.sid).tolist()

    def allowed_mask(self, device, vocab: int):
        return self.fsm.mask(self.sid, device, vocab)

    def advance(self, token):
        if token in self.eos:
            self.done = True
            return
        n = self.fsm.next_state(self.sid, token)
        if n < 0:                  # not allowed (e.g. sampled from an unmasked fallback row)
            self.done = True
            return
        self.sid = n
        # complete and cannot be extended: stop
        if self.fsm.char.accepting(n) and not self.fsm.can_continue(n):
            self.done = True

    def is_done(self):
        return self.done


def make_guided_state(params, tokenizer, vocab_size: int) -> GuidedState:
    eos = list(getattr(params, "eos_ids", None) or [getattr(tokenizer, "eos_token_id", 2)])
    if params.guided_choice:
        return ChoiceState(list(params.guided_choice), tokenizer, eos)
    if params.guided_regex:
        return RegexState(params.guided_regex, tokenizer, vocab_size, eos)
    if getattr(params, "guided_grammar", None):
        from .fsm import grammar_to_regex
        from .grammar import GrammarState, is_recursive
        if is_recursive(params.guided_grammar):
            return GrammarState(params.guided_grammar, tokenizer, vocab_size, eos)
        return RegexState(grammar_to_regex(params.guided_grammar), tokenizer, vocab_size, eos)
    if schema_needs_grammar(params.guided_json):
        from .grammar import GrammarState
        return GrammarState(schema_to_grammar(params.guided_json), tokenizer, vocab_size, eos)
    return RegexState(schema_to_regex(params.guided_json), tokenizer, vocab_size, eos)
