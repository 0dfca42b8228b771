"""Regex / grammar -> token-level finite-state machine for guided decoding (K13).

The per-step cost of the previous guided decoder was one partial regex match per vocabulary
entry (128k Python regex calls per generated token).  Here a pattern is compiled ONCE into a
character NFA (Thompson construction over a regex subset that covers the JSON-schema
compiler's output and ordinary ``guided_regex`` patterns), determinised lazily, and the
allowed-token set of a DFA state is found by walking a trie of the vocabulary's token strings
with the state (shared prefixes are stepped once; dead branches are pruned).  Each
(pattern, DFA state) is computed once per process and shared by every request using the same
pattern; its mask lives on the device as a bool row, so masking a guided row is one
``masked_fill_`` with no host->device copy after warm-up.

``grammar_to_regex`` accepts the regular (non-recursive) subset of GBNF / Lark-style EBNF
grammars (``guided_grammar``): rules of literals, character classes, /regex/ terminals, rule
references, grouping, alternation and ``* + ?``; recursive grammars (nested JSON, expression
languages) are context-free and run on the pushdown matcher of engine/grammar.py instead.
"""

from __future__ import annotations

import re as _stdre
import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import numpy as np

_MAX_NFA = 250_000


# ----------------------------------------------------------------------------- regex parser
class CharSet:
    __slots__ = ("ranges", "neg")

    def __init__(self, ranges, neg: bool = False):
        self.ranges = tuple(ranges)
        self.neg = neg

    def match(self, c: int) -> bool:
        for lo, hi in self.ranges:
            if lo <= c <= hi:
                return not self.neg
        return self.neg


_DIGIT = [(48, 57)]
_WORD = [(48, 57), (65, 90), (95, 95), (97, 122)]
_SPACE = [(9, 13), (32, 32)]
_SIMPLE_ESC = {"n": 10, "t": 9, "r": 13, "f": 12, "v": 11, "0": 0}


class _Parser:
    def __init__(self, pattern: str):
        self.p = pattern
        self.i = 0

    def peek(self) -> Optional[str]:
        return self.p[self.i] if self.i < len(self.p) else None

    def take(self) -> str:
        c = self.p[self.i]
        self.i += 1
        return c

    def parse(self):
        if self.peek() == "^":
            self.i += 1
        node = self.alt()
        if self.peek() == "$":
            self.i += 1
        if self.i != len(self.p):
            raise ValueError(f"unsupported regex syntax at {self.i}: {self.p[self.i:self.i + 10]!r}")
        return node

    def alt(self):
        parts = [self.concat()]
        while self.peek() == "|":
            self.i += 1
            parts.append(self.concat())
        return parts[0] if len(parts) == 1 else ("alt", parts)

    def concat(self):
        items = []
        while self.peek() is not None and self.peek() not in "|)":
            if self.peek() == "$" and self.i == len(self.p) - 1:
                break
            items.append(self.repeat())
        return ("cat", items)

    def repeat(self):
        node = self.atom()
        while True:
            c = self.peek()
            if c == "*":
                self.i += 1
                node = ("rep", node, 0, None)
            elif c == "+":
                self.i += 1
                node = ("rep", node, 1, None)
            elif c == "?":
                self.i += 1
                node = ("rep", node, 0, 1)
            elif c == "{" and _stdre.match(r"\{\d*(,\d*)?\}", self.p[self.i:]):
                m = _stdre.match(r"\{(\d*)(,?)(\d*)\}", self.p[self.i:])
                self.i += m.end()
                lo = int(m.group(1) or 0)
                hi = lo if not m.group(2) else (int(m.group(3)) if m.group(3) else None)
                node = ("rep", node, lo, hi)
            else:
                return node
            if self.peek() in ("?", "+") and node[0] == "rep":
                self.i += 1                       # lazy / possessive suffix: same language

    def atom(self):
        c = self.take()
        if c == "(":
            if self.p.startswith("?:", self.i):
                self.i += 2
            elif self.p.startswith("?P<", self.i) or self.p.startswith("?<", self.i):
                self.i = self.p.index(">", self.i) + 1
            elif self.peek() == "?":
                raise ValueError("unsupported group construct (lookaround / flags)")
            node = self.alt()
            if self.peek() != ")":
                raise ValueError("unbalanced parenthesis")
            self.i += 1
            return node
        if c == "[":
            return ("lit", self.charclass())
        if c == ".":
            return ("lit", CharSet([(10, 10)], neg=True))
        if c == "\\":
            return ("lit", self.escape(in_class=False))
        return ("lit", CharSet([(ord(c), ord(c))]))

    def escape(self, in_class: bool) -> CharSet:
        c = self.take()
        if c == "d":
            return CharSet(_DIGIT)
        if c == "D":
            return CharSet(_DIGIT, neg=True)
        if c == "w":
            return CharSet(_WORD)
        if c == "W":
            return CharSet(_WORD, neg=True)
        if c == "s":
            return CharSet(_SPACE)
        if c == "S":
            return CharSet(_SPACE, neg=True)
        if c == "x":
            v = int(self.p[self.i:self.i + 2], 16)
            self.i += 2
            return CharSet([(v, v)])
        if c == "u":
            v = int(self.p[self.i:self.i + 4], 16)
            self.i += 4
            return CharSet([(v, v)])
        if c in _SIMPLE_ESC:
            v = _SIMPLE_ESC[c]
            return CharSet([(v, v)])
        return CharSet([(ord(c), ord(c))])

    def charclass(self) -> CharSet:
        neg = False
        if self.peek() == "^":
            neg = True
            self.i += 1
        ranges: List[Tuple[int, int]] = []
        first = True
        while True:
            c = self.peek()
            if c is None:
                raise ValueError("unterminated character class")
            if c == "]" and not first:
                self.i += 1
                break
            first = False
            if c == "\\":
                self.i += 1
                cs = self.escape(in_class=True)
                if cs.neg or len(cs.ranges) != 1 or cs.ranges[0][0] != cs.ranges[0][1]:
                    if cs.neg:
                        raise ValueError("negated class escape inside [...] is not supported")
                    ranges.extend(cs.ranges)
                    continue
                lo = cs.ranges[0][0]
            else:
                self.i += 1
                lo = ord(c)
            if self.peek() == "-" and self.i + 1 < len(self.p) and self.p[self.i + 1] != "]":
                self.i += 1
                d = self.take()
                hi = self.escape(in_class=True).ranges[0][0] if d == "\\" else ord(d)
                ranges.append((lo, hi))
            else:
                ranges.append((lo, lo))
        return CharSet(ranges, neg)


# ----------------------------------------------------------------------------- NFA / DFA
class CharFSM:
    """Thompson NFA of a pattern with a lazily built DFA over frozensets of NFA states."""

    def __init__(self, pattern: str):
        self.eps: List[List[int]] = []
        self.edges: List[List[Tuple[CharSet, int]]] = []
        start, self.accept = self._build(_Parser(pattern).parse())
        self.sets: List[frozenset] = []
        self.index: Dict[frozenset, int] = {}
        self.trans: Dict[Tuple[int, str], int] = {}
        self.start = self._intern(self._closure({start}))

    def _new(self) -> int:
        if len(self.eps) >= _MAX_NFA:
            raise ValueError("guided pattern too large (bounded repetition expands too far)")
        self.eps.append([])
        self.edges.append([])
        return len(self.eps) - 1

    def _build(self, node) -> Tuple[int, int]:
        kind = node[0]
        if kind == "lit":
            a, b = self._new(), self._new()
            self.edges[a].append((node[1], b))
            return a, b
        if kind == "cat":
            a = self._new()
            cur = a
            for it in node[1]:
                s, e = self._build(it)
                self.eps[cur].append(s)
                cur = e
            return a, cur
        if kind == "alt":
            a, b = self._new(), self._new()
            for it in node[1]:
                s, e = self._build(it)
                self.eps[a].append(s)
                self.eps[e].append(b)
            return a, b
        if kind == "rep":
            _, sub, lo, hi = node
            a = self._new()
            cur = a
            for _ in range(lo):
                s, e = self._build(sub)
                self.eps[cur].append(s)
                cur = e
            if hi is None:
                s, e = self._build(sub)
                b = self._new()
                self.eps[cur] += [s, b]
                self.eps[e] += [s, b]
                return a, b
            b = self._new()
            self.eps[cur].append(b)
            for _ in range(hi - lo):
                s, e = self._build(sub)
                self.eps[cur].append(s)
                self.eps[e].append(b)
                cur = e
            return a, b
        raise ValueError(kind)

    def _closure(self, states) -> frozenset:
        stack = list(states)
        seen = set(states)
        while stack:
            s = stack.pop()
            for t in self.eps[s]:
                if t not in seen:
                    seen.add(t)
                    stack.append(t)
        # keep only states that matter for the future: char-edge sources and the accept state
        return frozenset(s for s in seen if self.edges[s] or s == self.accept)

    def _intern(self, fs: frozenset) -> int:
        if not fs:
            return -1
        i = self.index.get(fs)
        if i is None:
            i = len(self.sets)
            self.sets.append(fs)
            self.index[fs] = i
        return i

    def step(self, sid: int, ch: str) -> int:
        key = (sid, ch)
        r = self.trans.get(key)
        if r is None:
            c = ord(ch)
            nxt = set()
            for s in self.sets[sid]:
                for cs, t in self.edges[s]:
                    if cs.match(c):
                        nxt.add(t)
            r = self._intern(self._closure(nxt)) if nxt else -1
            self.trans[key] = r
        return r

    def accepting(self, sid: int) -> bool:
        return sid >= 0 and self.accept in self.sets[sid]

    def walk(self, sid: int, text: str) -> int:
        for ch in text:
            sid = self.step(sid, ch)
            if sid < 0:
                return -1
        return sid


# ----------------------------------------------------------------------------- token level
class _Trie:
    __slots__ = ("kids", "toks")

    def __init__(self):
        self.kids: Dict[str, "_Trie"] = {}
        self.toks: List[int] = []


_TRIES: Dict[int, Tuple[object, _Trie, List[str]]] = {}
_lock = threading.Lock()


def vocab_strings(tokenizer, vocab_size: int) -> List[str]:
    n = min(vocab_size, len(tokenizer))
    out = []
    for i in range(n):
        try:
            out.append(tokenizer.decode([i], skip_special_tokens=True))
        except Exception:   # noqa: BLE001
            out.append("")
    return out


def vocab_trie(tokenizer, vocab_size: int) -> Tuple[_Trie, List[str]]:
    key = id(tokenizer)
    with _lock:
        hit = _TRIES.get(key)
        if hit is not None and hit[0] is tokenizer and len(hit[2]) == min(vocab_size, len(tokenizer)):
            return hit[1], hit[2]
    strs = vocab_strings(tokenizer, vocab_size)
    root = _Trie()
    for i, s in enumerate(strs):
        if not s:
            continue
        node = root
        for ch in s:
            nxt = node.kids.get(ch)
            if nxt is None:
                nxt = node.kids[ch] = _Trie()
            node = nxt
        node.toks.append(i)
    with _lock:
        _TRIES[key] = (tokenizer, root, strs)
    return root, strs


class TokenFSM:
    """Allowed next tokens and token transitions of a CharFSM over one vocabulary."""

    def __init__(self, pattern: str, tokenizer, vocab_size: int, eos_ids: List[int],
                 max_masks: int = 512):
        self.char = CharFSM(pattern)
        self.trie, self.strs = vocab_trie(tokenizer, vocab_size)
        self.vocab_size = vocab_size
        self.eos = sorted(set(e for e in eos_ids if e is not None and 0 <= e < vocab_size))
        self._allowed: Dict[int, Tuple[np.ndarray, Dict[int, int]]] = {}
        self._masks: "OrderedDict[Tuple[int, str], object]" = OrderedDict()
        self._max_masks = max_masks
        self._lock = threading.Lock()

    @property
    def start(self) -> int:
        return self.char.start

    def _expand(self, sid: int) -> Tuple[np.ndarray, Dict[int, int]]:
        hit = self._allowed.get(sid)
        if hit is not None:
            return hit
        ids: List[int] = []
        nxt: Dict[int, int] = {}
        stack = [(self.trie, sid)]
        step = self.char.step
        while stack:
            node, s = stack.pop()
            for ch, kid in node.kids.items():
                n = step(s, ch)
                if n < 0:
                    continue
                for t in kid.toks:
                    ids.append(t)
                    nxt[t] = n
                if kid.kids:
                    stack.append((kid, n))
        out = (np.asarray(sorted(ids), dtype=np.int64), nxt)
        self._allowed[sid] = out
        return out

    def allowed_ids(self, sid: int) -> np.ndarray:
        ids, _ = self._expand(sid)
        if self.char.accepting(sid) and self.eos:
            ids = np.union1d(ids, np.asarray(self.eos, dtype=np.int64))
        if ids.size == 0:
            ids = np.asarray(self.eos, dtype=np.int64)
        return ids

    def next_state(self, sid: int, token: int) -> int:
        return self._expand(sid)[1].get(token, -1)

    def can_continue(self, sid: int) -> bool:
        return self._expand(sid)[0].size > 0

    def mask(self, sid: int, device, vocab: int):
        """bool [vocab] on `device`, True = allowed (cached per state and device)."""
        import torch

        key = (sid, str(device))
        with self._lock:
            m = self._masks.get(key)
            if m is not None and m.numel() == vocab:
                self._masks.move_to_end(key)
                return m
        ids = self.allowed_ids(sid)
        m = torch.zeros(vocab, dtype=torch.bool)
        m[torch.from_numpy(ids[ids < vocab])] = True
        m = m.to(device, non_blocking=False)
        with self._lock:
            self._masks[key] = m
            while len(self._masks) > self._max_masks:
                self._masks.popitem(last=False)
        return m


_FSMS: "OrderedDict[tuple, TokenFSM]" = OrderedDict()


def token_fsm(pattern: str, tokenizer, vocab_size: int, eos_ids: List[int]) -> TokenFSM:
    """Process-wide cache: requests with the same pattern share one compiled machine."""
    key = (pattern, id(tokenizer), vocab_size, tuple(sorted(eos_ids)))
    with _lock:
        f = _FSMS.get(key)
        if f is not None:
            _FSMS.move_to_end(key)
            return f
    f = TokenFSM(pattern, tokenizer, vocab_size, eos_ids)
    with _lock:
        _FSMS[key] = f
        while len(_FSMS) > 64:
            _FSMS.popitem(last=False)
    return f


# ----------------------------------------------------------------------------- grammars
_TOKEN_RE = _stdre.compile(r'''
    (?P<ws>\s+|\#[^\n]*)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<sq>'(?:[^'\\]|\\.)*')
  | (?P<cls>\[(?:[^\]\\]|\\.)*\])
  | (?P<rx>/(?:[^/\\]|\\.)+/[imslux]*)
  | (?P<name>[A-Za-z_][A-Za-z0-9_\-.]*)
  | (?P<op>::=|[|()*+?:])
''', _stdre.VERBOSE)


def _lex(text: str):
    i = 0
    out = []
    while i < len(text):
        m = _TOKEN_RE.match(text, i)
        if m is None:
            raise ValueError(f"grammar: cannot parse at {text[i:i + 20]!r}")
        i = m.end()
        if m.lastgroup != "ws":
            out.append((m.lastgroup, m.group()))
    return out


def _lit_regex(body: str) -> str:
    import json

    s = json.loads('"' + body[1:-1].replace("\\'", "'") + '"') if body[0] == '"' else \
        body[1:-1].encode().decode("unicode_escape")
    return _stdre.escape(s)


def grammar_to_regex(grammar: str) -> str:
    """Regular subset of GBNF (``name ::= ...``) / Lark EBNF (``name: ...``) -> one regex.
    Recursive grammars raise here; engine/guided.py routes them to engine/grammar.py."""
    from .grammar import split_rules
    rules, order = split_rules(grammar)
    entry = next((n for n in ("root", "start") if n in rules), order[0] if order else None)
    if entry is None:
        raise ValueError("grammar: no rules")

    def expand(name: str, stack: Tuple[str, ...]) -> str:
        if name in stack:
            raise ValueError(f"grammar: rule {name!r} is recursive; such grammars run on the "
                             "pushdown matcher (engine/grammar.py)")
        parts = []
        for kind, val in rules[name]:
            if kind in ("str", "sq"):
                parts.append("(?:" + _lit_regex(val) + ")")
            elif kind == "cls":
                parts.append(val)
            elif kind == "rx":
                body = val[1:val.rindex("/")]
                parts.append("(?:" + body + ")")
            elif kind == "name":
                ref = val.lstrip("?")
                if ref not in rules:
                    raise ValueError(f"grammar: undefined rule {ref!r}")
                parts.append("(?:" + expand(ref, stack + (name,)) + ")")
            elif val == "(":
                parts.append("(?:")
            elif val in (")", "|", "*", "+", "?"):
                parts.append(val)
            else:
                raise ValueError(f"grammar: unexpected {val!r}")
        return "".join(parts)

    return expand(entry, ())
