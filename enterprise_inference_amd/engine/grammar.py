"""Context-free ``guided_grammar`` (recursive GBNF / Lark EBNF) -> token masks.

The regular subset of a grammar compiles to a regex and runs on the cached token FSM
(engine/fsm.py).  A grammar whose rules recurse (nested JSON, arithmetic expressions, ...) is
not regular; it compiles here into a context-free grammar over character classes, and a
native pushdown matcher (csrc/runtime/grammar.cpp) tracks the set of parser stacks:

  * a stack is a list of (rule, alternative, position) frames; its top always points at a
    character-class terminal (rule references are expanded, finished alternatives popped),
  * a character advances every stack whose top class matches it,
  * stack sets are interned and (set, character) transitions cached, so the matcher is a
    lazily built automaton whose states are stack sets, shared by every request using the
    grammar (a JSON string body loops on one state),
  * a token is allowed when walking its characters keeps at least one stack alive -- found
    for the whole vocabulary by one walk of the vocabulary trie from the state (shared
    prefixes stepped once, dead branches pruned), cached per state, with its device mask,
  * EOS is allowed when some stack is empty (the start rule is complete).

Repetition (``* + ? {m,n}``) and groups become helper rules; string literals become class
sequences; ``/regex/`` terminals and ``[...]`` classes reuse the regex parser of engine/fsm.py.
Left-recursive rules (``expr ::= expr "+" term``) cannot be expanded top-down and are rejected
with a clear error (rewrite them right-recursively: ``expr ::= term ("+" term)*``).
"""

from __future__ import annotations

import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

from .fsm import CharSet, _lex, _Parser

MAX_CP = 0x10FFFF


class CFG:
    """Rules: list of alternatives; an alternative is a list of symbols (>= 0: class id,
    < 0: rule -(id+1)).  Classes: sorted code-point ranges, negation applied."""

    def __init__(self):
        self.classes: List[List[Tuple[int, int]]] = []
        self.rules: List[List[List[int]]] = []
        self.names: List[str] = []
        self.start = 0
        self._cls_ids: Dict[tuple, int] = {}

    def add_class(self, cs: CharSet) -> int:
        rng = sorted(cs.ranges)
        if cs.neg:                                   # complement over [0, MAX_CP]
            out, lo = [], 0
            for a, b in rng:
                if a > lo:
                    out.append((lo, a - 1))
                lo = max(lo, b + 1)
            if lo <= MAX_CP:
                out.append((lo, MAX_CP))
            rng = out
        key = tuple(rng)
        if key not in self._cls_ids:
            self._cls_ids[key] = len(self.classes)
            self.classes.append(list(rng))
        return self._cls_ids[key]

    def new_rule(self, name: str) -> int:
        self.rules.append([])
        self.names.append(name)
        return len(self.rules) - 1


def _rule_sym(rid: int) -> int:
    return -(rid + 1)


class _Lower:
    """AST (fsm._Parser node shapes + ("ref", name)) -> CFG alternatives."""

    def __init__(self, cfg: CFG, rule_ids: Dict[str, int]):
        self.cfg = cfg
        self.rule_ids = rule_ids
        self.n_helper = 0

    def helper(self, alts: List[List[int]]) -> int:
        rid = self.cfg.new_rule(f"_h{self.n_helper}")
        self.n_helper += 1
        self.cfg.rules[rid] = alts
        return rid

    def seq(self, node) -> List[int]:
        """Symbols of a node used inside a concatenation."""
        kind = node[0]
        if kind == "lit":
            return [self.cfg.add_class(node[1])]
        if kind == "ref":
            if node[1] not in self.rule_ids:
                raise ValueError(f"grammar: undefined rule {node[1]!r}")
            return [_rule_sym(self.rule_ids[node[1]])]
        if kind == "cat":
            out: List[int] = []
            for it in node[1]:
                out += self.seq(it)
            return out
        if kind == "alt":
            return [_rule_sym(self.helper([self.seq(p) for p in node[1]]))]
        if kind == "rep":
            _, sub, lo, hi = node
            body = self.seq(sub)
            out = body * lo
            if hi is None:                            # X* : S -> X S | eps
                rid = self.cfg.new_rule(f"_h{self.n_helper}")
                self.n_helper += 1
                self.cfg.rules[rid] = [body + [_rule_sym(rid)], []]
                out.append(_rule_sym(rid))
            elif hi > lo:                             # X{0,k}: nested optionals
                rid = None
                for _ in range(hi - lo):
                    alts = [body + ([_rule_sym(rid)] if rid is not None else []), []]
                    rid = self.helper(alts)
                out.append(_rule_sym(rid))
            return out
        raise ValueError(f"grammar: unsupported node {kind!r}")


def _parse_body(tokens) -> tuple:
    """Rule body tokens (fsm._lex) -> AST: alternation / concatenation / repetition / groups."""
    pos = 0

    def peek():
        return tokens[pos] if pos < len(tokens) else (None, None)

    def alt():
        nonlocal pos
        parts = [cat()]
        while peek()[1] == "|":
            pos += 1
            parts.append(cat())
        return parts[0] if len(parts) == 1 else ("alt", parts)

    def cat():
        items = []
        while peek()[0] is not None and peek()[1] not in ("|", ")"):
            items.append(rep())
        return ("cat", items)

    def rep():
        nonlocal pos
        node = atom()
        while peek()[1] in ("*", "+", "?"):
            op = peek()[1]
            pos += 1
            node = ("rep", node, 0 if op != "+" else 1, 1 if op == "?" else None)
        return node

    def atom():
        nonlocal pos
        kind, val = peek()
        pos += 1
        if val == "(":
            node = alt()
            if peek()[1] != ")":
                raise ValueError("grammar: unbalanced parenthesis")
            pos += 1
            return node
        if kind in ("str", "sq"):
            import json
            s = json.loads(val) if kind == "str" else \
                val[1:-1].encode().decode("unicode_escape")
            return ("cat", [("lit", CharSet([(ord(ch), ord(ch))])) for ch in s])
        if kind == "cls":
            return _Parser(val).parse()
        if kind == "rx":
            return _Parser(val[1:val.rindex("/")]).parse()
        if kind == "name":
            return ("ref", val.lstrip("?"))
        raise ValueError(f"grammar: unexpected {val!r}")

    node = alt()
    if pos != len(tokens):
        raise ValueError(f"grammar: unexpected {tokens[pos][1]!r}")
    return node


def split_rules(text: str) -> Tuple[Dict[str, list], List[str]]:
    """``name ::= body`` / ``name: body`` rules -> ({name: body tokens}, order)."""
    toks = _lex(text)
    rules: Dict[str, list] = {}
    order: List[str] = []
    i = 0
    while i < len(toks):
        if toks[i][1] == "?" and i + 1 < len(toks) and toks[i + 1][0] == "name":
            i += 1
        kind, val = toks[i]
        if kind != "name" or i + 1 >= len(toks) or toks[i + 1][1] not in ("::=", ":"):
            raise ValueError(f"grammar: expected 'name ::=' or 'name:' at {val!r}")
        name = val.lstrip("?")
        j = i + 2
        body = []
        depth = 0
        while j < len(toks):
            k2, v2 = toks[j]
            if depth == 0 and k2 == "name" and j + 1 < len(toks) and toks[j + 1][1] in ("::=", ":"):
                break
            # Lark's inline-rule marker (``?name:``); before ``name ::=`` a ``?`` is the
            # optional operator of the previous GBNF rule's last item
            if (depth == 0 and v2 == "?" and j + 2 < len(toks) and toks[j + 1][0] == "name"
                    and toks[j + 2][1] == ":"):
                break
            depth += v2 == "("
            depth -= v2 == ")"
            body.append(toks[j])
            j += 1
        rules[name] = body
        order.append(name)
        i = j
    if not order:
        raise ValueError("grammar: no rules")
    return rules, order


def _check_left_recursion(cfg: CFG) -> None:
    n = len(cfg.rules)
    nullable = [False] * n
    changed = True
    while changed:
        changed = False
        for r, alts in enumerate(cfg.rules):
            if nullable[r]:
                continue
            for a in alts:
                if all(s < 0 and nullable[-s - 1] for s in a):
                    nullable[r] = changed = True
                    break
    left: List[set] = [set() for _ in range(n)]      # rules reachable in leftmost position
    for r, alts in enumerate(cfg.rules):
        for a in alts:
            for s in a:
                if s >= 0:
                    break
                left[r].add(-s - 1)
                if not nullable[-s - 1]:
                    break
    for r in range(n):
        seen, todo = set(), list(left[r])
        while todo:
            x = todo.pop()
            if x == r:
                raise ValueError(f"grammar: rule {cfg.names[r]!r} is left-recursive; rewrite "
                                 "it right-recursively (e.g. expr ::= term (\"+\" term)*)")
            if x not in seen:
                seen.add(x)
                todo.extend(left[x])


def compile_cfg(text: str) -> CFG:
    rules, order = split_rules(text)
    cfg = CFG()
    ids = {name: cfg.new_rule(name) for name in order}
    low = _Lower(cfg, ids)
    for name in order:
        node = _parse_body(rules[name])
        alts = node[1] if node[0] == "alt" else [node]
        cfg.rules[ids[name]] = [low.seq(a) for a in alts]
    entry = next((n for n in ("root", "start") if n in ids), order[0])
    cfg.start = ids[entry]
    _check_left_recursion(cfg)
    return cfg


def is_recursive(text: str) -> bool:
    """True when some rule reaches itself (the grammar is not a regular language as written)."""
    rules, order = split_rules(text)
    refs = {n: {v.lstrip("?") for k, v in body if k == "name"} for n, body in rules.items()}
    for start in order:
        seen, todo = set(), list(refs[start])
        while todo:
            x = todo.pop()
            if x == start:
                return True
            if x in refs and x not in seen:
                seen.add(x)
                todo.extend(refs[x])
    return False


def validate_grammar(text: str) -> None:
    """ValueError for a grammar neither the regex path nor the pushdown matcher accepts."""
    if is_recursive(text):
        compile_cfg(text)
    else:
        from .fsm import grammar_to_regex
        grammar_to_regex(text)


# ----------------------------------------------------------------------------- native matcher
_VOCABS: Dict[int, tuple] = {}
_GRAMMARS: "OrderedDict[str, object]" = OrderedDict()
_lock = threading.Lock()


def native_vocab(tokenizer, vocab_size: int):
    """The vocabulary's code points in the native trie (built once per tokenizer)."""
    from .. import _native
    from .fsm import vocab_strings
    key = id(tokenizer)
    with _lock:
        hit = _VOCABS.get(key)
        if hit is not None and hit[0] is tokenizer and hit[2] == vocab_size:
            return hit[1]
    strs = vocab_strings(tokenizer, vocab_size)
    v = _native.runtime().GrammarVocab([[ord(c) for c in s] for s in strs])
    with _lock:
        _VOCABS[key] = (tokenizer, v, vocab_size)
    return v


def native_grammar(text: str):
    from .. import _native
    with _lock:
        g = _GRAMMARS.get(text)
        if g is not None:
            _GRAMMARS.move_to_end(text)
            return g
    cfg = compile_cfg(text)
    g = _native.runtime().Grammar(cfg.classes, cfg.rules, cfg.start)
    with _lock:
        _GRAMMARS[text] = g
        while len(_GRAMMARS) > 64:
            _GRAMMARS.popitem(last=False)
    return g


_DEV_MASKS: "OrderedDict[tuple, object]" = OrderedDict()


class GrammarState:
    """Per-sequence pushdown state (engine/guided.py GuidedState interface).  The automaton
    behind it is shared by every request with the same grammar text, and so are the device
    masks of its states (no host->device copy for a state seen before)."""

    def __init__(self, text: str, tokenizer, vocab_size: int, eos_ids: List[int]):
        from .. import _native
        self.grammar = native_grammar(text)
        self.vocab = native_vocab(tokenizer, vocab_size)
        self.m = _native.runtime().GrammarMatcher(self.grammar, self.vocab)
        self.eos = sorted(set(e for e in eos_ids if e is not None and 0 <= e < vocab_size))
        self.done = False

    def _host_mask(self, vocab: int):
        import numpy as np
        m = self.m.mask()
        out = np.zeros(vocab, dtype=np.bool_)
        n = min(vocab, m.shape[0])
        out[:n] = m[:n].astype(np.bool_)
        if self.m.accepting() or not out.any():
            e = [t for t in self.eos if t < vocab]
            out[e] = True
        return out

    def allowed_tokens(self) -> List[int]:
        import numpy as np
        return np.nonzero(self._host_mask(max(self.vocab.size, 1 + max(self.eos, default=0))))[0].tolist()

    def allowed_mask(self, device, vocab: int):
        import torch
        key = (id(self.grammar), id(self.vocab), self.m.state(), str(device), vocab)
        with _lock:
            hit = _DEV_MASKS.get(key)
            if hit is not None and hit[0] is self.grammar:
                _DEV_MASKS.move_to_end(key)
                return hit[1]
        t = torch.from_numpy(self._host_mask(vocab)).to(device)
        with _lock:
            _DEV_MASKS[key] = (self.grammar, t)
            while len(_DEV_MASKS) > 256:
                _DEV_MASKS.popitem(last=False)
        return t

    def advance(self, token: int) -> None:
        if token in self.eos:
            self.done = True
            return
        if not self.m.advance_token(int(token)):
            self.done = True            # not allowed (an unmasked fallback row sampled it)
            return
        if self.m.accepting() and not self.m.can_continue():
            self.done = True

    def is_done(self) -> bool:
        return self.done
