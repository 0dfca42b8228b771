"""Recursive ``guided_grammar`` (engine/grammar.py + csrc/runtime/grammar.cpp): the native
pushdown matcher against an independent Earley recognizer over the same CFG (full-string
acceptance and prefix viability), token-level allowed sets against brute force, and the engine
path producing grammar-conforming text.  Parity with the reference's own guided-grammar backend
is unpinned (it delegates to vLLM, not importable here); the oracle is the CFG's language."""

import random

import pytest
import torch

from enterprise_inference_amd import _native
from enterprise_inference_amd.engine.grammar import (compile_cfg, is_recursive, native_grammar,
                                                     validate_grammar)

PARENS = 'root ::= "(" root ")" root | ""'
EXPR = '''root ::= expr
expr ::= term (("+" | "-") term)*
term ::= factor ("*" factor)*
factor ::= [0-9]+ | "(" expr ")" | "-" factor'''
JSONISH = '''?start: value
value: array | object | NUMBER | "true"
array: "[" (value ("," value)*)? "]"
object: "{" (pair ("," pair)*)? "}"
pair: /"[a-z]{1,3}"/ ":" value
NUMBER: /-?[0-9]+/'''
GRAMMARS = {"parens": PARENS, "expr": EXPR, "json": JSONISH}
ALPHA = {"parens": "()", "expr": "0123-+*()", "json": '[]{},:"ab1-true'}


class Earley:
    """Textbook Earley recognizer over the compiled CFG (symbols: class id >= 0, rule < 0)."""

    def __init__(self, cfg):
        self.cfg = cfg

    def _match(self, cls, cp):
        return any(a <= cp <= b for a, b in self.cfg.classes[cls])

    def chart(self, text):
        rules = self.cfg.rules
        sets = [set() for _ in range(len(text) + 1)]
        sets[0] = {(self.cfg.start, a, 0, 0) for a in range(len(rules[self.cfg.start]))}
        for i in range(len(text) + 1):
            todo = list(sets[i])
            while todo:
                r, a, d, o = todo.pop()
                alt = rules[r][a]
                if d == len(alt):                         # complete
                    for (r2, a2, d2, o2) in list(sets[o]):
                        alt2 = rules[r2][a2]
                        if d2 < len(alt2) and alt2[d2] == -(r + 1):
                            it = (r2, a2, d2 + 1, o2)
                            if it not in sets[i]:
                                sets[i].add(it)
                                todo.append(it)
                    continue
                s = alt[d]
                if s < 0:                                 # predict
                    q = -s - 1
                    for a2 in range(len(rules[q])):
                        it = (q, a2, 0, i)
                        if it not in sets[i]:
                            sets[i].add(it)
                            todo.append(it)
                    # nullable completion already in this set
                    for (r2, a2, d2, o2) in list(sets[i]):
                        if r2 == q and o2 == i and d2 == len(rules[q][a2]):
                            it = (r, a, d + 1, o)
                            if it not in sets[i]:
                                sets[i].add(it)
                                todo.append(it)
                elif i < len(text) and self._match(s, ord(text[i])):
                    sets[i + 1].add((r, a, d + 1, o))
        return sets

    def accepts(self, text):
        last = self.chart(text)[-1]
        return any(r == self.cfg.start and o == 0 and d == len(self.cfg.rules[r][a])
                   for r, a, d, o in last)

    def viable(self, text):
        return bool(self.chart(text)[-1])


def _matcher(text, vocab_strs):
    rt = _native.runtime()
    v = rt.GrammarVocab([[ord(c) for c in s] for s in vocab_strs])
    return rt.GrammarMatcher(native_grammar(text), v)


@pytest.mark.parametrize("name", list(GRAMMARS))
def test_pushdown_matches_earley(name):
    g = GRAMMARS[name]
    assert is_recursive(g)
    cfg = compile_cfg(g)
    oracle = Earley(cfg)
    alpha = sorted(set(ALPHA[name]))
    rng = random.Random(0)
    samples = ["", "()", "(()())", "1+2*3", "(1+2)*-3", "[1,[2,{\"a\":true}],[]]", "{\"ab\":[-1]}"]
    for _ in range(300):
        samples.append("".join(rng.choice(alpha) for _ in range(rng.randint(0, 9))))
    for s in samples:
        m = _matcher(g, [])
        alive = m.advance_text([ord(c) for c in s])
        assert alive == oracle.viable(s), (name, s)
        if alive:
            assert m.accepting() == oracle.accepts(s), (name, s)


class _Tok:
    def __init__(self, pieces):
        self.vocab = ["<eos>", ""] + pieces
        self.eos_token_id = 0

    def __len__(self):
        return len(self.vocab)

    def decode(self, ids, skip_special_tokens=True):
        return "".join("" if (skip_special_tokens and i == 0) else self.vocab[i] for i in ids)


@pytest.mark.parametrize("name", list(GRAMMARS))
def test_token_allowed_sets_match_bruteforce(name):
    from enterprise_inference_amd.engine.grammar import GrammarState
    g = GRAMMARS[name]
    oracle = Earley(compile_cfg(g))
    pieces = sorted(set(ALPHA[name])) + ["((", "))", "()", "12", "+(", ")*", "[1", "],", "true",
                                         '{"a":', '"b"', ",[", "]]", "-1"]
    tok = _Tok(pieces)
    rng = random.Random(2)
    for _ in range(12):
        st = GrammarState(g, tok, len(tok), [0])
        text = ""
        for _ in range(10):
            got = set(st.allowed_tokens())
            want = {i for i, s in enumerate(tok.vocab) if i > 1 and oracle.viable(text + s)}
            if oracle.accepts(text):
                want.add(0)
            if not want:
                want = {0}
            assert got == want, (name, text)
            choices = sorted(got - {0})
            if not choices or st.is_done():
                break
            t = rng.choice(choices)
            st.advance(t)
            text += tok.vocab[t]
        m = st.allowed_mask("cpu", len(tok) + 2)
        assert set(torch.nonzero(m).flatten().tolist()) == set(st.allowed_tokens())


def test_deep_nesting_keeps_stacks_bounded():
    m = _matcher(EXPR, [])
    s = "(" * 300 + "1" + ")" * 300 + "+2" * 500
    assert m.advance_text([ord(c) for c in s])
    assert m.accepting() and m.num_stacks() < 16


def test_rejections():
    with pytest.raises(ValueError, match="left-recursive"):
        validate_grammar('root ::= root "+" "1" | "1"')
    with pytest.raises(ValueError, match="undefined"):
        validate_grammar('root ::= "(" nope ")" root | ""')
    validate_grammar(PARENS)
    validate_grammar('root ::= "a" | "b"')                  # regular: the regex path


def test_engine_recursive_grammar_outputs_parse():
    from enterprise_inference_amd.config import (CacheConfig, EngineConfig, ModelConfig,
                                                 SchedulerConfig)
    from enterprise_inference_amd.engine.llm_engine import LLMEngine
    from enterprise_inference_amd.engine.sampling_params import SamplingParams
    from enterprise_inference_amd.models.catalog import tiny_config

    d = tiny_config("LlamaForCausalLM", vocab_size=300)
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d), cache=CacheConfig(block_size=16,
                       num_gpu_blocks=64), scheduler=SchedulerConfig(max_num_seqs=8,
                       max_num_batched_tokens=256, max_model_len=256), device="cpu",
                       dtype=torch.float32, load_format="dummy")
    eng = LLMEngine(cfg)
    oracle = Earley(compile_cfg(EXPR))
    outs = eng.generate(prompts=["calc", "x", "expr:"], params=SamplingParams(
        max_tokens=24, temperature=1.0, seed=5, guided_grammar=EXPR))
    for o in outs:
        c = o.outputs[0]
        if c.finish_reason == "stop":
            assert oracle.accepts(c.text), c.text
        else:
            assert oracle.viable(c.text), c.text


TREE = {"$defs": {"node": {"type": "object", "properties": {
    "v": {"type": "integer"}, "kids": {"type": "array", "items": {"$ref": "#/$defs/node"}}},
    "required": ["v", "kids"]}}, "$ref": "#/$defs/node"}


def _accepts_text(grammar, text):
    m = _matcher(grammar, [])
    return m.advance_text([ord(c) for c in text]) and m.accepting()


def test_schema_to_grammar_recursive_and_free_form():
    import json
    from enterprise_inference_amd.engine.guided import schema_needs_grammar, schema_to_grammar
    assert schema_needs_grammar(TREE) and schema_needs_grammar({})
    assert not schema_needs_grammar({"type": "object", "properties": {"a": {"type": "integer"}}})
    g = schema_to_grammar(TREE)
    deep = {"v": 1, "kids": [{"v": 2, "kids": []}]}
    for _ in range(8):                                   # nesting far past the regex bound
        deep = {"v": 0, "kids": [deep, {"v": -3, "kids": []}]}
    assert _accepts_text(g, json.dumps(deep))
    assert _accepts_text(g, json.dumps(deep, separators=(",", ":")))
    assert not _accepts_text(g, json.dumps({"v": "x", "kids": []}))
    assert not _accepts_text(g, json.dumps({"kids": [], "v": 1}))     # property order kept
    free = schema_to_grammar({})
    doc = {"a": [1, 2.5e3, {"b": {"c": [True, None, {"d": "e\\né"}]}}], "f": "g"}
    assert _accepts_text(free, json.dumps(doc))
    assert _accepts_text(free, json.dumps(doc, ensure_ascii=False))
    assert not _accepts_text(free, '{"a": [1,]}')
    enum = schema_to_grammar({"type": "object", "properties": {
        "k": {"enum": ["x\"y", 3]}, "r": {"$ref": "#"}}, "required": ["k"]})
    assert _accepts_text(enum, '{"k": "x\\"y", "r": {"k": 3}}')


def test_engine_recursive_json_schema_outputs_parse():
    import json
    from enterprise_inference_amd.config import (CacheConfig, EngineConfig, ModelConfig,
                                                 SchedulerConfig)
    from enterprise_inference_amd.engine.guided import schema_to_grammar
    from enterprise_inference_amd.engine.llm_engine import LLMEngine
    from enterprise_inference_amd.engine.sampling_params import SamplingParams
    from enterprise_inference_amd.models.catalog import tiny_config

    d = tiny_config("LlamaForCausalLM", vocab_size=300)
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d), cache=CacheConfig(block_size=16,
                       num_gpu_blocks=64), scheduler=SchedulerConfig(max_num_seqs=8,
                       max_num_batched_tokens=256, max_model_len=256), device="cpu",
                       dtype=torch.float32, load_format="dummy")
    eng = LLMEngine(cfg)
    g = schema_to_grammar(TREE)
    outs = eng.generate(prompts=["tree:", "t"], params=SamplingParams(
        max_tokens=60, temperature=0.7, seed=3, guided_json=TREE))
    for o in outs:
        c = o.outputs[0]
        m = _matcher(g, [])
        assert m.advance_text([ord(ch) for ch in c.text]), c.text
        if c.finish_reason == "stop":
            assert m.accepting()
            assert "v" in json.loads(c.text)
