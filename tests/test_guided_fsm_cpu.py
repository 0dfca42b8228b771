"""Guided decoding FSM (engine/fsm.py): regex subset semantics against the `regex` module,
token-level allowed sets against brute-force partial matching, grammar conversion, and the
engine path with cached masks."""

import random

import pytest
import regex
import torch

from enterprise_inference_amd.engine.fsm import CharFSM, TokenFSM, grammar_to_regex
from enterprise_inference_amd.engine.guided import schema_to_regex

PATTERNS = [
    r"[a-c]+x?", r"(?:ab|cd)*e", r"\d{2,4}-\d+", r"[^\"\\]{0,3}z", r"(yes|no|maybe)",
    r"\{[ \t\n]{0,2}\"k\"[ \t\n]{0,2}:[ \t\n]{0,2}-?(?:0|[1-9][0-9]*)\}", r"a.c", r"[\x41-\x43]{3}",
    r"A\w\s\S", schema_to_regex({"type": "object", "properties": {
        "a": {"type": "integer"}, "b": {"type": "string"}, "c": {"type": "array",
                                                              "items": {"type": "boolean"}}}}),
    schema_to_regex({"enum": ["red", "green", 3]}),
]
ALPHA = 'abcdexz-0123456789"\\{}[]:, \t\ntruefalsekABC'


def _accepts(f: CharFSM, s: str) -> bool:
    sid = f.walk(f.start, s)
    return f.accepting(sid)


@pytest.mark.parametrize("pat", PATTERNS)
def test_char_fsm_matches_regex_module(pat):
    f = CharFSM(pat)
    r = regex.compile(pat)
    rng = random.Random(0)
    samples = ["", "abc", "ababe", "12-3", "yes", '{"k": 12}', '{"a": 3, "b": "x"}', "a\nc",
               "ABC", "A1 x", "red", "3", "\"green\""]
    for _ in range(400):
        samples.append("".join(rng.choice(ALPHA) for _ in range(rng.randint(0, 10))))
    for s in samples:
        full = r.fullmatch(s) is not None
        part = r.fullmatch(s, partial=True) is not None
        sid = f.walk(f.start, s)
        assert f.accepting(sid) == full, (pat, s)
        assert (sid >= 0) == part, (pat, s)


class _Tok:
    """Tiny tokenizer: multi-char tokens over a small alphabet (exercises the trie)."""

    def __init__(self):
        base = list('abcxyz0123456789"{}[]:, -') + ["ab", "abc", "12", '{"', '":', "yes", "no",
                                                    "true", "false", '"a', "xyz", "\n"]
        self.vocab = ["<eos>", ""] + base
        self.eos_token_id = 0

    def __len__(self):
        return len(self.vocab)

    def decode(self, ids, skip_special_tokens=True):
        return "".join("" if (skip_special_tokens and i == 0) else self.vocab[i] for i in ids)


@pytest.mark.parametrize("pat", [r"(?:ab|c)+x", r"\d{1,3}", r'\{"a": (?:true|false)\}', r"yes|no"])
def test_token_allowed_sets_match_bruteforce(pat):
    tok = _Tok()
    f = TokenFSM(pat, tok, len(tok), [0])
    r = regex.compile(pat)
    rng = random.Random(1)
    for _ in range(30):                 # random walks through allowed tokens
        sid, text = f.start, ""
        for _ in range(8):
            got = set(f.allowed_ids(sid).tolist())
            want = {i for i, s in enumerate(tok.vocab) if i > 1 and
                    r.fullmatch(text + s, partial=True) is not None}
            if r.fullmatch(text) is not None:
                want.add(0)
            if not want:
                want = {0}
            assert got == want, (pat, text)
            choices = sorted(got - {0})
            if not choices:
                break
            t = rng.choice(choices)
            sid = f.next_state(sid, t)
            text += tok.vocab[t]
        m = f.mask(sid, "cpu", len(tok) + 3)
        assert m.dtype == torch.bool and m.numel() == len(tok) + 3
        assert set(torch.nonzero(m).flatten().tolist()) == set(f.allowed_ids(sid).tolist())


def test_grammar_to_regex_gbnf_and_lark():
    g1 = 'root ::= "SELECT " col " FROM " tbl\ncol ::= "a" | "b" [0-9]+\ntbl ::= "t1" | "t2"'
    r1 = regex.compile(grammar_to_regex(g1))
    assert r1.fullmatch("SELECT a FROM t1") and r1.fullmatch("SELECT b42 FROM t2")
    assert not r1.fullmatch("SELECT c FROM t1")
    g2 = '?start: greeting name\ngreeting: "hi " | "hello "\nname: /[A-Z][a-z]+/'
    r2 = regex.compile(grammar_to_regex(g2))
    assert r2.fullmatch("hello Bob") and not r2.fullmatch("hey Bob")
    with pytest.raises(ValueError, match="recursive"):
        grammar_to_regex('root ::= "(" root ")" | "x"')


def test_engine_guided_regex_and_grammar_outputs_match():
    from enterprise_inference_amd.engine.llm_engine import LLMEngine
    from enterprise_inference_amd.engine.sampling_params import SamplingParams
    from enterprise_inference_amd.config import EngineConfig, ModelConfig, CacheConfig, SchedulerConfig
    from enterprise_inference_amd.models.catalog import tiny_config

    d = tiny_config("LlamaForCausalLM", vocab_size=300)
    cfg = EngineConfig(model=ModelConfig.from_hf_dict(d), cache=CacheConfig(block_size=16,
                       num_gpu_blocks=64), scheduler=SchedulerConfig(max_num_seqs=8,
                       max_num_batched_tokens=256, max_model_len=256), device="cpu",
                       dtype=torch.float32, load_format="dummy")
    eng = LLMEngine(cfg)
    pat = r"[0-9]{3}-[a-c]{2}"
    outs = eng.generate(prompts=["id:", "code"], params=SamplingParams(
        max_tokens=20, temperature=0.8, seed=1, guided_regex=pat))
    for o in outs:
        assert regex.fullmatch(pat, o.outputs[0].text), o.outputs[0].text
    g = 'root ::= "ans=" ("yes" | "no")'
    o = eng.generate(prompts=["q"], params=SamplingParams(max_tokens=20, temperature=1.0, seed=2,
                                                          guided_grammar=g))[0]
    assert o.outputs[0].text in ("ans=yes", "ans=no"), o.outputs[0].text
