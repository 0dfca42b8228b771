"""GPU-engine vs fp32-oracle parity checks (used by tests/test_e2e_gpu.py and smoke()).

Greedy tokens of a bf16 engine may legitimately differ from an fp32 run where two logits
are closer than bf16 rounding, so a generated token is checked by *teacher forcing*: the
fp32 oracle (HF transformers on the CPU, same weights) scores the engine's own prefix and
the engine's token must be within ``tol`` of the oracle's best logit at every step.  A
real kernel bug (wrong KV slot, stale graph input, bad split-K merge) picks tokens far
from the oracle's argmax within a few steps.
"""

from __future__ import annotations

from typing import Dict, List, Sequence

import torch

_HF_CFG = {"LlamaForCausalLM": "LlamaConfig", "Qwen2ForCausalLM": "Qwen2Config",
           "Qwen3ForCausalLM": "Qwen3Config", "MistralForCausalLM": "MistralConfig",
           "MixtralForCausalLM": "MixtralConfig"}


def hf_reference_model(cfg: dict, seed: int = 0):
    """fp32 CPU transformers model of a (tiny) HF config dict, seeded random weights."""
    import transformers

    arch = cfg["architectures"][0]
    hc = getattr(transformers, _HF_CFG[arch])(**{k: v for k, v in cfg.items()
                                                 if k != "architectures"})
    hc.architectures = [arch]
    torch.manual_seed(seed)
    return getattr(transformers, arch)(hc).float().eval()


@torch.no_grad()
def teacher_forced_margins(hf, prompts: Sequence[List[int]],
                           outputs: Sequence[List[int]], with_scale: bool = False):
    """Per generated token: oracle(best logit) - oracle(logit of the engine's token) >= 0
    (and, with ``with_scale``, the oracle row's logit std -- the scale bf16 rounding of the
    logits grows with)."""
    margins, scales = [], []
    for p, o in zip(prompts, outputs):
        full = torch.tensor([list(p) + list(o)])
        logits = hf(full).logits[0].float()
        rows = logits[len(p) - 1:len(p) - 1 + len(o)]
        best = rows.max(-1).values
        got = rows.gather(1, torch.tensor(o)[:, None])[:, 0]
        margins.append((best - got).tolist())
        scales.append(rows.std(-1).tolist())
    return (margins, scales) if with_scale else margins


def check_greedy(hf, prompts, outputs, tol: float, rel: float = 0.0) -> Dict[str, float]:
    """Every engine token within max(tol, rel * logit-row std) of the oracle's best logit."""
    m, sc = teacher_forced_margins(hf, prompts, outputs, with_scale=True)
    worst = max(max(x) for x in m)
    over = [(x, s) for r, rs in zip(m, sc) for x, s in zip(r, rs) if x > max(tol, rel * s)]
    exact = sum(x == 0.0 for r in m for x in r) / max(1, sum(len(r) for r in m))
    if over:
        raise AssertionError(f"engine token {over[0][0]:.4f} below the fp32 oracle's best logit "
                             f"(tol {tol}, rel {rel} x std {over[0][1]:.3f}); margins {m}")
    return {"worst_margin": worst, "argmax_agreement": exact}


@torch.no_grad()
def check_logprobs(hf, prompts, outputs, engine_logprobs, tol: float) -> Dict[str, float]:
    """Logits-level bound: for every generated step the engine's reported log-probs (its
    top-k + the chosen token, i.e. ``SamplingParams(logprobs=k)``) must match the fp32
    oracle's log-softmax over the same prefix within ``tol`` nats.  Log-probs are the logits
    minus their logsumexp, so this bounds the whole logit row's shape on the entries that
    matter for sampling -- a much sharper check than the token margin on near-flat rows."""
    worst = 0.0
    n = 0
    for p, o, lps in zip(prompts, outputs, engine_logprobs):
        full = torch.tensor([list(p) + list(o)])
        ref = torch.log_softmax(hf(full).logits[0].float(), -1)[len(p) - 1:len(p) - 1 + len(o)]
        for r, d in enumerate(lps):
            ids = torch.tensor(list(d.keys()))
            got = torch.tensor(list(d.values()), dtype=torch.float32)
            err = (got - ref[r, ids]).abs().max().item()
            worst = max(worst, err)
            n += len(d)
    if worst > tol:
        raise AssertionError(f"engine log-probs differ from the fp32 oracle by {worst:.4f} "
                             f"nats (tol {tol})")
    return {"logprob_max_abs": worst, "entries": n}
