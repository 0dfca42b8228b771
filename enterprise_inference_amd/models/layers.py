"""Tensor-parallel building blocks (SURVEY §2.11 "TP" row).

Weights are stored [out, in] (torch Linear convention) so ``F.linear`` goes to
hipBLASLt for the plain GEMMs (K6).  Every parameter carries a ``weight_loader``
that takes the FULL checkpoint tensor and keeps this rank's shard, so the same
loader serves TP=1..8 and the TP-vs-TP1 equivalence tests.
"""

from __future__ import annotations

import os

from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import gemm
from ..parallel import comm, state


def _param(shape, dtype, device) -> nn.Parameter:
    return nn.Parameter(torch.empty(shape, dtype=dtype, device=device), requires_grad=False)


def _shard(t: torch.Tensor, dim: int, rank: int, size: int) -> torch.Tensor:
    n = t.shape[dim]
    if n % size != 0:
        raise ValueError(f"dim {dim} of size {n} not divisible by tp={size}")
    return t.narrow(dim, rank * (n // size), n // size)


def default_loader(param: nn.Parameter, loaded: torch.Tensor) -> None:
    if param.shape != loaded.shape:
        raise ValueError(f"shape mismatch {tuple(param.shape)} vs {tuple(loaded.shape)}")
    param.data.copy_(loaded)


class ColumnParallelLinear(nn.Module):
    """y = x W^T (+b), W split along the output dim; optional gather of y."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False,
                 gather_output: bool = False, dtype=torch.bfloat16, device=None):
        super().__init__()
        tp = state.tp_size()
        self.in_features, self.out_features = in_features, out_features
        self.out_local = out_features // tp
        self.gather_output = gather_output
        self.weight = _param((self.out_local, in_features), dtype, device)
        self.weight.weight_loader = self._load
        self.bias = _param((self.out_local,), dtype, device) if bias else None
        if self.bias is not None:
            self.bias.weight_loader = self._load

    def _load(self, param, loaded, shard_id=None):
        param.data.copy_(_shard(loaded, 0, state.tp_rank(), state.tp_size()))

    def forward(self, x):
        y = gemm.linear(x, self.weight, self.bias)
        if self.gather_output:
            y = comm.all_gather(y, -1)
        return y


class MergedColumnParallelLinear(ColumnParallelLinear):
    """Several column-parallel outputs fused into one GEMM (e.g. gate_up_proj)."""

    def __init__(self, in_features: int, out_sizes: Sequence[int], bias: bool = False,
                 dtype=torch.bfloat16, device=None):
        super().__init__(in_features, sum(out_sizes), bias, False, dtype, device)
        self.out_sizes = list(out_sizes)

    def _load(self, param, loaded, shard_id=None):
        tp, r = state.tp_size(), state.tp_rank()
        if shard_id is None:   # fused checkpoint tensor: split per part first
            parts = torch.split(loaded, self.out_sizes, dim=0)
            param.data.copy_(torch.cat([_shard(p, 0, r, tp) for p in parts], 0))
            return
        off = sum(self.out_sizes[:shard_id]) // tp
        n = self.out_sizes[shard_id] // tp
        param.data.narrow(0, off, n).copy_(_shard(loaded, 0, r, tp))

    def forward_act_and_mul(self, x, act: str = "silu"):
        """act(x Wg^T) * (x Wu^T) for a [gate; up] merged projection.

        Decode-sized batches run the fused SwiGLU GEMM (K7: the 2I-wide
        intermediate never reaches HBM); prompt-sized ones hipBLASLt (TunableOp picks, 1.5-1.6
        PFLOP/s) + the act_and_mul kernel -- a hand MFMA form with the epilogue fused reached
        1.2 PFLOP/s and lost in the prefill step, so it was removed (docs/performance.md).
        """
        if act == "silu" and self.bias is None and len(self.out_sizes) == 2 and \
                x.dim() == 2 and gemm.skinny_ok(x, self.weight, swiglu=True):
            return gemm.swiglu_gemm(x, self.weight)
        from ..ops import activation
        return activation.act_and_mul(gemm.linear(x, self.weight, self.bias), act)


class QKVParallelLinear(ColumnParallelLinear):
    """Fused q/k/v projection; heads split across ranks (kv heads replicated if < tp)."""

    def __init__(self, hidden: int, head_dim: int, num_heads: int, num_kv_heads: int,
                 bias: bool = False, dtype=torch.bfloat16, device=None):
        tp = state.tp_size()
        if num_heads % tp != 0:
            raise ValueError("num_heads must be divisible by tensor_parallel_size")
        self.head_dim = head_dim
        self.num_heads = num_heads // tp
        self.kv_replicas = max(1, tp // num_kv_heads)
        self.num_kv_heads = max(1, num_kv_heads // tp)
        self.total_kv_heads = num_kv_heads
        out_local = (self.num_heads + 2 * self.num_kv_heads) * head_dim
        nn.Module.__init__(self)
        self.in_features = hidden
        self.out_local = out_local
        self.gather_output = False
        self.weight = _param((out_local, hidden), dtype, device)
        self.weight.weight_loader = self._load
        self.bias = _param((out_local,), dtype, device) if bias else None
        if self.bias is not None:
            self.bias.weight_loader = self._load

    def _kv_head_range(self):
        r = state.tp_rank()
        first = (r // self.kv_replicas) * self.num_kv_heads
        return first, self.num_kv_heads

    def _load(self, param, loaded, shard_id=None):
        d = self.head_dim
        r = state.tp_rank()
        qn, kvn = self.num_heads * d, self.num_kv_heads * d
        if shard_id is None:  # fused [q; k; v] checkpoint tensor
            tq = self.num_heads * state.tp_size() * d
            tkv = self.total_kv_heads * d
            q, k, v = torch.split(loaded, [tq, tkv, tkv], dim=0)
            for sid, t in (("q", q), ("k", k), ("v", v)):
                self._load(param, t, sid)
            return
        if shard_id == "q":
            param.data.narrow(0, 0, qn).copy_(loaded.narrow(0, r * qn, qn))
        else:
            first, n = self._kv_head_range()
            src = loaded.narrow(0, first * d, n * d)
            off = qn if shard_id == "k" else qn + kvn
            param.data.narrow(0, off, kvn).copy_(src)


class PendingAllReduce:
    """Row-parallel partial sums whose TP all-reduce is deferred to the consumer: an
    add+RMSNorm fuses it (``comm.all_reduce_add_rmsnorm``), anything else materialises."""

    __slots__ = ("partial",)

    def __init__(self, partial: torch.Tensor):
        self.partial = partial

    def materialize(self) -> torch.Tensor:
        p = self.partial
        if hasattr(p, "materialize"):          # split-K slabs (gemm.SplitK)
            p = p.materialize()
        return comm.all_reduce(p)


class RowParallelLinear(nn.Module):
    """y = x W^T (+b), W split along the input dim; all-reduce of the partial sums."""

    def __init__(self, in_features: int, out_features: int, bias: bool = False,
                 reduce_results: bool = True, dtype=torch.bfloat16, device=None):
        super().__init__()
        tp = state.tp_size()
        self.in_local = in_features // tp
        self.out_features = out_features
        self.reduce_results = reduce_results
        self.weight = _param((out_features, self.in_local), dtype, device)
        self.weight.weight_loader = self._load
        self.bias = _param((out_features,), dtype, device) if bias else None
        if self.bias is not None:
            self.bias.weight_loader = default_loader

    def _load(self, param, loaded, shard_id=None):
        param.data.copy_(_shard(loaded, 1, state.tp_rank(), state.tp_size()))

    def forward(self, x, defer_reduce: bool = False):
        """With ``defer_reduce`` the consumer's add+RMSNorm absorbs the reduction: at TP=1 the
        result may be a ``gemm.SplitK`` (split-K partials summed in the norm kernel), at TP>1
        a ``PendingAllReduce`` (all-reduce + add + norm in one xGMI kernel).  Prefill-sized
        inputs at TP>1 overlap the reduction with the GEMM instead (``_gemm_ar_overlapped``)."""
        if defer_reduce and (state.tp_size() == 1 or not self.reduce_results):
            return gemm.linear(x, self.weight, self.bias, defer_reduce=True)
        if (self.reduce_results and state.tp_size() > 1 and x.dim() == 2
                and x.shape[0] >= _overlap_min_tokens()):
            y = self._gemm_ar_overlapped(x)
            return y + self.bias if self.bias is not None else y
        if defer_reduce and self.bias is None and x.dim() == 2:
            # decode: the GEMM's split-K slabs (if it splits) go straight to the fused
            # all-reduce + add + RMSNorm kernel, which sums them while staging
            return PendingAllReduce(gemm.linear(x, self.weight, defer_reduce=True))
        y = gemm.linear(x, self.weight)
        if self.reduce_results:
            y = comm.all_reduce(y)
        if self.bias is not None:
            y = y + self.bias
        return y


    def _gemm_ar_overlapped(self, x: torch.Tensor) -> torch.Tensor:
        """Token chunks: GEMM(chunk i+1) on the compute stream while RCCL all-reduces chunk i
        on its own stream (async_op), so the xGMI reduction of a prefill step hides behind
        the next chunk's MFMA work instead of following the whole GEMM."""
        T = x.shape[0]
        n = max(2, min(_OVERLAP_MAX_CHUNKS, T // _overlap_min_tokens() * 2))
        y = torch.empty(T, self.out_features, dtype=x.dtype, device=x.device)
        step = -(-T // n)
        works = []
        for a in range(0, T, step):
            b = min(T, a + step)
            torch.matmul(x[a:b], self.weight.t(), out=y[a:b])
            works.append(comm.all_reduce_async(y[a:b]))
        for w in works:
            if w is not None:
                w.wait()
        return y


_OVERLAP_MAX_CHUNKS = 4


def _overlap_min_tokens() -> int:
    """Read per call: every TP rank must take the same branch (EIA_TP_OVERLAP_MIN_TOKENS,
    0 disables)."""
    v = int(os.environ.get("EIA_TP_OVERLAP_MIN_TOKENS", "1024"))
    return v if v > 0 else 1 << 62


class ReplicatedLinear(nn.Module):
    def __init__(self, in_features, out_features, bias=False, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.weight = _param((out_features, in_features), dtype, device)
        self.weight.weight_loader = default_loader
        self.bias = _param((out_features,), dtype, device) if bias else None
        if self.bias is not None:
            self.bias.weight_loader = default_loader

    def forward(self, x):
        return gemm.linear(x, self.weight, self.bias)


class VocabParallelEmbedding(nn.Module):
    """Embedding with the vocab split across ranks (K10 + C3)."""

    def __init__(self, vocab: int, dim: int, dtype=torch.bfloat16, device=None):
        super().__init__()
        tp = state.tp_size()
        self.vocab = vocab
        self.vocab_padded = ((vocab + 64 * tp - 1) // (64 * tp)) * 64 * tp
        self.per_rank = self.vocab_padded // tp
        self.start = state.tp_rank() * self.per_rank
        self.weight = _param((self.per_rank, dim), dtype, device)
        self.weight.weight_loader = self._load

    def _load(self, param, loaded, shard_id=None):
        n = max(0, min(self.per_rank, loaded.shape[0] - self.start))
        param.data.zero_()
        if n > 0:
            param.data[:n].copy_(loaded[self.start:self.start + n])

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        if state.tp_size() == 1:
            return F.embedding(ids, self.weight)
        local = ids - self.start
        mask = (local < 0) | (local >= self.per_rank)
        out = F.embedding(local.masked_fill(mask, 0), self.weight)
        out = out.masked_fill(mask[:, None], 0)
        return comm.all_reduce(out)


class ParallelLMHead(nn.Module):
    """Vocab-parallel LM head; logits gathered across ranks (C4)."""

    def __init__(self, vocab: int, dim: int, dtype=torch.bfloat16, device=None,
                 tied: Optional[VocabParallelEmbedding] = None):
        super().__init__()
        tp = state.tp_size()
        self.vocab = vocab
        self.vocab_padded = ((vocab + 64 * tp - 1) // (64 * tp)) * 64 * tp
        self.per_rank = self.vocab_padded // tp
        self.start = state.tp_rank() * self.per_rank
        if tied is not None:
            self.weight = tied.weight
        else:
            self.weight = _param((self.per_rank, dim), dtype, device)
            self.weight.weight_loader = VocabParallelEmbedding._load.__get__(self)

    @property
    def valid_local(self) -> int:
        """Columns of this rank's shard that are real vocabulary (the rest is padding)."""
        return max(0, min(self.per_rank, self.vocab - self.start))

    def forward_local(self, h: torch.Tensor) -> torch.Tensor:
        """This rank's vocab shard of the logits (no collective)."""
        return gemm.linear(h, self.weight)

    def gather(self, local: torch.Tensor) -> torch.Tensor:
        if state.tp_size() > 1:
            local = comm.all_gather(local, -1)
        return local[..., :self.vocab]

    def forward(self, h: torch.Tensor) -> torch.Tensor:
        return self.gather(self.forward_local(h))

    def forward_f32(self, h: torch.Tensor) -> torch.Tensor:
        """fp32 logits [T, vocab]: one rank, unpadded vocabulary and a decode-sized batch write
        them from the GEMM's fp32 accumulators (no bf16 round trip, no conversion kernel)."""
        if state.tp_size() == 1 and self.per_rank == self.vocab:
            out = gemm.linear_f32(h, self.weight)
            if out is not None:
                return out
        return self.forward(h).float()


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.eps = eps
        self.weight = _param((dim,), dtype, device)
        self.weight.weight_loader = default_loader

    def forward(self, x, residual=None):
        from ..ops import norm
        if isinstance(x, PendingAllReduce):
            if residual is not None:
                return comm.all_reduce_add_rmsnorm(x.partial, residual, self.weight, self.eps)
            x = x.materialize()
        if isinstance(x, gemm.SplitK):
            if residual is not None:
                return gemm.splitk_add_rmsnorm(x, residual, self.weight, self.eps)
            x = x.materialize()
        from ..ops import moe as moe_ops
        if isinstance(x, moe_ops.MoECombine):
            if residual is not None:
                return moe_ops.combine_add_rmsnorm(x, residual, self.weight, self.eps)
            x = x.materialize()
        if residual is None:
            return norm.rms_norm(x, self.weight, self.eps)
        return norm.fused_add_rms_norm(x, residual, self.weight, self.eps)


class LayerNorm(nn.Module):
    def __init__(self, dim: int, eps: float, bias: bool = True, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.eps = eps
        self.weight = _param((dim,), dtype, device)
        self.weight.weight_loader = default_loader
        self.bias = _param((dim,), dtype, device) if bias else None
        if self.bias is not None:
            self.bias.weight_loader = default_loader

    def forward(self, x, residual=None):
        from ..ops import norm
        return norm.layer_norm(x, self.weight, self.bias, self.eps, residual)


class PPMissingLayer(nn.Module):
    """Placeholder for a decoder layer owned by another pipeline stage (no parameters)."""

    def forward(self, *args, **kwargs):   # pragma: no cover - never called
        raise RuntimeError("layer belongs to another pipeline stage")


def init_random_(module: nn.Module, seed: int = 0, std: float = 0.02) -> None:
    """Deterministic random init of every parameter (north star: random weights).

    Norm weights -> 1, biases -> 0, matrices ~ N(0, std). Generated on the
    parameter's device (fast for 70B on GPU), seeded per parameter NAME so that
    a pipeline stage holding a subset of the layers gets the same values.
    """
    import re
    import zlib

    norm_w = re.compile(r"(norm|ln\d*|ln_\w+|layer_norm|layernorm)\.weight$", re.IGNORECASE)
    for name, p in module.named_parameters():
        g = torch.Generator(device=p.device)
        g.manual_seed(seed * 1000003 + zlib.crc32(name.encode()))
        if p.dim() == 1:
            if norm_w.search(name):
                p.data.fill_(1.0)
            else:
                p.data.zero_()
        else:
            p.data.normal_(0.0, std, generator=g)


def all_weight_loaders(module: nn.Module) -> List[str]:
    return [n for n, p in module.named_parameters() if not hasattr(p, "weight_loader")]
