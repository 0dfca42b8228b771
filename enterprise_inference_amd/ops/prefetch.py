"""Infinity Cache (MALL) warm-up of decode weight streams on a parallel graph branch.

The decode layer chain QKV -> attention -> O -> norm -> gate_up -> down is strictly serial, but
the weights each GEMM streams depend on nothing: while the latency-bound attention kernel runs
(~2 TB/s of HBM in use at batch 65), a read sweep of the O projection (and a prefix of gate_up)
on a side stream fills the 256 MB memory-side cache, and those GEMMs then start from cache
(csrc/kernels/prefetch.hip).  Forked right after the QKV GEMM and joined right before the O
GEMM, so the sweep never competes with a bandwidth-bound GEMM.  Switch: EIA_MALL_PREFETCH=1
(MB of gate_up to include: EIA_MALL_PREFETCH_GATE_MB, default 0)."""

from __future__ import annotations

import os
from typing import Callable, List, Optional, Tuple

import torch

from ._dispatch import check, lib, ptr, stream

ENABLED = os.environ.get("EIA_MALL_PREFETCH", "0") == "1"
GATE_MB = int(os.environ.get("EIA_MALL_PREFETCH_GATE_MB", "0"))
WGS = int(os.environ.get("EIA_MALL_PREFETCH_WGS", "128"))

_side = {}
_sink = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _side.get(dev)
    if s is None:
        s = _side[dev] = torch.cuda.Stream(device=dev)
        _sink[dev] = torch.zeros(64, dtype=torch.int32, device=dev)
    return s


def mall_prefetch(t: torch.Tensor, nbytes: Optional[int] = None, wgs: int = WGS) -> None:
    """Read the first ``nbytes`` of ``t`` (all of it by default) on the current stream."""
    n = t.numel() * t.element_size() if nbytes is None else min(nbytes, t.numel() * t.element_size())
    n -= n % 16
    check(lib().eia_mall_prefetch(ptr(t), n, wgs, ptr(_sink[t.device]), stream(t)),
          "mall_prefetch")


def fork(ranges: List[Tuple[torch.Tensor, Optional[int]]]) -> Callable[[], None]:
    """Launch the sweeps of ``ranges`` on the side stream (ordered after the current stream's
    work so far); returns the join to call before the first consumer."""
    cur = torch.cuda.current_stream()
    side = _side_stream(cur.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        for t, nb in ranges:
            mall_prefetch(t, nb)

    def join() -> None:
        cur.wait_stream(side)
    return join
