"""Process-group state: one process per GPU, TP groups of consecutive ranks.

Replaces the reference's implicit HCCL setup inside vLLM-Gaudi
(``PT_HPU_ENABLE_LAZY_COLLECTIVES``, core/helm-charts/vllm/gaudi-values.yaml:168):
here ``torch.distributed`` with backend "nccl" is RCCL over xGMI on ROCm, and
"gloo" serves the CPU path / CPU tests.  With world = DP x TP, rank r belongs to
TP group r // TP and DP group r % TP.  EP (``--enable-expert-parallel``,
core/helm-charts/vllm/gaudi3-values.yaml:492) reuses the TP group.
"""

from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch
import torch.distributed as dist

_TP_GROUP: Optional[dist.ProcessGroup] = None
_DP_GROUP: Optional[dist.ProcessGroup] = None
_CPU_GROUP: Optional[dist.ProcessGroup] = None   # gloo mirror of the TP group (host metadata)
_TP_RANK = 0
_TP_SIZE = 1
_TP_RANKS: List[int] = [0]
_EP_ENABLED = False


def env_rank() -> int:
    return int(os.environ.get("RANK", "0"))


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def env_local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def init_distributed(tp_size: int = 1, backend: Optional[str] = None,
                     enable_expert_parallel: bool = False, timeout_s: float = 600.0) -> None:
    """Initialise torch.distributed from the torchrun env (no-op for a single process)."""
    global _TP_GROUP, _DP_GROUP, _CPU_GROUP, _TP_RANK, _TP_SIZE, _TP_RANKS, _EP_ENABLED
    world = env_world()
    _EP_ENABLED = enable_expert_parallel
    if world == 1 and tp_size == 1:
        _TP_RANK, _TP_SIZE, _TP_RANKS = 0, 1, [0]
        return
    if world % tp_size != 0:
        raise ValueError(f"WORLD_SIZE={world} not divisible by tensor_parallel_size={tp_size}")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", env_local_rank())
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s),
                                **kw)
    rank = dist.get_rank()
    # every rank must create every group in the same order
    for g in range(world // tp_size):
        ranks = list(range(g * tp_size, (g + 1) * tp_size))
        grp = dist.new_group(ranks) if tp_size > 1 else None
        cpu = dist.new_group(ranks, backend="gloo") if tp_size > 1 else None
        if rank in ranks:
            _TP_GROUP, _CPU_GROUP, _TP_RANKS = grp, cpu, ranks
    for i in range(tp_size):
        ranks = list(range(i, world, tp_size))
        grp = dist.new_group(ranks) if len(ranks) > 1 else None
        if rank in ranks:
            _DP_GROUP = grp
    _TP_SIZE = tp_size
    _TP_RANK = rank % tp_size


def destroy_distributed() -> None:
    global _TP_GROUP, _DP_GROUP, _CPU_GROUP, _TP_RANK, _TP_SIZE, _TP_RANKS
    if dist.is_initialized():
        dist.destroy_process_group()
    _TP_GROUP = _DP_GROUP = _CPU_GROUP = None
    _TP_RANK, _TP_SIZE, _TP_RANKS = 0, 1, [0]


def tp_rank() -> int:
    return _TP_RANK


def tp_size() -> int:
    return _TP_SIZE


def tp_group() -> Optional[dist.ProcessGroup]:
    return _TP_GROUP


def tp_cpu_group() -> Optional[dist.ProcessGroup]:
    return _CPU_GROUP


def tp_ranks() -> List[int]:
    return list(_TP_RANKS)


def dp_group() -> Optional[dist.ProcessGroup]:
    return _DP_GROUP


def ep_enabled() -> bool:
    return _EP_ENABLED and _TP_SIZE > 1


def is_driver() -> bool:
    return _TP_RANK == 0


def set_tp_for_testing(rank: int, size: int) -> None:
    """Pretend to be TP rank `rank` of `size` without communication (weight-sharding tests)."""
    global _TP_RANK, _TP_SIZE
    _TP_RANK, _TP_SIZE = rank, size
