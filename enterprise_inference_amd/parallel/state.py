"""Process-group state: one process per GPU, TP groups of consecutive ranks.

Replaces the reference's implicit HCCL setup inside vLLM-Gaudi
(``PT_HPU_ENABLE_LAZY_COLLECTIVES``, core/helm-charts/vllm/gaudi-values.yaml:168):
here ``torch.distributed`` with backend "nccl" is RCCL over xGMI on ROCm, and
"gloo" serves the CPU path / CPU tests.  World = DP x PP x TP; global rank
r = replica * (PP*TP) + stage * TP + tp_rank, so a TP group is TP consecutive ranks of one
pipeline stage, a PP group is the ranks of one replica with the same tp_rank, and DP groups
join the same position of every replica.  EP (``--enable-expert-parallel``,
core/helm-charts/vllm/gaudi3-values.yaml:492) reuses the TP group.  PP mirrors the
reference's CPU-only ``--pipeline-parallel-size`` (core/helm-charts/vllm/templates/
deployment.yaml:75-81); on MI355X a 405B bf16 model fits one node's HBM with TP=8.
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
_PP_RANK = 0
_PP_SIZE = 1
_PP_RANKS: List[int] = [0]           # global ranks of my PP group, by stage
_REPLICA_RANKS: List[int] = [0]      # all PP*TP ranks of my model replica
_REPLICA_CPU_GROUP: Optional[dist.ProcessGroup] = None
_BACKEND = "none"


def env_rank() -> int:
    return int(os.environ.get("RANK", "0"))


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def env_local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def init_distributed(tp_size: int = 1, backend: Optional[str] = None,
                     enable_expert_parallel: bool = False, timeout_s: float = 600.0,
                     pp_size: int = 1) -> None:
    """Initialise torch.distributed from the torchrun env (no-op for a single process)."""
    global _TP_GROUP, _DP_GROUP, _CPU_GROUP, _TP_RANK, _TP_SIZE, _TP_RANKS, _EP_ENABLED
    global _PP_RANK, _PP_SIZE, _PP_RANKS, _REPLICA_RANKS, _REPLICA_CPU_GROUP, _BACKEND
    world = env_world()
    _EP_ENABLED = enable_expert_parallel
    if world == 1 and tp_size == 1 and pp_size == 1:
        _TP_RANK, _TP_SIZE, _TP_RANKS = 0, 1, [0]
        _PP_RANK, _PP_SIZE, _PP_RANKS, _REPLICA_RANKS = 0, 1, [0], [0]
        return
    rep = tp_size * pp_size
    if world % rep != 0:
        raise ValueError(f"WORLD_SIZE={world} not divisible by tensor_parallel_size x "
                         f"pipeline_parallel_size = {rep}")
    if backend in (None, "auto"):
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", env_local_rank())
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s),
                                **kw)
    _BACKEND = dist.get_backend()
    rank = dist.get_rank()
    # every rank must create every group in the same order
    for g in range(world // tp_size):
        ranks = list(range(g * tp_size, (g + 1) * tp_size))
        grp = dist.new_group(ranks) if tp_size > 1 else None
        cpu = dist.new_group(ranks, backend="gloo") if tp_size > 1 else None
        if rank in ranks:
            _TP_GROUP, _CPU_GROUP, _TP_RANKS = grp, cpu, ranks
    for r0 in range(0, world, rep):
        for t in range(tp_size):
            ranks = [r0 + s * tp_size + t for s in range(pp_size)]
            if rank in ranks:
                _PP_RANKS = ranks
        ranks = list(range(r0, r0 + rep))
        cpu = dist.new_group(ranks, backend="gloo") if rep > 1 else None
        if rank in ranks:
            _REPLICA_RANKS, _REPLICA_CPU_GROUP = ranks, cpu
    for i in range(rep):
        ranks = list(range(i, world, rep))
        grp = dist.new_group(ranks) if len(ranks) > 1 else None
        if rank in ranks:
            _DP_GROUP = grp
    _TP_SIZE = tp_size
    _TP_RANK = rank % tp_size
    _PP_SIZE = pp_size
    _PP_RANK = (rank % rep) // tp_size


def destroy_distributed() -> None:
    global _TP_GROUP, _DP_GROUP, _CPU_GROUP, _TP_RANK, _TP_SIZE, _TP_RANKS
    global _PP_RANK, _PP_SIZE, _PP_RANKS, _REPLICA_RANKS, _REPLICA_CPU_GROUP, _BACKEND
    _BACKEND = "none"
    if dist.is_initialized():
        dist.destroy_process_group()
    _TP_GROUP = _DP_GROUP = _CPU_GROUP = _REPLICA_CPU_GROUP = None
    _TP_RANK, _TP_SIZE, _TP_RANKS = 0, 1, [0]
    _PP_RANK, _PP_SIZE, _PP_RANKS, _REPLICA_RANKS = 0, 1, [0], [0]


def backend() -> str:
    """"nccl" (RCCL), "gloo" or "none" (single process)."""
    return _BACKEND


def host_staged() -> bool:
    """Device tensors cross a gloo group through host memory (one-GPU TP rehearsal,
    EIA_TP_SHARE_DEVICE): the collectives in parallel/comm.py stage them."""
    return _BACKEND == "gloo"


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


def ep_dispatch() -> str:
    """EP form: "allreduce" (experts sharded, tokens replicated, the layer all-reduce sums)
    or "all_to_all" (token slices dispatched to the expert owners,
    parallel/expert_parallel.py).  --expert-parallel-dispatch / EIA_EP_DISPATCH."""
    v = os.environ.get("EIA_EP_DISPATCH", "allreduce")
    return v if v in ("allreduce", "all_to_all") else "allreduce"


def is_driver() -> bool:
    """Rank 0 of its model replica (owns the scheduler)."""
    return _TP_RANK == 0 and _PP_RANK == 0


def pp_rank() -> int:
    return _PP_RANK


def pp_size() -> int:
    return _PP_SIZE


def is_first_stage() -> bool:
    return _PP_RANK == 0


def is_last_stage() -> bool:
    return _PP_RANK == _PP_SIZE - 1


def pp_prev_rank() -> int:
    return _PP_RANKS[_PP_RANK - 1]


def pp_next_rank() -> int:
    return _PP_RANKS[_PP_RANK + 1]


def replica_ranks() -> List[int]:
    return list(_REPLICA_RANKS)


def replica_cpu_group() -> Optional[dist.ProcessGroup]:
    return _REPLICA_CPU_GROUP


def stage_layer_range(num_layers: int, stage: Optional[int] = None,
                      stages: Optional[int] = None) -> "tuple[int, int]":
    """Contiguous layer range of a pipeline stage; the remainder goes to the first stages."""
    stage = _PP_RANK if stage is None else stage
    stages = _PP_SIZE if stages is None else stages
    base, rem = divmod(num_layers, stages)
    start = stage * base + min(stage, rem)
    return start, start + base + (1 if stage < rem else 0)


def set_tp_for_testing(rank: int, size: int) -> None:
    """Pretend to be TP rank `rank` of `size` without communication (weight-sharding tests)."""
    global _TP_RANK, _TP_SIZE
    _TP_RANK, _TP_SIZE = rank, size
