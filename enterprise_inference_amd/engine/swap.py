"""KV swap space (K14): preempted sequences park their KV blocks in pinned host memory
instead of being recomputed (vLLM ``--swap-space``, reference chart
core/helm-charts/vllm/values.yaml; ``vllm:cpu_cache_usage_perc`` /
``vllm:num_requests_swapped`` metrics).

The host side is a plain block allocator; the copies run in the model runner
(ModelRunner.swap_out / swap_in): one gather kernel over every layer's K and V of the victim's
blocks plus one device->pinned copy out, and the reverse on the way back in -- both on the
step stream ahead of the next step's kernels, so a swapped-out block is read after the
in-flight step that wrote it and a swapped-in block is complete before any kernel reads it.
"""

from __future__ import annotations

from typing import List


class SwapSpace:
    def __init__(self, num_blocks: int):
        self.num_blocks = int(num_blocks)
        self._free: List[int] = list(range(self.num_blocks - 1, -1, -1))

    def can_allocate(self, n: int) -> bool:
        return n <= len(self._free)

    def allocate(self, n: int) -> List[int]:
        if n > len(self._free):
            raise RuntimeError("swap space exhausted")
        return [self._free.pop() for _ in range(n)]

    def free(self, ids: List[int]) -> None:
        self._free.extend(ids)

    def usage(self) -> float:
        return 1.0 - len(self._free) / self.num_blocks if self.num_blocks else 0.0


def swap_blocks_for(num_kv_bytes_per_block: int, swap_space_gb: float) -> int:
    if swap_space_gb <= 0 or num_kv_bytes_per_block <= 0:
        return 0
    return int(swap_space_gb * 2**30 // num_kv_bytes_per_block)
