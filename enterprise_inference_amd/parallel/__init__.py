"""Tensor / expert parallelism over RCCL (xGMI) + custom xGMI all-reduce."""
