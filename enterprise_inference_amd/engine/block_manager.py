"""Thin Python facade over the native KVCacheManager (csrc/runtime/kv_manager.cpp)."""

from __future__ import annotations

import numpy as np

from .. import _native
from .sequence import Sequence


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int, prefix_caching: bool = True):
        rt = _native.runtime()
        self.native = rt.KVCacheManager(num_blocks, block_size, prefix_caching)
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.prefix_caching = prefix_caching
        self._committed = {}   # seq_id -> full blocks already hashed

    @staticmethod
    def _toks(seq: Sequence) -> np.ndarray:
        return np.asarray(seq.all_token_ids, dtype=np.int32)

    def has(self, seq: Sequence) -> bool:
        return self.native.has_seq(seq.seq_id)

    def allocate_prefix(self, seq: Sequence) -> int:
        return self.native.allocate_prefix(seq.seq_id, self._toks(seq),
                                           getattr(seq, "cache_salt", 0) or 0)

    def ensure(self, seq: Sequence, num_tokens: int) -> bool:
        return self.native.ensure(seq.seq_id, num_tokens)

    def commit(self, seq: Sequence) -> None:
        if not self.prefix_caching:
            return
        nfull = seq.num_computed_tokens // self.block_size
        if nfull > self._committed.get(seq.seq_id, 0):
            toks = np.asarray(seq.all_token_ids[: nfull * self.block_size], dtype=np.int32)
            self.native.commit(seq.seq_id, toks, nfull * self.block_size,
                               getattr(seq, "cache_salt", 0) or 0)
            self._committed[seq.seq_id] = nfull

    def free(self, seq: Sequence) -> None:
        self.native.free(seq.seq_id)
        self._committed.pop(seq.seq_id, None)

    def block_table(self, seq: Sequence):
        return self.native.block_table(seq.seq_id)

    def usage(self) -> float:
        return self.native.usage()

    def num_free_blocks(self) -> int:
        return self.native.num_free_blocks()

    def reset_prefix_cache(self) -> None:
        self.native.reset_prefix_cache()

    def check_invariants(self) -> str:
        return self.native.check_invariants()

    def stats(self) -> dict:
        return dict(self.native.stats())
