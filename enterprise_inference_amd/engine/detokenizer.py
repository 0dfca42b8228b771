"""Incremental detokenisation + stop-string handling for streaming outputs."""

from __future__ import annotations

from typing import List, Optional, Tuple

from .sequence import Sequence


class Detokenizer:
    def __init__(self, tokenizer):
        self.tok = tokenizer
        self._byte_level = tokenizer.__class__.__name__ == "ByteTokenizer"

    def step(self, seq: Sequence) -> str:
        """Decode newly generated tokens of `seq`; returns the new text (may be '')."""
        ids = seq.output_token_ids
        skip = seq.params.skip_special_tokens
        if self._byte_level:
            new = self.tok.decode(ids[seq.read_offset:], skip_special_tokens=skip)
            # hold back an incomplete UTF-8 tail
            if new.endswith("�"):
                return ""
            seq.read_offset = len(ids)
            seq.output_text += new
            return new
        # generic HF path: decode a sliding window and diff (handles merges / byte fallback)
        prefix = self.tok.decode(ids[seq.prefix_offset:seq.read_offset], skip_special_tokens=skip)
        full = self.tok.decode(ids[seq.prefix_offset:], skip_special_tokens=skip)
        if len(full) > len(prefix) and not full.endswith("�"):
            new = full[len(prefix):]
            seq.prefix_offset = seq.read_offset
            seq.read_offset = len(ids)
            seq.output_text += new
            return new
        return ""

    @staticmethod
    def check_stop_strings(seq: Sequence, new_text: str) -> Optional[Tuple[str, int]]:
        """If a stop string appeared, truncate output_text; returns (stop, removed_chars)."""
        stops = seq.params.stop
        if not stops or not new_text:
            return None
        text = seq.output_text
        window_start = max(0, len(text) - len(new_text) - max(len(s) for s in stops) + 1)
        for s in stops:
            idx = text.find(s, window_start)
            if idx >= 0:
                cut = idx + (len(s) if seq.params.include_stop_str_in_output else 0)
                removed = len(text) - cut
                seq.output_text = text[:cut]
                return s, removed
        return None
