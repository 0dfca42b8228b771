"""Tokenizer loading.

Uses a local HF tokenizer directory when one is given (``--tokenizer`` or the
model dir, the reference mounts it under HF_HOME=/data).  The byte-level
tokenizer below is used only when the caller allows it -- random-init weights
(``--load-format dummy``, the north-star benchmark setting) or a bare
``ModelConfig`` in tests -- so the full serving path (chat templates, streaming
detokenisation, stop strings) still works without a checkpoint.  A real
checkpoint without a loadable tokenizer is an error.
"""

from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional, Union

_SPECIALS = ["<pad>", "<s>", "</s>"]
_BYTE_OFFSET = 3


class ByteTokenizer:
    """ids: 0 pad, 1 bos, 2 eos, 3..258 = UTF-8 bytes, >=259 = filler letters."""

    is_fast = True

    def __init__(self, vocab_size: int = 32000, eos_token_id: Optional[int] = None,
                 bos_token_id: Optional[int] = None, name: str = "byte-level"):
        self.vocab_size = max(vocab_size, 259)
        self.pad_token_id = 0
        self.bos_token_id = 1 if bos_token_id is None or bos_token_id >= self.vocab_size else bos_token_id
        self.eos_token_id = 2 if eos_token_id is None or eos_token_id >= self.vocab_size else eos_token_id
        self.name_or_path = name
        self.chat_template = None
        self.all_special_ids = sorted({self.pad_token_id, self.bos_token_id, self.eos_token_id})

    def __len__(self) -> int:
        return self.vocab_size

    def encode(self, text: str, add_special_tokens: bool = True) -> List[int]:
        ids = [b + _BYTE_OFFSET for b in text.encode("utf-8")]
        return ([self.bos_token_id] + ids) if add_special_tokens else ids

    def __call__(self, text, add_special_tokens=True, **_):
        if isinstance(text, list):
            return {"input_ids": [self.encode(t, add_special_tokens) for t in text]}
        return {"input_ids": self.encode(text, add_special_tokens)}

    def _tok_bytes(self, i: int) -> bytes:
        if i < _BYTE_OFFSET:
            return _SPECIALS[i].encode() if i < len(_SPECIALS) else b""
        if i < 256 + _BYTE_OFFSET:
            return bytes([i - _BYTE_OFFSET])
        return bytes([97 + (i % 26)])

    def decode(self, ids: List[int], skip_special_tokens: bool = True, **_) -> str:
        out = bytearray()
        for i in ids:
            if skip_special_tokens and i in self.all_special_ids:
                continue
            out += self._tok_bytes(int(i))
        return out.decode("utf-8", errors="replace")

    def convert_ids_to_tokens(self, ids):
        if isinstance(ids, int):
            return self._tok_bytes(ids).decode("latin-1")
        return [self._tok_bytes(i).decode("latin-1") for i in ids]

    def get_vocab(self) -> Dict[str, int]:
        return {f"<0x{b:02X}>": b + _BYTE_OFFSET for b in range(256)}

    def apply_chat_template(self, messages: List[Dict[str, Any]], tools=None,
                            add_generation_prompt: bool = True, tokenize: bool = False,
                            **kwargs) -> Union[str, List[int]]:
        parts = []
        if tools:
            parts.append("<|system|>\nYou can call these tools (JSON):\n" + json.dumps(tools) + "\n")
        for m in messages:
            content = m.get("content")
            if isinstance(content, list):
                content = "".join(c.get("text", "") for c in content if isinstance(c, dict))
            parts.append(f"<|{m.get('role', 'user')}|>\n{content or ''}\n")
        if add_generation_prompt:
            parts.append("<|assistant|>\n")
        text = "".join(parts)
        return self.encode(text, add_special_tokens=True) if tokenize else text


def get_tokenizer(path: Optional[str], vocab_size: int = 32000, eos_token_id=None,
                  bos_token_id=None, trust_remote_code: bool = False,
                  chat_template: Optional[str] = None, allow_byte_fallback: bool = True):
    tok = None
    err = None
    if path and os.path.isdir(path) and any(
            os.path.exists(os.path.join(path, f))
            for f in ("tokenizer.json", "tokenizer.model", "tokenizer_config.json", "vocab.txt")):
        try:
            from transformers import AutoTokenizer

            tok = AutoTokenizer.from_pretrained(path, local_files_only=True,
                                                trust_remote_code=trust_remote_code)
        except Exception as e:   # noqa: BLE001 - byte level only if allowed
            tok, err = None, e
    if tok is None and not allow_byte_fallback:
        raise RuntimeError(f"no loadable tokenizer under {path!r}"
                           + (f": {err!r}" if err else "") +
                           " (pass --tokenizer, or --load-format dummy for random weights)")
    if tok is None:
        eos = eos_token_id[0] if isinstance(eos_token_id, list) else eos_token_id
        tok = ByteTokenizer(vocab_size, eos, bos_token_id, name=path or "byte-level")
    if chat_template:
        if os.path.exists(chat_template):
            with open(chat_template) as f:
                chat_template = f.read()
        try:
            tok.chat_template = chat_template
        except Exception:   # noqa: BLE001
            pass
    return tok
