"""Tokenizers for the preprocessor.

* HFTokenizer: a real `tokenizer.json` found on disk (HF_HOME / model dir) via the installed Rust
  `tokenizers` library.
* ByteTokenizer: self-contained fallback for the offline GPU box / random-init weights.  UTF-8
  bytes map to ids [BYTE0, BYTE0 + 256), chat-template special tokens map to the model's real
  special ids (Llama-3 / ChatML / Mistral), and any other id (random weights produce arbitrary
  ids) decodes to a deterministic pseudo-word so streamed text stays readable.
Both expose encode / decode / an incremental detokenizer used for streaming.
"""
from __future__ import annotations

import os
from typing import Optional

from ..models.config import ModelConfig, find_local_model_dir

BYTE0 = 3

_SPECIALS = {
    "llama3": {"<|begin_of_text|>": 128000, "<|end_of_text|>": 128001, "<|start_header_id|>": 128006,
               "<|end_header_id|>": 128007, "<|eom_id|>": 128008, "<|eot_id|>": 128009},
    "chatml": {"<|endoftext|>": 151643, "<|im_start|>": 151644, "<|im_end|>": 151645, "<think>": 151667,
               "</think>": 151668},
    "mistral": {"<s>": 1, "</s>": 2, "[INST]": 3, "[/INST]": 4},
}

_SYL = ["ka", "lo", "mi", "ne", "ru", "sa", "ti", "vo", "ze", "an", "el", "or", "um", "is", "ya", "po"]


class ByteTokenizer:
    def __init__(self, cfg: ModelConfig):
        self.vocab_size = cfg.vocab_size
        specials = dict(_SPECIALS.get(cfg.chat_template, {}))
        # keep only specials that fit the vocab (tiny test models)
        self.special_to_id = {k: v for k, v in specials.items() if v < cfg.vocab_size}
        self.id_to_special = {v: k for k, v in self.special_to_id.items()}
        self.byte0 = BYTE0 if cfg.chat_template != "mistral" else 8
        self.eos_token_ids = list(cfg.eos_token_ids)
        self.bos_token_id = cfg.bos_token_id
        self._sorted_specials = sorted(self.special_to_id, key=len, reverse=True)
        self._pieces: dict = {}

    def encode(self, text: str, add_special_tokens: bool = False) -> list[int]:
        ids: list[int] = []
        if add_special_tokens and self.bos_token_id is not None:
            ids.append(self.bos_token_id)
        i = 0
        n = len(text)
        while i < n:
            if text[i] in "<[":
                hit = next((s for s in self._sorted_specials if text.startswith(s, i)), None)
                if hit is not None:
                    ids.append(self.special_to_id[hit])
                    i += len(hit)
                    continue
            j = i
            while j < n and text[j] not in "<[":
                j += 1
            if j == i:
                j = i + 1
            ids.extend(self.byte0 + b for b in text[i:j].encode("utf-8"))
            i = j
        return ids

    def _piece(self, t: int, skip_special: bool) -> bytes:
        p = self._pieces.get((t, skip_special))
        if p is None:
            p = self._pieces[(t, skip_special)] = self._make_piece(t, skip_special)
            if len(self._pieces) > 1 << 18:
                self._pieces.clear()
        return p

    def _make_piece(self, t: int, skip_special: bool) -> bytes:
        if self.byte0 <= t < self.byte0 + 256:
            return bytes([t - self.byte0])
        if t in self.id_to_special:
            return b"" if skip_special else self.id_to_special[t].encode()
        if t < self.byte0:
            return b""
        # deterministic pseudo-word for ids outside the byte range
        x = (t * 2654435761) & 0xFFFFFFFF
        w = _SYL[x & 15] + _SYL[(x >> 4) & 15] + (_SYL[(x >> 8) & 15] if x & 0x1000 else "")
        return (" " + w).encode()

    def decode(self, ids: list[int], skip_special_tokens: bool = True) -> str:
        piece = self._piece
        return b"".join([piece(t, skip_special_tokens) for t in ids]).decode("utf-8", errors="replace")

    def piece_bytes(self, t: int, skip_special_tokens: bool = True) -> bytes:
        """The bytes of one id, independent of its neighbours (what makes an O(1) incremental
        decode exact for this tokenizer: IncrementalDetokenizer's byte mode)."""
        return self._piece(t, skip_special_tokens)

    def convert_special(self, name: str) -> Optional[int]:
        return self.special_to_id.get(name)


class HFTokenizer:
    def __init__(self, path: str, cfg: ModelConfig):
        from tokenizers import Tokenizer
        self.tok = Tokenizer.from_file(path)
        self.vocab_size = self.tok.get_vocab_size()
        self.eos_token_ids = list(cfg.eos_token_ids)
        self.bos_token_id = cfg.bos_token_id

    def encode(self, text: str, add_special_tokens: bool = False) -> list[int]:
        return self.tok.encode(text, add_special_tokens=add_special_tokens).ids

    def decode(self, ids: list[int], skip_special_tokens: bool = True) -> str:
        return self.tok.decode(list(ids), skip_special_tokens=skip_special_tokens)

    def convert_special(self, name: str) -> Optional[int]:
        return self.tok.token_to_id(name)


def load_tokenizer(cfg: ModelConfig, tokenizer_path: Optional[str] = None):
    path = tokenizer_path
    if path is None:
        d = find_local_model_dir(cfg.name)
        if d is not None and os.path.exists(os.path.join(d, "tokenizer.json")):
            path = os.path.join(d, "tokenizer.json")
    if path and os.path.exists(path):
        return HFTokenizer(path, cfg)
    return ByteTokenizer(cfg)


class IncrementalDetokenizer:
    """Streams text deltas in O(1) work per token: each step decodes only a short window of ids
    (from `prefix` to the end), not the whole output -- a full re-decode per token is O(n^2) over a
    500-token answer, ~10^5 tokens decoded per request at OSL 500.  The window starts a few tokens
    back so byte-fallback / leading-space merges resolve as in a full decode; an incomplete UTF-8
    sequence (U+FFFD at the tail) is held back until its next byte arrives.  The window start stays
    put for up to WINDOW tokens, so the text of [prefix, read) is the previous step's decode: one
    tokenizer call per token instead of two."""

    WINDOW = 8

    def __init__(self, tokenizer, prompt_tail: Optional[list] = None, skip_special_tokens: bool = True):
        self.tok = tokenizer
        self.skip = skip_special_tokens
        self.ids: list[int] = list(prompt_tail or [])[-5:]
        self.prefix = 0  # window start
        self.read = len(self.ids)  # end of the text already emitted
        self._ptext: Optional[str] = None  # decode of ids[prefix:read], when known
        # tokenizers whose ids map to context-free byte strings: an incremental UTF-8 decoder is
        # the exact full decode, at one dict lookup per token (no window)
        self._piece = getattr(tokenizer, "piece_bytes", None)
        if self._piece is not None:
            import codecs
            self._utf8 = codecs.getincrementaldecoder("utf-8")("replace")

    def _decode(self, a: int, b: Optional[int] = None) -> str:
        return self.tok.decode(self.ids[a:b], skip_special_tokens=self.skip)

    def add(self, token_id: int) -> str:
        if self._piece is not None:
            return self._utf8.decode(self._piece(int(token_id), self.skip))
        self.ids.append(int(token_id))
        return self._advance()

    def add_many(self, token_ids: list) -> str:
        """A batch of tokens that arrived together: one window decode instead of one per token
        (the same text as adding them one by one)."""
        if not token_ids:
            return ""
        if self._piece is not None:
            return self._utf8.decode(b"".join(self._piece(int(t), self.skip) for t in token_ids))
        self.ids.extend(int(t) for t in token_ids)
        return self._advance()

    def _advance(self) -> str:
        prefix_text = self._ptext if self._ptext is not None else self._decode(self.prefix, self.read)
        new_text = self._decode(self.prefix)
        if len(new_text) <= len(prefix_text) or new_text.endswith("\ufffd"):
            self._ptext = prefix_text
            return ""
        delta = new_text[len(prefix_text):]
        if len(self.ids) - self.prefix > self.WINDOW:  # slide: the text of the new window is not known
            self.prefix, self._ptext = self.read, None
        else:
            self._ptext = new_text
        self.read = len(self.ids)
        return delta

    def flush(self) -> str:
        if self._piece is not None:
            return self._utf8.decode(b"", final=True)
        prefix_text = self._ptext if self._ptext is not None else self._decode(self.prefix, self.read)
        new_text = self._decode(self.prefix)
        delta = new_text[len(prefix_text):] if len(new_text) > len(prefix_text) else ""
        self.prefix = self.read = len(self.ids)
        self._ptext = None
        return delta
