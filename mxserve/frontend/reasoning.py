"""Reasoning parsers: split a chat completion's `<think>...</think>` block into the OpenAI-style
`reasoning_content` field, so clients get the final answer in `content` (what chat.sh extracts
by hand, chat.sh:37-82).  Dynamo's frontend does this with `--dyn-reasoning-parser`.

  qwen3 / basic   reasoning only inside an explicit <think> ... </think>
  deepseek_r1     the completion starts in reasoning mode (the template opened <think>), until </think>

Streaming-safe: text that could be the start of a tag is held back until it is disambiguated.
"""
from __future__ import annotations

from typing import Optional

PARSERS = ("qwen3", "basic", "deepseek_r1")
_OPEN, _CLOSE = "<think>", "</think>"


class ReasoningSplitter:
    def __init__(self, parser: str):
        if parser not in PARSERS:
            raise ValueError(f"reasoning parser must be one of {PARSERS}, got {parser!r}")
        self.in_reasoning = parser == "deepseek_r1"
        self._buf = ""

    @staticmethod
    def _partial_tag_len(text: str, tag: str) -> int:
        """Length of the longest suffix of `text` that is a proper prefix of `tag`."""
        for n in range(min(len(tag) - 1, len(text)), 0, -1):
            if text.endswith(tag[:n]):
                return n
        return 0

    def feed(self, text: str, final: bool = False) -> tuple[str, str]:
        """Returns (reasoning_delta, content_delta) for this chunk of generated text."""
        self._buf += text
        reasoning, content = [], []
        while True:
            tag = _CLOSE if self.in_reasoning else _OPEN
            i = self._buf.find(tag)
            if i < 0:
                keep = 0 if final else self._partial_tag_len(self._buf, tag)
                out, self._buf = self._buf[:len(self._buf) - keep], self._buf[len(self._buf) - keep:]
                (reasoning if self.in_reasoning else content).append(out)
                break
            (reasoning if self.in_reasoning else content).append(self._buf[:i])
            self._buf = self._buf[i + len(tag):]
            self.in_reasoning = not self.in_reasoning
        return "".join(reasoning), "".join(content)


def split_text(text: str, parser: Optional[str]) -> tuple[Optional[str], str]:
    """Whole-text split for unary responses: (reasoning_content or None, content)."""
    if not parser:
        return None, text
    sp = ReasoningSplitter(parser)
    started = sp.in_reasoning or _OPEN in text
    r, c = sp.feed(text, final=True)
    return (r.strip("\n") if started else None), c.lstrip("\n")
