"""Interactive chat REPL behind `chat.sh` (reference chat.sh:3-147 behaviour):

* history is kept across turns, requests use temperature 0 and max_tokens 512;
* the shown answer is the text after a `FINAL:` line, else the text after the last `</think>`;
* if neither exists, a second "rewrite as a final answer only" request is made and any
  <think>...</think> blocks are stripped from its reply;
* the raw assistant text (not the extracted answer) goes back into the history.
"""
from __future__ import annotations

import os
import re
import sys

from .openai_client import APIError, chat

REPAIR_SYSTEM = ("Rewrite the answer as a final answer only. Do NOT include <think> or any reasoning. "
                 "Output only the final answer text.")


def extract_final(raw: str) -> str:
    lines = raw.splitlines()
    for i, ln in enumerate(lines):
        if ln.startswith("FINAL:"):
            out = [ln[len("FINAL:"):].lstrip()] + lines[i + 1:]
            return "\n".join(x.lstrip() for x in out).strip()
    if "</think>" in raw:
        return raw.rsplit("</think>", 1)[1].strip()
    return ""


def strip_think(text: str) -> str:
    text = re.sub(r"<think>.*?</think>", "", text, flags=re.S)
    text = re.sub(r"<think>.*", "", text, flags=re.S)
    return "\n".join(ln.strip() for ln in text.splitlines() if ln.strip())


def answer(api_url: str, model: str, history: list, user_input: str) -> tuple[str, str]:
    """One REPL turn: returns (shown_final_answer, raw_reply)."""
    raw = chat(api_url, model, history + [{"role": "user", "content": user_input}], 0, 512)
    final = "\n".join(ln for ln in extract_final(raw).splitlines() if ln.strip())
    if not final:
        repair = [{"role": "system", "content": REPAIR_SYSTEM},
                  {"role": "user", "content": f"User question: {user_input}\n\nModel output to rewrite:\n{raw}"}]
        final = strip_think(chat(api_url, model, repair, 0, 512))
    return final or "(no final answer returned)", raw


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    api_url = argv[0] if len(argv) >= 1 else os.environ.get("API_URL", "http://127.0.0.1:8000/v1/chat/completions")
    model = argv[1] if len(argv) >= 2 else os.environ.get("MODEL", "Qwen/Qwen3-0.6B")
    print("Interactive chat (final answers only)\nPress Ctrl+C to exit\n", flush=True)
    history: list = []
    try:
        while True:
            try:
                user = input("You: ")
            except EOFError:
                return 0
            try:
                final, raw = answer(api_url, model, history, user)
            except APIError as e:
                print(f"Assistant: (error: {e})\n", flush=True)
                continue
            print(f"Assistant: {final}\n", flush=True)
            history += [{"role": "user", "content": user}, {"role": "assistant", "content": raw}]
    except KeyboardInterrupt:
        print()
        return 0


if __name__ == "__main__":
    sys.exit(main())
