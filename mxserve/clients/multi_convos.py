"""Parallel multi-turn load test behind `multi_convos_parallel.sh` (reference
examples/dgdr/trtllm/multi_convos_parallel.sh:4-176): NUM_CONVOS conversations of 3 turns
(system + user, then two follow-ups), at most CONCURRENCY in flight, transcripts printed in order,
exit status 1 if any request failed."""
from __future__ import annotations

import os
import sys
from concurrent.futures import ThreadPoolExecutor

from .openai_client import APIError, chat

FOLLOW_UPS = ("Now explain that fun fact in 2 sentences.", "Thanks! End with a one-line summary.")


def run_convo(cid: int, api_url: str, model: str, temperature: float, max_tokens: int) -> tuple[bool, str]:
    msgs = [{"role": "system", "content": "You are a helpful assistant."},
            {"role": "user", "content": f"Conversation {cid}: Give me a short fun fact about Denmark."}]
    ok = True
    err = ""
    try:
        for turn in range(3):
            if turn:
                msgs.append({"role": "user", "content": FOLLOW_UPS[turn - 1]})
            msgs.append({"role": "assistant", "content": chat(api_url, model, msgs, temperature, max_tokens)})
    except APIError as e:
        ok = False
        err = f"API error: {e}\n"
    bar = "=" * 30
    body = "".join(f"{m['role'].upper()}: {m['content']}\n\n" for m in msgs)
    return ok, f"{bar}\n Transcript: Conversation {cid}\n{bar}\n{err}{body}"


def main() -> int:
    api_url = os.environ.get("API_URL", "http://localhost:8000/v1/chat/completions")
    model = os.environ.get("MODEL", "Qwen/Qwen3-0.6B")
    temperature = float(os.environ.get("TEMPERATURE", "0.7"))
    max_tokens = int(os.environ.get("MAX_TOKENS", "200"))
    n = int(os.environ.get("NUM_CONVOS", "10"))
    conc = int(os.environ.get("CONCURRENCY", "5"))
    print(f"API_URL={api_url}\nMODEL={model}\nNUM_CONVOS={n}\nCONCURRENCY={conc}\n", flush=True)
    with ThreadPoolExecutor(max_workers=max(1, conc)) as ex:
        results = list(ex.map(lambda c: run_convo(c, api_url, model, temperature, max_tokens), range(1, n + 1)))
    for _, text in results:
        print("\n" + text, end="")
    if all(ok for ok, _ in results):
        print("\nDone.")
        return 0
    print("\nDone (with some failures). See logs above.")
    return 1


if __name__ == "__main__":
    sys.exit(main())
