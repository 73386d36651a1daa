"""Tiny synchronous OpenAI-compatible client (stdlib only, so the scripts need no extra deps)."""
from __future__ import annotations

import json
import urllib.error
import urllib.request


class APIError(RuntimeError):
    pass


def chat(api_url: str, model: str, messages: list, temperature: float, max_tokens: int,
         timeout: float = 600.0, **extra) -> str:
    """POST a chat completion; returns choices[0].message.content or raises APIError with the
    server's `.error.message`."""
    body = dict(model=model, messages=messages, temperature=temperature, max_tokens=max_tokens, **extra)
    req = urllib.request.Request(api_url, data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json", "Authorization": "Bearer dummy"})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            payload = json.loads(r.read().decode() or "{}")
    except urllib.error.HTTPError as e:
        try:
            payload = json.loads(e.read().decode() or "{}")
        except ValueError:
            raise APIError(f"HTTP {e.code}") from None
    except urllib.error.URLError as e:
        raise APIError(f"cannot reach {api_url}: {e.reason}") from None
    if "error" in payload:
        err = payload["error"]
        raise APIError(err.get("message", str(err)) if isinstance(err, dict) else str(err))
    try:
        return payload["choices"][0]["message"]["content"] or ""
    except (KeyError, IndexError, TypeError):
        raise APIError(f"unexpected response: {payload!r:.200}") from None
