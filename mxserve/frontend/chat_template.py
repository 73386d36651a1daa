"""Chat templates rendered natively (no Jinja needed on the GPU box): Llama-3, ChatML (Qwen3) and
Mistral [INST].  Output matches the public HF chat templates for plain-text messages with
add_generation_prompt=True."""
from __future__ import annotations


def _content(m: dict) -> str:
    c = m.get("content", "")
    if isinstance(c, list):  # OpenAI content parts
        return "".join(p.get("text", "") for p in c if isinstance(p, dict) and p.get("type", "text") == "text")
    return "" if c is None else str(c)


def render_llama3(messages: list[dict]) -> str:
    out = ["<|begin_of_text|>"]
    for m in messages:
        out.append(f"<|start_header_id|>{m.get('role', 'user')}<|end_header_id|>\n\n{_content(m).strip()}<|eot_id|>")
    out.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
    return "".join(out)


def render_chatml(messages: list[dict]) -> str:
    out = []
    for m in messages:
        out.append(f"<|im_start|>{m.get('role', 'user')}\n{_content(m)}<|im_end|>\n")
    out.append("<|im_start|>assistant\n")
    return "".join(out)


def render_mistral(messages: list[dict]) -> str:
    out = ["<s>"]
    system = ""
    for m in messages:
        role = m.get("role", "user")
        if role == "system":
            system = _content(m) + "\n\n"
        elif role == "user":
            out.append(f"[INST] {system}{_content(m)} [/INST]")
            system = ""
        else:
            out.append(f" {_content(m)}</s>")
    return "".join(out)


_TEMPLATES = {"llama3": render_llama3, "chatml": render_chatml, "mistral": render_mistral}


def render(template: str, messages: list[dict]) -> str:
    if not isinstance(messages, list) or not messages:
        raise ValueError("messages must be a non-empty list")
    for m in messages:
        if not isinstance(m, dict) or "role" not in m:
            raise ValueError("each message needs a role")
    return _TEMPLATES.get(template, render_llama3)(messages)
