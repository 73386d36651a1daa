"""Chat templates.  A model directory with weights (HF_HOME / the model-cache PVC,
examples/dgdr/trtllm/disagg_cache.yaml:29-34) ships its own Jinja template in
tokenizer_config.json (`chat_template`, a string or a list of named templates): that one is
rendered in a sandboxed Jinja environment, as HF `apply_chat_template(..., add_generation_prompt=
True)` does.  Without one (random-init serving on the GPU box) the built-in renderers below --
Llama-3, ChatML (Qwen3) and Mistral [INST] -- produce the same text for plain-text messages."""
from __future__ import annotations

import functools
import json
import os
from typing import Optional


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


@functools.lru_cache(maxsize=16)
def load_hf_template(model_dir: Optional[str]) -> Optional[tuple]:
    """(jinja template source, special tokens) from <model_dir>/tokenizer_config.json, or None."""
    if not model_dir:
        return None
    path = os.path.join(model_dir, "tokenizer_config.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        cfg = json.load(f)
    tpl = cfg.get("chat_template")
    if isinstance(tpl, list):  # [{"name": "default", "template": ...}, {"name": "tool_use", ...}]
        named = {t.get("name"): t.get("template") for t in tpl if isinstance(t, dict)}
        tpl = named.get("default") or next(iter(named.values()), None)
    if not tpl:
        return None

    def tok(k):
        v = cfg.get(k)
        return v.get("content") if isinstance(v, dict) else v
    return tpl, {"bos_token": tok("bos_token") or "", "eos_token": tok("eos_token") or ""}


@functools.lru_cache(maxsize=16)
def _compile(source: str):
    from jinja2.sandbox import ImmutableSandboxedEnvironment

    def raise_exception(msg):
        raise ValueError(msg)
    env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)
    env.globals["raise_exception"] = raise_exception
    env.filters["tojson"] = lambda x, indent=None, **kw: json.dumps(x, indent=indent, ensure_ascii=False)
    return env.from_string(source)


def render_jinja(source: str, messages: list[dict], special: dict, add_generation_prompt: bool = True) -> str:
    from jinja2 import TemplateError
    try:
        return _compile(source).render(messages=messages, add_generation_prompt=add_generation_prompt, **special)
    except TemplateError as e:
        raise ValueError(f"chat template error: {e}") from e


def render(template: str, messages: list[dict], model_dir: Optional[str] = None) -> str:
    if not isinstance(messages, list) or not messages:
        raise ValueError("messages must be a non-empty list")
    for m in messages:
        if not isinstance(m, dict) or "role" not in m:
            raise ValueError("each message needs a role")
    hf = load_hf_template(model_dir)
    if hf is not None:
        return render_jinja(hf[0], messages, hf[1])
    return _TEMPLATES.get(template, render_llama3)(messages)
