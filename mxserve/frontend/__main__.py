"""`python -m mxserve.frontend` (also `python -m dynamo.frontend`): the OpenAI HTTP frontend.

Workers register themselves (MXS_FRONTEND_URL); `--local-model` additionally runs an engine inside
the frontend process (single-process serving, no request-plane hop)."""
from __future__ import annotations

import argparse
import logging
import os


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m dynamo.frontend")
    ap.add_argument("--http-host", default=os.environ.get("DYN_HTTP_HOST", "0.0.0.0"))
    ap.add_argument("--http-port", type=int, default=int(os.environ.get("DYN_HTTP_PORT", "8000")))
    ap.add_argument("--router-mode", choices=["round_robin", "random", "kv"],
                    default=os.environ.get("DYN_ROUTER_MODE", "kv"))
    ap.add_argument("--lease-ttl", type=float, default=float(os.environ.get("MXS_LEASE_TTL", "10")))
    ap.add_argument("--namespace", default=os.environ.get("DYN_NAMESPACE", "default"))
    ap.add_argument("--reasoning-parser", "--dyn-reasoning-parser", dest="reasoning_parser",
                    choices=["qwen3", "basic", "deepseek_r1"], default=os.environ.get("MXS_REASONING_PARSER"),
                    help="split <think> blocks of chat completions into message.reasoning_content")
    ap.add_argument("--local-model", default=os.environ.get("MXS_LOCAL_MODEL"),
                    help="also serve this model from an in-process engine")
    ap.add_argument("--local-device", default=os.environ.get("MXS_LOCAL_DEVICE", "auto"))
    ap.add_argument("--num-procs", type=int, default=int(os.environ.get("MXS_FRONTEND_PROCS", "1")),
                    help="frontend processes sharing the port (SO_REUSEPORT); >1 spreads the per-token "
                         "streaming work over cores (frontend/multiproc.py)")
    return ap


def main(argv=None) -> None:
    from .app import Frontend, serve_app
    a = build_parser().parse_args(argv)
    from ..utils.logs import setup_logging
    setup_logging()
    if a.num_procs > 1:
        if a.local_model:
            raise SystemExit("--local-model runs the engine in the frontend process: use --num-procs 1")
        from .multiproc import serve
        raise SystemExit(serve({"host": a.http_host, "port": a.http_port, "router_mode": a.router_mode,
                                "ttl": a.lease_ttl, "namespace": a.namespace,
                                "reasoning_parser": a.reasoning_parser}, a.num_procs))
    fe = Frontend(router_mode=a.router_mode, ttl=a.lease_ttl, namespace=a.namespace,
                  reasoning_parser=a.reasoning_parser)
    if a.local_model:
        from ..config import EngineArgs, env_overrides
        from ..engine.engine import AsyncEngine, LLMEngine
        kw = env_overrides()
        kw.update(model=a.local_model, device=a.local_device)
        eng = LLMEngine(EngineArgs(**kw))
        fe.add_local_worker(AsyncEngine(eng), eng.args.name, eng.runner.num_blocks)
    serve_app(fe, host=a.http_host, port=a.http_port)


if __name__ == "__main__":
    main()
