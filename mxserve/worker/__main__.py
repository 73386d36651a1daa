"""`python -m mxserve.worker [--dialect vllm|sglang|trtllm] <engine flags>`."""
from __future__ import annotations

import sys


def main(argv=None, dialect: str = "vllm") -> None:
    from .args import parse_worker_args
    from .server import serve
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv[:1] == ["--dialect"]:
        dialect, argv = argv[1], argv[2:]
    serve(parse_worker_args(argv, dialect))


if __name__ == "__main__":
    main()
