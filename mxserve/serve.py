"""Single-process serving: frontend + in-process engine on one port.

    python -m mxserve.serve --model meta-llama/Llama-3.2-1B-Instruct --port 8000
"""
from __future__ import annotations

import sys


def main(argv=None) -> None:
    from .frontend.__main__ import main as fe_main
    argv = list(sys.argv[1:] if argv is None else argv)
    out = []
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ("--model", "--model-path"):
            out += ["--local-model", argv[i + 1]]
            i += 2
        elif a == "--port":
            out += ["--http-port", argv[i + 1]]
            i += 2
        elif a == "--device":
            out += ["--local-device", argv[i + 1]]
            i += 2
        else:
            out.append(a)
            i += 1
    fe_main(out)


if __name__ == "__main__":
    main()
