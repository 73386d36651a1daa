#!/usr/bin/env python3
"""Run mxserve.tools.mgpu_probe as N ranks (all sections unless MXS_PROBE_SECTIONS), the way bench.py
runs it after its serving phases, and print rank 0's PROBE line.  argv: N [timeout_s]."""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    n = int(sys.argv[1])
    timeout = float(sys.argv[2]) if len(sys.argv) > 2 else 600.0
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    t0 = time.time()
    env0 = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env0.pop("MXS_PROBE_DISAGG_ARGV", None)
    procs = []
    for r in range(n):
        env = dict(env0, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), LOCAL_RANK=str(r),
                   WORLD_SIZE=str(n), PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0",
                   MXS_PROBE_DEADLINE=repr(t0 + timeout - 30), MXS_PROBE_TIMEOUT_S=repr(timeout - 60))
        procs.append(subprocess.Popen([sys.executable, "-m", "mxserve.tools.mgpu_probe"], stdin=subprocess.PIPE,
                                      stdout=subprocess.PIPE, env=env, cwd=ROOT, start_new_session=True))
    for p in procs:
        p.stdin.write(b"go\n")
        p.stdin.close()
        p.stdin = None
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=max(1.0, t0 + timeout - time.time()))[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    lines = [ln for ln in outs[0].decode(errors="replace").splitlines() if ln.startswith("PROBE ")] if outs else []
    res = json.loads(lines[-1][len("PROBE "):]) if lines else {"status": "failed", "error": "no PROBE line"}
    res["returncodes"] = [p.returncode for p in procs]
    res["runner_wall_s"] = round(time.time() - t0, 1)
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
