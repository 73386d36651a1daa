"""P/D group pod launcher: several decode and prefill workers in ONE container that holds all their
GPUs (cross-pod caveat, mitigation #1).

The reference runs prefill and decode as separate services, each scaled by its own `replicas`
(examples/deploy/vllm/disagg.yaml:18-57, sglang/disagg.yaml:18-87).  On MI355X the prompt's KV moves
prefill -> decode by IPC-mapping the decode GPU's staging arena (hipIpcOpenMemHandle) and pushing
over xGMI; that needs both processes to see both GPUs, which two pods that each own one GPU do not.
So the operator packs a graph's prefill and decode workers into group pods (resources.pd_groups:
any P:D ratio, as few pods as fit one node -- 3P+5D is one 8-GPU pod) and runs this launcher with
the workers in MXS_GROUP_SPEC = [{"role": "decode"|"prefill", "cmd": [...], "gpus": n}, ...]:

  worker i   GPUs [sum of the earlier workers' gpus, + its own), port DYN_SYSTEM_PORT + i
             (decode workers first: worker 0's port is the pod's readiness / metrics port)
Every worker registers with the frontend under the same group id (the pod name), and the frontend
hands a decode worker a prefill worker of its own group first.  /dev/shm is shared too, so the
host-staged fallback is the shm arena, not HTTP.  The launcher forwards SIGTERM and exits with the
first child that exits (k8s then restarts the whole group).

The older pair form (MXS_PAIR_DECODE_CMD / MXS_PAIR_PREFILL_CMD: one worker of each role) is still
accepted.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import time


def _tp_of(cmd: list) -> int:
    for flag in ("--tp", "--tensor-parallel-size", "--tp-size"):
        if flag in cmd and cmd.index(flag) + 1 < len(cmd):
            return int(cmd[cmd.index(flag) + 1])
    return 1


def group_envs(base: dict, spec: list) -> list:
    """(cmd, env) of every worker of the group: its GPU offset, port and ids."""
    port = int(base.get("DYN_SYSTEM_PORT", base.get("MXS_WORKER_PORT", "8081")))
    group = base.get("MXS_PAIR_ID") or base.get("POD_NAME") or socket.gethostname()
    common = dict(base, MXS_PAIR_ID=group, HSA_ENABLE_IPC_MODE_LEGACY=base.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    out, off, seen = [], 0, {}
    for i, w in enumerate(spec):
        cmd = [str(c) for c in w["cmd"]]
        gpus = int(w.get("gpus") or _tp_of(cmd))
        role = w["role"]
        k = seen[role] = seen.get(role, -1) + 1
        wid = f"{role}-{group}" + (f"-{k}" if k else "")
        out.append((cmd, dict(common, MXS_DEVICE_OFFSET=str(off), DYN_SYSTEM_PORT=str(port + i),
                              MXS_WORKER_ID=wid, MXS_STREAM_PORT=str(port + 100 + i))))
        off += gpus
    return out


def child_envs(base: dict, decode_cmd: list, prefill_cmd: list) -> tuple:
    """The pair form: decode GPUs [0, tp_d) on the pod's port, prefill the next GPUs on port + 1."""
    (_, dec), (_, pre) = group_envs(base, [{"role": "decode", "cmd": decode_cmd, "gpus": _tp_of(decode_cmd)},
                                           {"role": "prefill", "cmd": prefill_cmd, "gpus": _tp_of(prefill_cmd)}])
    return dec, pre


def main() -> int:
    if os.environ.get("MXS_GROUP_SPEC"):
        spec = json.loads(os.environ["MXS_GROUP_SPEC"])
    else:
        spec = [{"role": "decode", "cmd": json.loads(os.environ["MXS_PAIR_DECODE_CMD"])},
                {"role": "prefill", "cmd": json.loads(os.environ["MXS_PAIR_PREFILL_CMD"])}]
    procs = [subprocess.Popen(cmd, env=env) for cmd, env in group_envs(dict(os.environ), spec)]

    def stop(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    while True:
        for p in procs:
            rc = p.poll()
            if rc is not None:
                stop(signal.SIGTERM, None)
                deadline = time.time() + 30
                for q in procs:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
                return rc
        time.sleep(0.5)


if __name__ == "__main__":
    sys.exit(main())
