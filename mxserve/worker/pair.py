"""P/D pair pod launcher: one decode worker and one prefill worker in ONE container that holds both
groups of GPUs (cross-pod caveat, mitigation #1).

The reference runs prefill and decode as separate services with `gpu: "1"` each
(examples/deploy/vllm/disagg.yaml:18-57, sglang/disagg.yaml:18-87).  On MI355X the prompt's KV moves
prefill -> decode by IPC-mapping the decode GPU's staging arena (hipIpcOpenMemHandle) and pushing
over xGMI; that needs both processes to see both GPUs, which two pods that each own one GPU do not.
So the operator renders every decode replica of a graph that also has a prefill service as a pair
pod: `amd.com/gpu: <decode tp> + <prefill tp>`, this launcher as the command, and the two services'
own commands in MXS_PAIR_DECODE_CMD / MXS_PAIR_PREFILL_CMD.

  decode   GPUs [0, tp_d), port DYN_SYSTEM_PORT (the pod's readiness / metrics port)
  prefill  GPUs [tp_d, tp_d + tp_p), port DYN_SYSTEM_PORT + 1
Both register with the frontend under the same pair id (the pod name), and the frontend hands a
decode worker a prefill worker of its own pair first.  /dev/shm is shared too, so the host-staged
fallback is the shm arena, not HTTP.  The launcher forwards SIGTERM and exits with the first child
that exits (k8s then restarts the whole pair).
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


def child_envs(base: dict, decode_cmd: list, prefill_cmd: list) -> tuple:
    port = int(base.get("DYN_SYSTEM_PORT", base.get("MXS_WORKER_PORT", "8081")))
    pair = base.get("MXS_PAIR_ID") or base.get("POD_NAME") or socket.gethostname()
    tp_d = _tp_of(decode_cmd)
    common = dict(base, MXS_PAIR_ID=pair, HSA_ENABLE_IPC_MODE_LEGACY=base.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    dec = dict(common, MXS_DEVICE_OFFSET="0", DYN_SYSTEM_PORT=str(port), MXS_WORKER_ID=f"decode-{pair}")
    pre = dict(common, MXS_DEVICE_OFFSET=str(tp_d), DYN_SYSTEM_PORT=str(port + 1), MXS_WORKER_ID=f"prefill-{pair}")
    return dec, pre


def main() -> int:
    decode_cmd = json.loads(os.environ["MXS_PAIR_DECODE_CMD"])
    prefill_cmd = json.loads(os.environ["MXS_PAIR_PREFILL_CMD"])
    dec_env, pre_env = child_envs(dict(os.environ), decode_cmd, prefill_cmd)
    procs = [subprocess.Popen(decode_cmd, env=dec_env), subprocess.Popen(prefill_cmd, env=pre_env)]

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
