#!/usr/bin/env python3
"""Which processes have the GPU open (/dev/kfd or a /dev/dri render node), sampled every `every`
seconds while a command runs: argv every_s out_file -- command...  (The pool's process guard
allows 16 per GPU; bench.py --gpus N puts N ranks + N probe processes on every GPU of a node.)"""
import json
import os
import subprocess
import sys
import time


def census() -> list:
    rows = []
    for pid in os.listdir("/proc"):
        if not pid.isdigit():
            continue
        try:
            fds = os.listdir(f"/proc/{pid}/fd")
        except OSError:
            continue
        gpu = False
        for fd in fds:
            try:
                t = os.readlink(f"/proc/{pid}/fd/{fd}")
            except OSError:
                continue
            if t == "/dev/kfd" or t.startswith("/dev/dri/render"):
                gpu = True
                break
        if not gpu:
            continue
        try:
            cmd = open(f"/proc/{pid}/cmdline", "rb").read().replace(b"\0", b" ").decode(errors="replace")[:160]
            ppid = int(open(f"/proc/{pid}/stat").read().split(")")[1].split()[1])
        except OSError:
            continue
        rows.append({"pid": int(pid), "ppid": ppid, "cmd": cmd})
    return rows


def main() -> int:
    every, out = float(sys.argv[1]), sys.argv[2]
    cmd = sys.argv[sys.argv.index("--") + 1:]
    p = subprocess.Popen(cmd)
    with open(out, "w") as f:
        while p.poll() is None:
            time.sleep(every)
            rows = census()
            f.write(json.dumps({"t": round(time.time(), 1), "n": len(rows), "procs": rows}) + "\n")
            f.flush()
    return p.returncode


if __name__ == "__main__":
    sys.exit(main())
