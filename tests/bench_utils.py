"""Helpers for tests that launch bench.py: every launch runs in a session of its own, a timeout
kills that whole process group, and a tag in the environment finds any process left behind."""
from __future__ import annotations

import os
import signal
import subprocess
import time
import uuid


class Result:
    def __init__(self, returncode: int, stdout: str, stderr: str, wall_s: float):
        self.returncode, self.stdout, self.stderr, self.wall_s = returncode, stdout, stderr, wall_s


def run_group(cmd: list, timeout: float, **kw) -> Result:
    """subprocess.run with the child in a new session: on timeout the whole group is SIGKILLed
    (torchrun, its ranks) instead of orphaning them; raises AssertionError then."""
    t0 = time.time()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True, **kw)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        out, err = p.communicate()
        raise AssertionError(f"timed out after {timeout}s; stderr tail:\n{err[-3000:]}")
    return Result(p.returncode, out, err, time.time() - t0)


def new_tag() -> str:
    return uuid.uuid4().hex


def tagged_pids(tag: str) -> list:
    """PIDs of live processes whose environment carries MXS_TEST_TAG=tag."""
    import psutil
    out = []
    for pr in psutil.process_iter(["pid"]):
        try:
            if pr.environ().get("MXS_TEST_TAG") == tag and pr.status() != psutil.STATUS_ZOMBIE:
                out.append(pr.pid)
        except (psutil.NoSuchProcess, psutil.AccessDenied, psutil.ZombieProcess):
            continue
    return out


def wait_gone(tag: str, timeout: float) -> list:
    t_end = time.time() + timeout
    left = tagged_pids(tag)
    while left and time.time() < t_end:
        time.sleep(0.5)
        left = tagged_pids(tag)
    return left
