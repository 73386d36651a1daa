"""bench.py always finishes within its wall budget and leaves nothing behind (VERDICT r2 next-step
#1): the budget arithmetic stays under the driver's 600 s timeout, a hung probe section is cut at
the deadline with the line still printed once, and killing the launcher kills every rank and probe."""
import json
import os
import signal
import subprocess
import sys
import time

import pytest

from tests.bench_utils import new_tag, run_group, tagged_pids, wait_gone

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _base_env(tag: str, **kw) -> dict:
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", MXS_TEST_TAG=tag, **kw)
    return env


def _cpu_args(n: int, *extra: str) -> list:
    return [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "6", "--warmup", "4", "--qps", "8",
            "--device", "cpu", "--gpus", str(n), "--max-warmup-s", "6", "--steady-window-s", "1",
            "--min-ttft-samples", "4", "--iters-per-step", "10", *extra]


def test_budget_arithmetic_under_driver_timeout():
    """Default wall budget + what happens before the deadline clock starts (torchrun start, Python
    start) + the deadline's own exit path stay below 540 s; the probe reports _RESERVE_S ahead."""
    import bench
    a = bench.parse([])
    startup_s, exit_s = 30.0, 20.0  # torchrun + interpreter before bench's clock; watchdog kill + print
    assert a.time_budget_s + startup_s + exit_s <= 540, a.time_budget_s
    assert bench._RESERVE_S >= 10.0  # finish_probe waits until remaining - 10 s: the probe's line comes first
    g = bench.Guard(a.time_budget_s, 0)
    assert abs(g.remaining() - (a.time_budget_s - (time.time() - bench._WALL0))) < 1.0


def test_deadline_cuts_a_hung_probe_section(tmp_path):
    """A probe section that never returns: at the run's deadline rank 0 still prints exactly one
    line (agg numbers, the probe marked partial with the hung section named) and nothing survives."""
    tag = new_tag()
    budget = 75.0
    r = run_group(_cpu_args(2, "--mode", "agg", "--time-budget-s", str(budget)), timeout=budget + 60,
                  cwd=str(tmp_path), env=_base_env(tag, MXS_PROBE_FAULT="hang:collectives"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["n_gpus"] == 2
    pr = d["multi_gpu_probe"]
    assert pr["status"] in ("partial", "failed"), pr
    if pr["status"] == "partial":
        assert pr["timed_out_section"] == "collectives", pr
    assert r.wall_s < budget + 30, r.wall_s
    assert wait_gone(tag, 15) == []


def test_hosted_disagg_hang_keeps_agg_line(tmp_path):
    """The hosted disagg phase hangs (probe section `disagg_headline`): the agg line survives with
    the disagg marked failed, inside the budget."""
    tag = new_tag()
    budget = 80.0
    r = run_group(_cpu_args(2, "--mode", "both", "--time-budget-s", str(budget), "--disagg-qps", "4"),
                  timeout=budget + 60, cwd=str(tmp_path), env=_base_env(tag, MXS_PROBE_FAULT="hang:disagg_headline"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["config"]["mode"] == "both"
    assert d["disagg"]["status"] == "failed", d["disagg"]
    assert r.wall_s < budget + 30, r.wall_s
    assert wait_gone(tag, 15) == []


@pytest.mark.parametrize("victim", ["torchrun", "rank"])
def test_killed_launcher_leaves_no_process(tmp_path, victim):
    """SIGKILL the torchrun launcher (or one rank) mid-run: every rank and probe process exits."""
    import psutil
    tag = new_tag()
    with __import__("socket").socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port)] + _cpu_args(2, "--mode", "agg", "--time-budget-s", "200")[1:]
    p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=str(tmp_path),
                         env=_base_env(tag), start_new_session=True)
    try:
        t_end = time.time() + 90
        probes = []
        while time.time() < t_end:  # wait until both probe processes are up
            probes = [q for q in tagged_pids(tag) if "mgpu_probe" in " ".join(psutil.Process(q).cmdline())]
            if len(probes) >= 2:
                break
            time.sleep(0.5)
        assert len(probes) >= 2, "probe processes never started"
        if victim == "torchrun":
            os.kill(p.pid, signal.SIGKILL)
        else:
            ranks = [q for q in tagged_pids(tag) if q != p.pid and "bench.py" in " ".join(psutil.Process(q).cmdline())]
            os.kill(ranks[0], signal.SIGKILL)
        left = wait_gone(tag, 30)
        assert left == [], [" ".join(psutil.Process(q).cmdline())[:200] for q in left if psutil.pid_exists(q)]
    finally:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        for q in tagged_pids(tag):
            try:
                os.kill(q, signal.SIGKILL)
            except OSError:
                pass


def _ns(**kw):
    import argparse
    d = dict(model="meta-llama/Llama-3.2-1B-Instruct", isl=4000, osl=500, qps=42.0, disagg_qps=0.0,
             disagg_prefill_ranks=0)
    d.update(kw)
    return argparse.Namespace(**d)


def test_disagg_plan_like_for_like():
    """The disagg phase runs at the agg phase's arrival rate whenever its P:D split can carry it
    (3P+5D on 8 GPUs), and falls back to the capacity rate when it cannot (1P+1D on 2 GPUs)."""
    import bench
    p, d, q = bench.disagg_plan(_ns(), 8)
    assert (p, d) == (3, 5) and q == 42.0
    p, d, q = bench.disagg_plan(_ns(), 2)
    assert (p, d) == (1, 1) and q < 42.0
    assert bench.disagg_plan(_ns(disagg_qps=-1), 8)[2] < 42.0
    assert bench.disagg_plan(_ns(disagg_qps=30.0), 8)[2] == 30.0
    # the default arrival rate (QPS 44) is carried like-for-like by 3P+5D; 4 GPUs split 2P+2D
    assert bench.disagg_plan(_ns(qps=44.0), 8) == (3, 5, 44.0)
    assert bench.disagg_plan(_ns(qps=44.0), 4)[:2] == (2, 2)
    assert bench.disagg_plan(_ns(qps=44.0), 3)[:2] == (1, 2)


def test_compare_modes_marks_winners():
    import bench
    agg = {"value": 20000.0, "ttft_p50_ms": 35.0, "ttft_p90_ms": 60.0, "itl_p50_ms": 9.0, "itl_p90_ms": 22.0}
    dis = {"value": 19800.0, "ttft_p50_ms": 50.0, "ttft_p90_ms": 80.0, "itl_p50_ms": 12.0, "itl_p90_ms": 13.0,
           "qps_per_gpu": 42.0}
    c = bench.compare_modes(agg, dis, 42.0)
    assert c["like_for_like"] is True
    assert c["value"]["better"] == "agg" and c["itl_p90_ms"]["better"] == "disagg"
    assert c["ttft_p50_ms"]["better"] == "agg"
