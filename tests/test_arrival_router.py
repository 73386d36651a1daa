"""Routed arrivals for the N-GPU bench: one Poisson stream at the node's rate,
each request placed by the frontend's KV-aware router (mxserve/router/router.py) from the load the
ranks report (mxserve/tools/arrival_hub.py), per-rank counts and TTFT in the bench line."""
import json
import os
import sys
import threading
import time

from tests.bench_utils import new_tag, run_group, wait_gone

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _load(active=0, waiting=0, added=0, total=1000):
    return {"num_running": 0, "num_waiting": 0, "kv_total_blocks": total, "kv_free_blocks": total - active,
            "kv_waiting_blocks": waiting, "num_added": added}


def test_router_spreads_a_burst_between_heartbeats():
    """Arrivals between two load reports count against the worker they went to, so a burst does not
    all land on the worker that looked emptiest at the last report; a report that includes them
    (num_added moved) retires them."""
    from mxserve.router.router import Registry, Router, WorkerInfo
    reg = Registry()
    for i in range(2):
        reg.register(WorkerInfo(worker_id=f"w{i}", url="", model="m", kv_total_blocks=1000))
        reg.heartbeat(f"w{i}", _load())
    r = Router(reg, mode="kv")
    prompt = list(range(100, 100 + 400))  # 26 blocks with the first token
    picks = [r.pick(reg.list(), prompt)[0].worker_id for _ in range(8)]
    assert picks.count("w0") == 4 and picks.count("w1") == 4, picks
    w0 = reg.workers["w0"]
    assert len(w0.unseen) == 4 and w0.load_blocks() == 4 * 26
    # w0's report now holds 3 of its 4 requests (as waiting demand): one stays unseen
    reg.heartbeat("w0", _load(waiting=3 * 26, added=3))
    assert len(w0.unseen) == 1 and w0.load_blocks() == 4 * 26
    # a worker that does not report num_added: its report is all the router knows
    reg.heartbeat("w1", {"kv_total_blocks": 1000, "kv_free_blocks": 1000})
    assert not reg.workers["w1"].unseen


def test_router_unseen_load_does_not_leak():
    """Phantom load: a failed dispatch is forgotten at once, an entry the worker never
    reports expires after unseen_ttl, and a worker restart (num_added going backwards) drops every
    entry routed before it."""
    from mxserve.router.router import Registry, Router, WorkerInfo
    reg = Registry(unseen_ttl=0.2)
    reg.register(WorkerInfo(worker_id="w0", url="", model="m", kv_total_blocks=1000))
    reg.heartbeat("w0", _load(added=5))
    r = Router(reg, mode="kv")
    w0 = reg.workers["w0"]
    prompt = list(range(100, 100 + 400))  # 26 blocks with the first token
    r.pick([w0], prompt, request_id="a")
    r.pick([w0], prompt, request_id="b")
    assert w0.load_blocks() == 2 * 26
    assert r.forget(w0, "a") and not r.forget(w0, "a") and not r.forget(w0, "zz")
    assert w0.load_blocks() == 26 and len(w0.unseen) == 1
    reg.heartbeat("w0", _load(waiting=26, added=6))  # "b" reached the queue: its report holds it now
    assert not w0.unseen and w0.load_blocks() == 26
    r.pick([w0], prompt, request_id="c")  # never reported (e.g. rejected by the worker): expires
    assert w0.load_blocks() == 2 * 26
    time.sleep(0.25)
    assert w0.load_blocks() == 26 and not w0.unseen
    r.pick([w0], prompt, request_id="d")
    reg.heartbeat("w0", _load(added=0))  # restarted: its counter starts over
    assert not w0.unseen and w0.load_blocks() == 0


def test_scheduler_reports_admission_counter_and_waiting_demand():
    from mxserve.config import EngineArgs
    from mxserve.engine.engine import LLMEngine
    from mxserve.engine.request import SamplingParams
    eng = LLMEngine(EngineArgs(model="tiny-llama", device="cpu", max_model_len=512, cpu_num_blocks=256))
    try:
        sp = SamplingParams(max_tokens=2, ignore_eos=True)
        eng.add_request(list(range(10, 50)), sp, request_id="a")
        eng.add_request(list(range(10, 30)), sp, request_id="b")
        st = eng.scheduler.stats()
        assert st["num_added"] == 2
        bs = eng.scheduler.kv.block_size
        assert st["kv_waiting_blocks"] == -(-41 // bs) + -(-21 // bs)
        while eng.has_unfinished():
            eng.step()
        st = eng.scheduler.stats()
        assert st["num_added"] == 2 and st["kv_waiting_blocks"] == 0
    finally:
        eng.close()


def test_hub_routes_one_stream_over_ranks():
    """In-process hub + two clients: every request reaches exactly one rank, at its scheduled arrival
    time on the shared clock, and the summary counts them per rank."""
    from mxserve.tools.arrival_hub import ArrivalClient, ArrivalHub
    hub = ArrivalHub([0, 1], rate=400.0, isl=64, vocab=1000, seed=1)
    cls = [ArrivalClient(hub.address, r, kv_total_blocks=10000) for r in (0, 1)]
    got = {0: [], 1: []}
    stop = threading.Event()

    def serve(k):
        cl = cls[k]
        n = 0
        cl.report(lambda: _load(added=n), force=True)
        cl.start()
        while not stop.is_set():
            for rid, t_arr, prompt in cl.poll(0.01):
                assert len(prompt) == 64 and t_arr <= time.perf_counter() + 1e-3
                got[k].append(rid)
                n += 1
            cl.report(lambda: _load(active=26 * n, added=n))
        cl.stop()
    ts = [threading.Thread(target=serve, args=(k,)) for k in (0, 1)]
    for t in ts:
        t.start()
    time.sleep(0.6)
    stop.set()
    for t in ts:
        t.join(5)
    hub.close(5)
    s = hub.summary()
    for cl in cls:
        cl.close()
    assert s["error"] is None, s
    n0, n1 = len(got[0]), len(got[1])
    assert n0 + n1 >= 100, (n0, n1)
    assert set(got[0]).isdisjoint(got[1])
    assert s["per_rank"]["0"] >= n0 and s["per_rank"]["1"] >= n1
    assert min(n0, n1) >= 0.3 * (n0 + n1), (n0, n1)  # load-balanced, not all on one rank


def test_bench_two_ranks_routes_arrivals(tmp_path):
    """bench.py --gpus 2 (CPU plumbing run): the line reports the router's per-rank request counts
    and each rank's token rate and TTFT."""
    tag = new_tag()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="1", MXS_TEST_TAG=tag)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "6", "--warmup", "4", "--qps", "8",
           "--device", "cpu", "--gpus", "2", "--max-warmup-s", "6", "--steady-window-s", "1",
           "--min-ttft-samples", "4", "--iters-per-step", "10", "--mode", "agg", "--probe-timeout-s", "0"]
    r = run_group(cmd, timeout=180, cwd=str(tmp_path), env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    arr = d["arrivals"]
    assert arr["router"] == "kv" and arr["error"] is None and arr["node_rate"] == 16.0
    assert sum(arr["per_rank"].values()) == arr["requests"] > 0
    assert all(v > 0 for v in arr["per_rank"].values()), arr
    pr = d["per_rank"]
    assert pr["rank"] == [0, 1] and len(pr["ttft_p50_ms"]) == 2 and all(x > 0 for x in pr["tok_s"])
    assert wait_gone(tag, 15) == []
