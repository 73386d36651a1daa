"""The disagg prefill loop (mxserve/disagg/prefill_loop.py) never waits for a KV push: with a push
still in flight it keeps launching prefill steps, "done" leaves only once the push's event fires,
and the source blocks stay allocated until then.  A stop phase drains the
pushes, joins the barrier and returns without reading the channel again (the EOFError of VERDICT
r5 weak #4).  CPU engine, a fake transfer agent whose events complete when the test says so."""
import threading
import time
from multiprocessing import Pipe

from mxserve.config import EngineArgs
from mxserve.disagg.prefill_loop import serve_prefill
from mxserve.engine.engine import LLMEngine


class FakeEvent:
    def __init__(self):
        self.fired = threading.Event()

    def query(self) -> bool:
        return self.fired.is_set()

    def synchronize(self) -> None:
        assert self.fired.wait(30), "a push never completed"


class FakeAgent:
    backend = "xgmi"

    def __init__(self, eng):
        self.eng = eng
        self.pushes = []  # (engine steps at issue, [rids' src blocks], event)
        self.closed = False

    def connect(self, target):
        pass

    def push_async(self, jobs, after=None):
        ev = FakeEvent()
        self.pushes.append((self.eng.num_steps, [list(j[0]) for j in jobs], ev))
        return ev

    def read_blocks(self, src):
        raise AssertionError("the host path is not used here")

    def close(self):
        self.closed = True


def _wait(cond, timeout=60.0):
    t0 = time.time()
    while not cond():
        assert time.time() - t0 < timeout, "timed out"
        time.sleep(0.005)


def test_prefill_keeps_stepping_while_a_push_is_in_flight():
    ea = EngineArgs(model="tiny-llama", device="cpu", cpu_num_blocks=256, max_model_len=512,
                    max_num_batched_tokens=32, max_num_seqs=8, load_format="random", seed=3)
    eng = LLMEngine(ea)
    agent = FakeAgent(eng)
    ours, theirs = Pipe()
    barriers = []
    res = {}
    t = threading.Thread(target=lambda: res.setdefault("moved", serve_prefill(
        eng, 0.0, lambda: barriers.append(time.time()), [ours], agent=agent)), daemon=True)
    t.start()
    theirs.send(("desc", {"backend": "xgmi"}))
    assert theirs.recv() == ("mapped", True)
    theirs.send(("phase", "warmup"))
    # A: 20 tokens, one step.  Its push is issued and held.
    theirs.send(("prefill", "A", list(range(10, 30)), [0, 1], 0, 0, None))
    _wait(lambda: len(agent.pushes) == 1)
    steps_at_push = agent.pushes[0][0]
    # B: 100 tokens at 32 per step -> 4 prefill steps, launched while A's push is still in flight
    theirs.send(("prefill", "B", list(range(200, 300)), list(range(2, 9)), 0, 16, None))
    _wait(lambda: eng.num_steps >= steps_at_push + 2)
    assert not agent.pushes[0][2].query()
    assert not theirs.poll(0.05), "done for A sent before its push completed"
    assert "A" in eng.requests, "A's source blocks released before its push completed"
    agent.pushes[0][2].fired.set()
    msg = theirs.recv()
    assert msg[0] == "done" and msg[1] == "A" and len(msg[4]) == 4
    t_recv, t_sched, t_first, t_done = msg[4]
    assert t_recv <= t_sched <= t_first <= t_done
    _wait(lambda: "A" not in eng.requests)  # released once its push is done
    _wait(lambda: len(agent.pushes) == 2)
    assert agent.pushes[1][0] >= steps_at_push + 2
    # stop: the in-flight push of B is drained before the barrier; nothing is read after it
    theirs.send(("phase", "stop"))
    time.sleep(0.2)
    assert t.is_alive(), "stop must wait for the in-flight push"
    agent.pushes[1][2].fired.set()
    t.join(timeout=30)
    assert not t.is_alive() and len(barriers) == 2 and agent.closed
    assert theirs.recv()[1] == "B"
    theirs.close()  # the decode side closes right after the barrier: the loop has already returned
    assert res["moved"] == 2 + 7
