"""Open-loop arrivals for a multi-rank serving benchmark, routed by the frontend's KV-aware router.

The reference serves Llama-3.2-1B as `replicas:` of single-GPU workers behind one frontend whose
router picks a worker per request (examples/deploy/vllm/agg.yaml:14,21; the router mode flag in
examples/deploy/vllm/agg_router.yaml).  bench.py reproduces that on N GPUs: ONE Poisson stream at
the node's rate, each request sent to the rank that mxserve.router.Router.pick (the same Registry /
Router / native KvIndexer code the frontend runs) chooses from the load the ranks report, instead
of N independent per-rank streams.

  hub (a process rank 0 starts: spawn())     rank r (ArrivalClient)
    ("hello", r, kv_total_blocks, block_size) <-  connect after its engine is built
    ("start", r)                              <-  every rank in steady loop: arrivals start
    ("load", r, scheduler stats)              <-  every few ms: Registry.heartbeat
    -> ("req", rid, t_arrival, prompt)            to the routed rank at its arrival time
    ("stop", r)                               <-  the rank's timed window ended

Arrival times are CLOCK_MONOTONIC, which time.perf_counter reads on Linux (one clock for every
process of the node).  Per-rank request counts come back in ArrivalHub.summary().
"""
from __future__ import annotations

import queue
import threading
import time
from multiprocessing.connection import Client, Listener
from typing import Optional

import numpy as np

AUTHKEY = b"mxs-arrivals"


class ArrivalHub:
    def __init__(self, ranks: list, rate: float, isl: int, vocab: int, seed: int = 4321, mode: str = "kv",
                 model: str = "bench"):
        from ..router.router import Registry, Router, WorkerInfo
        self._WorkerInfo = WorkerInfo
        self.ranks = list(ranks)
        self.rate = float(rate)
        self.isl = int(isl)
        self.vocab = int(vocab)
        self.model = model
        self.rng = np.random.default_rng(seed)
        self.reg = Registry(ttl=1e9)
        self.router = Router(self.reg, mode=mode, seed=seed)
        self.lst = Listener(("127.0.0.1", 0), authkey=AUTHKEY, backlog=max(8, len(self.ranks)))
        self.address = self.lst.address
        self.conns: dict = {}
        self.sent = {r: 0 for r in self.ranks}
        self.started: set = set()
        self.stopped: set = set()
        self._start = threading.Event()
        self._done = threading.Event()
        self.t0 = 0.0
        self.n = 0
        self.late_s = 0.0
        self.error: Optional[str] = None
        self._thread = threading.Thread(target=self._run, name="arrival-hub", daemon=True)
        self._thread.start()

    # ---------------------------------------------------------------- hub side
    def _run(self) -> None:
        try:
            for _ in self.ranks:
                c = self.lst.accept()
                msg = c.recv()
                assert msg[0] == "hello", msg
                r = int(msg[1])
                self.conns[r] = c
                self.reg.register(self._WorkerInfo(worker_id=str(r), url="", model=self.model,
                                                   kv_total_blocks=int(msg[2]), block_size=int(msg[3])))
            self.lst.close()
            for r, c in self.conns.items():
                threading.Thread(target=self._reader, args=(r, c), daemon=True).start()
            self._start.wait()
            self._dispatch()
        except Exception as e:  # noqa: BLE001 - reported in summary(); ranks see their channel close
            self.error = repr(e)[:300]
        finally:
            self._done.set()
            for c in self.conns.values():  # every rank stopped: its reader sees EOF and ends
                try:
                    c.close()
                except OSError:
                    pass

    def _reader(self, r: int, c) -> None:
        try:
            while True:
                msg = c.recv()
                kind = msg[0]
                if kind == "load":
                    self.reg.heartbeat(str(r), msg[2])
                elif kind == "start":
                    self.started.add(r)
                    if len(self.started) == len(self.ranks):
                        self.t0 = time.monotonic()
                        self._start.set()
                elif kind == "stop":
                    self.stopped.add(r)
                    if len(self.stopped) == len(self.ranks):
                        self._start.set()
                        return
        except (EOFError, OSError):
            self.stopped.add(r)
            self._start.set()

    def _dispatch(self) -> None:
        t_next = self.t0 + self.rng.exponential(1.0 / self.rate)
        while len(self.stopped) < len(self.ranks):
            now = time.monotonic()
            if t_next > now:
                time.sleep(min(0.02, t_next - now))
                continue
            self.late_s = max(self.late_s, now - t_next)
            prompt = self.rng.integers(100, self.vocab - 100, size=self.isl, dtype=np.int64)
            cands = [w for w in self.reg.list() if int(w.worker_id) not in self.stopped]
            if not cands:
                break
            w, _ = self.router.pick(cands, prompt.tolist())
            r = int(w.worker_id)
            rid = f"q{self.n}"
            self.n += 1
            self.sent[r] += 1
            try:
                self.conns[r].send(("req", rid, t_next, prompt.astype(np.int32)))
            except (OSError, BrokenPipeError):
                self.stopped.add(r)
            t_next += self.rng.exponential(1.0 / self.rate)

    def close(self, timeout: float = 5.0) -> None:
        self._start.set()
        self._done.wait(timeout)
        for c in self.conns.values():
            try:
                c.close()
            except OSError:
                pass

    def summary(self) -> dict:
        n = max(1, self.n)
        return {"router": self.router.mode, "node_rate": self.rate, "requests": self.n,
                "per_rank": {str(r): self.sent[r] for r in self.ranks},
                "share_max_over_mean": round(max(self.sent.values()) * len(self.ranks) / n, 3),
                "dispatch_late_ms_max": round(self.late_s * 1e3, 2), "error": self.error}


class ArrivalClient:
    """A rank's end of the hub channel: a reader thread queues the requests routed here."""

    def __init__(self, address, rank: int, kv_total_blocks: int, block_size: int = 16,
                 report_every_s: float = 0.004):
        self.rank = rank
        self.conn = Client(tuple(address), authkey=AUTHKEY)
        self.conn.send(("hello", rank, int(kv_total_blocks), int(block_size)))
        self.q: queue.Queue = queue.Queue()
        self.report_every_s = report_every_s
        self._last = 0.0
        self.received = 0
        self._lock = threading.Lock()
        self._ev = threading.Event()
        self._thread = threading.Thread(target=self._reader, daemon=True)
        self._thread.start()

    def _reader(self) -> None:
        try:
            while True:
                msg = self.conn.recv()
                if msg[0] == "req":
                    self.q.put((msg[1], float(msg[2]), msg[3]))
                    self._ev.set()
        except (EOFError, OSError, TypeError, ValueError):
            pass  # the hub closed its end (every rank stopped) or this end was closed

    def wait(self, timeout: float) -> None:
        """Block until a request is queued here (or timeout)."""
        if self.q.empty():
            self._ev.wait(timeout)

    def _send(self, msg) -> None:
        with self._lock:
            try:
                self.conn.send(msg)
            except (OSError, BrokenPipeError):
                pass

    def start(self) -> None:
        self._send(("start", self.rank))

    def stop(self) -> None:
        self._send(("stop", self.rank))

    def report(self, stats_fn, force: bool = False) -> None:
        """Send the scheduler's load (rate limited to one message per report_every_s)."""
        now = time.monotonic()
        if force or now - self._last >= self.report_every_s:
            self._last = now
            self._send(("load", self.rank, stats_fn()))

    def poll(self, wait_s: float = 0.0) -> list:
        """[(request_id, arrival time on the perf_counter clock, prompt token ids)] routed here."""
        out = []
        self._ev.clear()
        try:
            if wait_s > 0:
                out.append(self.q.get(timeout=wait_s))
            while True:
                out.append(self.q.get_nowait())
        except queue.Empty:
            pass
        self.received += len(out)
        return out

    def close(self, timeout: float = 10.0) -> None:
        """The hub closes its end once every rank has stopped; the reader then sees EOF.  Close this
        end only after that: closing a socket under a reader blocked in it frees the descriptor
        number while the reader may still read from it, and a socket opened next (the next phase's
        control channels) could take that number."""
        self._thread.join(timeout)
        try:
            self.conn.close()
        except OSError:
            pass


def spawn(ranks: list, rate: float, isl: int, vocab: int, seed: int = 4321, mode: str = "kv"):
    """Start the hub in a process of its own (no GPU, no GIL shared with an engine loop); returns
    (Popen, port).  Its last stdout line is the summary, once every rank has stopped."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([root] + [x for x in [os.environ.get("PYTHONPATH")] if x]))
    spec = json.dumps({"ranks": list(ranks), "rate": rate, "isl": isl, "vocab": vocab, "seed": seed, "mode": mode,
                       "parent": os.getpid()})
    p = subprocess.Popen([sys.executable, "-m", "mxserve.tools.arrival_hub", spec], stdout=subprocess.PIPE,
                         stdin=subprocess.DEVNULL, env=env, cwd=root)
    line = p.stdout.readline().decode()
    if not line.startswith("ADDR "):
        p.kill()
        raise RuntimeError(f"arrival hub did not start: {line!r}")
    return p, int(line.split()[1])


def collect(p, timeout: float = 15.0) -> dict:
    """The hub's summary (after every rank sent stop), or an error record."""
    import json
    import subprocess
    try:
        out, _ = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        p.communicate()
        return {"error": f"arrival hub gave no summary within {timeout:.0f}s"}
    lines = [ln for ln in out.decode(errors="replace").splitlines() if ln.startswith("SUMMARY ")]
    return json.loads(lines[-1][len("SUMMARY "):]) if lines else {"error": f"hub exited {p.returncode}"}


def _main(spec: str) -> int:
    import json
    import os
    d = json.loads(spec)
    parent = int(d.pop("parent"))
    hub = ArrivalHub(**d)

    def watch_parent():  # the rank that started this hub is gone: nothing will stop it otherwise
        while os.getppid() == parent:
            time.sleep(0.5)
        os._exit(1)
    threading.Thread(target=watch_parent, daemon=True).start()
    print(f"ADDR {hub.address[1]}", flush=True)
    hub._done.wait()
    print("SUMMARY " + json.dumps(hub.summary()), flush=True)
    hub.close(1.0)
    return 0


if __name__ == "__main__":
    import sys
    sys.exit(_main(sys.argv[1]))
