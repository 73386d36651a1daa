#!/usr/bin/env python3
"""Headline benchmark: output tok/s (node) + p50 TTFT at a fixed QPS, Llama-3.2-1B-Instruct,
aggregated vs disaggregated serving (BASELINE.json metric / configs 2-3).

Launch: `python bench.py --gpus N` spawns N ranks itself (torch.distributed.run, one process per
GPU) before anything touches the GPU; under an external launcher WORLD_SIZE must equal --gpus.

Phases (--mode auto: agg for N = 1, agg then disagg for N >= 2, both in the one JSON line):
  probe   N >= 2: the multi-GPU probe (mxserve/tools/mgpu_probe.py; TP / EP vs the unsharded model,
          collectives, peer copies) in processes started before the ranks touch the GPU
  agg     each rank runs an independent engine replica -- the reference scales Llama-3.2-1B by
          `replicas:` of single-GPU workers behind the frontend router (examples/deploy/vllm/agg.yaml:14,21;
          SURVEY.md §2.4 P01) -- under an open-loop Poisson arrival process of --qps requests/s
          per GPU (weak scaling).  `value` is this phase.  N >= 2 (--arrivals router, default):
          ONE stream at N x --qps, each request placed by the frontend's KV-aware router
          (mxserve.router.Router, native KvIndexer) from the ranks' scheduler load reports, as
          the reference's frontend places requests over its replicas (mxserve/tools/arrival_hub.py;
          the line's `arrivals` / `per_rank` show the split and each rank's TTFT and token rate).
  disagg  ranks [0, P) prefill, [P, N) decode (examples/deploy/vllm/disagg.yaml:18-57: separate
          prefill and decode workers, each scaled by its own `replicas`).  disagg_plan() sizes P:D
          from the two roles' capacities for this workload (mxserve/profiler/capacity_mi355x.json,
          measured: a decode GPU is KV-bandwidth bound at 76.7 req/s, a prefill GPU computes 127.6
          req/s: 1P+1D at N = 2, 2P+2D at 4, 3P+5D at 8)
          and offers the node the rate that loads the tighter role to 85 %; when the split carries
          the agg rate, the disagg phase runs at it (like-for-like).  Default rate 47 req/s per GPU,
          6 % below the measured saturation of one MI355X (50 req/s: the running set reaches the
          448-sequence cap and TTFT p90 leaves the 100 ms range; 51 queues, TTFT p50 276 ms), so a
          slower device of the pool still holds TTFT: QPS 45 / 47 / 48 / 49 / 50 / 51 give 21.6 / 22.1 /
          22.3 / 22.8 / 23.2 / 23.5k tok/s at TTFT p50 30 / 34 / 41 / 49 / 64 / 277 ms
          (profiles/r5/qps_sweep/).  The realised Poisson rate of the fixed-seed arrival stream over those windows
          is 97-98 % of nominal, which with the request tail bounds value at ~94 % of QPS x OSL.
          Requests arrive at the decode ranks (routed over them like the agg phase's when D >= 2);
          a decode rank reserves KV blocks and hands each
          prompt to the prefill rank with the fewest prompts in flight, which computes it, pushes
          the blocks into the decode rank's staging arena with the IPC copy kernel (xGMI between
          GPUs; mxserve/disagg/kv_transfer.py) and returns the first token.  TTFT includes the
          KV transfer.

Workload: ISL 4000 / OSL 500, the only request shape the reference quantifies
(examples/dgdr/trtllm/dgdr.yaml:22-26).  Synthetic random prompt token ids, random-init weights of
the real architecture (no network on the GPU box); every request generates exactly OSL tokens.

Steps and steady state.  A step is --iters-per-step (default 50) engine iterations (continuous
batching: decodes + chunked prefill under the token budget) of a request-owning rank.  Under an
open-loop Poisson load the token rate of a short window follows the running set, which drifts with
the arrivals of the last request lifetime (~4 s here), and the number of prefill-carrying iterations
in it: measured on one MI355X at QPS 40-42, 20 windows of 20 iterations (0.2 s) spread 17.3-21.1k
tok/s and windows of 200 iterations (2 s) 16.9-19.8k, against ~20.3k over 1,500 iterations.  K = 20
steps of 50 iterations is a ~9 s window, a couple of request lifetimes.  The
warmup runs at least W steps and
until the open-loop system is in steady state on every rank: over the last two windows the mean
running set is flat, completions match arrivals and two request lifetimes have passed (or
--max-warmup-s passes; reported).  Then a
short soak collects TTFT samples in steady state, and exactly K steps are timed between a
barrier + device sync on both sides.  value = output tokens produced in the timed window summed
over ranks / the slowest rank's window.  TTFT is measured from each request's scheduled Poisson
arrival (queueing included) for first tokens landing in the steady-state soak + timed window.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

BASELINE_METRIC = "output tok/s (node) + p50 TTFT at fixed QPS, Llama-3.2-1B agg vs disagg"
_VERBOSE = os.environ.get("MXS_BENCH_VERBOSE", "0") == "1"
_T0 = time.perf_counter()
_WALL0 = time.time()  # the whole-run wall budget (--time-budget-s) counts from here


if _VERBOSE:  # stacks of every thread once a minute: where a stalled rank is waiting
    import faulthandler
    faulthandler.dump_traceback_later(45, repeat=True)



# One MI355X, this build, bench.py --steps 20 --warmup 5 --qps Q (profiles/r5/qps_sweep/): QPS ->
# (tok/s, TTFT p50 ms, TTFT p90 ms).  Saturation: 50 req/s (the running set reaches the 448 cap, TTFT
# p90 205 ms; 51 queues).  The default sits 6 % below it.
SATURATION_QPS = 50.0
SATURATION_SWEEP = {45: (21636, 30, 53), 47: (22116, 34, 60), 48: (22265, 41, 73), 49: (22815, 49, 82),
                    50: (23189, 64, 205), 51: (23471, 277, 626)}
DEFAULT_QPS = 47.0

def vlog(msg: str) -> None:
    if _VERBOSE:
        print(f"[bench r{os.environ.get('RANK', '0')} {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr,
              flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--iters-per-step", type=int, default=int(os.environ.get("MXS_BENCH_ITERS_PER_STEP", "50")),
                    help="engine iterations per bench step (see the module docstring: a window must span a few "
                         "request lifetimes for the token rate of an open-loop Poisson load to settle)")
    ap.add_argument("--mode", choices=["auto", "agg", "disagg", "both"], default=os.environ.get("MXS_BENCH_MODE", "auto"))
    ap.add_argument("--model", default="meta-llama/Llama-3.2-1B-Instruct")
    ap.add_argument("--isl", type=int, default=4000)
    ap.add_argument("--osl", type=int, default=500)
    ap.add_argument("--qps", type=float, default=float(os.environ.get("MXS_BENCH_QPS", str(DEFAULT_QPS))),
                    help="Poisson arrival rate per GPU (requests/s)")
    ap.add_argument("--arrivals", choices=["router", "local"], default=os.environ.get("MXS_BENCH_ARRIVALS", "router"),
                    help="N >= 2: router = one Poisson stream at the node's rate, each request routed to a rank "
                         "by the frontend's KV-aware router from the ranks' load reports "
                         "(mxserve/tools/arrival_hub.py); local = an independent stream per rank")
    ap.add_argument("--router-mode", choices=["kv", "round_robin", "random"], default="kv")
    ap.add_argument("--max-num-seqs", type=int, default=int(os.environ.get("MXS_BENCH_MAX_SEQS", "448")),
                    help="running-sequence cap (448: at QPS 49 the 384 cap made arrivals wait for a slot, TTFT p90 194 vs 82 ms, profiles/r4/s2/max_num_seqs/)")
    ap.add_argument("--disagg-max-num-seqs", type=int, default=512,
                    help="decode ranks of the disagg phase carry 2x the per-GPU request rate")
    ap.add_argument("--disagg-qps", type=float, default=float(os.environ.get("MXS_BENCH_DISAGG_QPS", "0")),
                    help="disagg phase arrival rate per GPU; 0 = the agg rate (like-for-like) when the split "
                         "can carry it, else the capacity rate; < 0 = the capacity rate of disagg_plan()")
    ap.add_argument("--disagg-prefill-ranks", type=int, default=int(os.environ.get("MXS_BENCH_DISAGG_P", "0")),
                    help="prefill ranks of the disagg phase (the rest decode); 0 = disagg_plan()")
    ap.add_argument("--max-num-batched-tokens", type=int, default=int(os.environ.get("MXS_BENCH_MNBT", "6144")),
                    help="token budget of a step (prefill chunk + decode rows): 6144 holds ITL p90 at 21 ms at QPS 48 "
                         "where 8192 sits at 24-25 ms, at the same output rate (profiles/r4/sched_q48_*.json)")
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--itl-target-ms", type=float, default=float(os.environ.get("MXS_BENCH_ITL_TARGET_MS", "0")),
                    help="decode-aware prefill chunk budget (0 = fixed --max-num-batched-tokens chunks)")
    ap.add_argument("--enforce-eager", action="store_true")
    ap.add_argument("--kv-cache-dtype", default=os.environ.get("MXS_BENCH_KV_DTYPE", "auto"),
                    help="auto (bf16, the headline) | fp8 (e4m3fn KV cache: a separate, labelled data point)")
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--max-warmup-s", type=float, default=90.0,
                    help="cap on the warmup that waits for steady state")
    ap.add_argument("--steady-window-s", type=float, default=2.5,
                    help="length of each of the two windows compared by the steady-state test")
    ap.add_argument("--min-ttft-samples", type=int, default=40,
                    help="TTFT samples per request-owning rank collected in steady state before timing")
    ap.add_argument("--phase-timeout-s", type=float, default=float(os.environ.get("MXS_BENCH_PHASE_TIMEOUT", "420")),
                    help="a disagg phase that has not finished by then is reported as failed")
    ap.add_argument("--num-gpu-blocks", type=int, default=None,
                    help="KV pool size per rank (default: what the GPU's free memory allows)")
    ap.add_argument("--probe-timeout-s", type=float, default=float(os.environ.get("MXS_BENCH_PROBE_TIMEOUT", "300")),
                    help="N >= 2: budget of the multi-GPU probe run after the serving phases (0: no probe)")
    ap.add_argument("--served", type=int, default=int(os.environ.get("MXS_BENCH_SERVED", "1")),
                    help="N = 1: after the engine-direct phase, drive the same Poisson stream through the served "
                         "stack (frontend HTTP/SSE -> worker streamer -> engine) and report it as the line's "
                         "`served` block (mxserve/tools/served_phase.py); 0 = skip")
    ap.add_argument("--time-budget-s", type=float, default=float(os.environ.get("MXS_BENCH_BUDGET_S", "450")),
                    help="wall budget of the whole run, from process start: the probe and the disagg phase get "
                         "what the agg phase leaves; at the deadline rank 0 prints the line it has and every "
                         "rank exits (the driver's own timeout is 600 s)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------- wall budget
_RESERVE_S = 25.0  # what the probe leaves the ranks to collect its result and print before the deadline


class Guard:
    """Whole-run deadline of one rank.

    Every rank arms it at start.  The probe processes (and the disagg phase they host) get absolute
    deadlines derived from it, finish_probe waits only until it, and a watchdog thread enforces it:
    at the deadline rank 0 prints the best line it has (the provisional agg line, with the phases
    that did not finish marked), the children are killed with their process groups, and the rank
    exits 0 (a non-zero worker exit would make torchrun SIGTERM rank 0 before it has printed).  A
    rank whose parent (torchrun) dies exits too, so nothing outlives a killed launcher."""

    def __init__(self, budget_s: float, rank: int):
        self.deadline = _WALL0 + budget_s
        self.rank = rank
        self.lock = threading.Lock()
        self.printed = False
        self.pending = None  # rank 0: the line to print if the budget runs out
        self.children: list = []

    def remaining(self) -> float:
        return self.deadline - time.time()

    def emit(self, line: dict) -> bool:
        with self.lock:
            if self.printed:
                return False
            self.printed = True
        print(json.dumps(line), flush=True)
        return True

    def arm(self) -> "Guard":
        threading.Thread(target=self._watch, daemon=True, name="bench-deadline").start()
        if os.environ.get("TORCHELASTIC_RUN_ID") or os.environ.get("WORLD_SIZE"):
            ppid = os.getppid()
            threading.Thread(target=self._watch_parent, args=(ppid,), daemon=True, name="bench-ppid").start()
        return self

    def _watch(self) -> None:
        # ranks > 0 wait a little longer: rank 0 prints first, whatever the others do
        slack = 0.0 if self.rank == 0 else 10.0
        while self.remaining() + slack > 0:
            time.sleep(min(1.0, max(0.05, self.remaining() + slack)))
        self.expire(f"time budget of {self.deadline - _WALL0:.0f}s spent")

    def _watch_parent(self, ppid: int) -> None:
        while os.getppid() == ppid:
            time.sleep(1.0)
        self.kill_children()
        os._exit(1)

    def kill_children(self) -> None:
        import signal
        for p in self.children:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    p.kill()

    def expire(self, why: str) -> None:
        print(f"bench.py rank {self.rank}: {why}; killing children and exiting", file=sys.stderr, flush=True)
        self.kill_children()
        if self.rank == 0:
            line = self.pending
            if line is None:  # not even the agg phase finished: a failure line, not silence
                line = {"metric": BASELINE_METRIC, "value": None, "unit": "tok/s", "status": "failed",
                        "error": why, "higher_is_better": True}
            else:
                line = dict(line)
                for k in ("disagg", "multi_gpu_probe"):
                    if isinstance(line.get(k), dict) and line[k].get("status") == "pending":
                        line[k] = {"status": "failed", "error": why}
            self.emit(line)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0 if (self.rank != 0 or self.pending is not None) else 3)


_PREFILL_STEP_TOKENS = 16384


def disagg_plan(a, world: int) -> tuple:
    """(prefill ranks, decode ranks, arrival rate per GPU) of the disagg phase.  The role capacities
    come from the same model the DGDR profiler plans with (mxserve/profiler/capacity.py: the measured
    MI355X table for this workload, else its roofline); the split maximises the tighter role's
    capacity (3 prefill : 5 decode GPUs on 8 for the headline workload) and the capacity-derived rate
    loads that role to 85 %."""
    from mxserve.profiler import capacity as capm
    cap = capm.capacity(a.model, a.isl, a.osl)
    cp, cd = cap["prefill_rps"], cap["decode_rps"]
    p = a.disagg_prefill_ranks
    if p <= 0:
        p = capm.pd_split(world, cp, cd)[0]
    p = min(max(1, p), world - 1)
    d = world - p
    full = min(p * cp, d * cd) / world  # per GPU
    qps = a.disagg_qps
    if qps == 0:
        # like-for-like with the agg phase (the same arrival rate per GPU) unless this split cannot
        # carry it (1P+1D on 2 GPUs has one decode GPU for twice its share): then the planned rate
        qps = a.qps if a.qps <= 0.95 * full + 1e-9 else capm.PLAN_UTIL * full
    elif qps < 0:  # capacity-derived: the tighter role loaded to 85 %
        qps = capm.PLAN_UTIL * full
    return p, d, qps


# ---------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def start_probe(a, world: int, guard: Guard, host_disagg: bool = False):
    """N >= 2: one multi-GPU probe process per rank (mxserve/tools/mgpu_probe.py: TP / EP against the
    unsharded model, RCCL and custom all-reduce bandwidth, xGMI peer copies), started BEFORE this rank
    touches the GPU and idle until finish_probe: a crash or hang there costs only the probe.
    host_disagg: the probe processes also run this bench's disagg phase (first, with this bench's
    arguments), so a fault on the cross-GPU KV path cannot take the aggregated result with it.
    The probe runs in a session of its own (killed as a group at the deadline), watches this rank
    (exits when it dies) and reports by an absolute deadline _RESERVE_S ahead of this rank's."""
    if world < 2 or a.probe_timeout_s <= 0:
        return None
    root = os.path.dirname(os.path.abspath(__file__))
    # its own rendezvous: rank 0's probe hosts the store (not torchrun's agent store of this job)
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env["MXS_PROBE_DEADLINE"] = repr(guard.deadline - _RESERVE_S)
    env["MXS_PROBE_TIMEOUT_S"] = repr(a.probe_timeout_s)  # the optional sections' own cap, after disagg
    if host_disagg:
        env["MXS_PROBE_DISAGG_ARGV"] = json.dumps(sys.argv[1:])
    else:
        env.pop("MXS_PROBE_DISAGG_ARGV", None)
    env.update(MXS_PROBE_DEVICE="cpu" if a.device == "cpu" else "auto",
               PYTHONPATH=os.pathsep.join([root] + [x for x in [os.environ.get("PYTHONPATH")] if x]))
    p = subprocess.Popen([sys.executable, "-m", "mxserve.tools.mgpu_probe"], stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, env=env, cwd=root, start_new_session=True)
    guard.children.append(p)
    return p


def finish_probe(p, guard: Guard, ctx):
    """Release the probe (this rank's engine is gone) with the rendezvous port rank 0 picked, and
    wait for it until the deadline leaves just enough to print; rank 0's carries the result."""
    if p is None:
        return None
    port = ctx.gather([float(_free_port()) if ctx.rank == 0 else 0.0])[0, 0]
    # ranks > 0 hand their probe over ("detach": it no longer exits with its bench rank) and leave:
    # only rank 0's probe reports, and a rank that stays holds a GPU context and its memory while the
    # probe runs -- on a node every process maps every GPU, so N ranks + N probes is 2N processes on
    # each GPU against the pool's limit of 16 per GPU, and the probe's engines want the memory
    detach = ctx.rank != 0
    try:
        p.stdin.write(f"go {int(port)}{' detach' if detach else ''}\n".encode())
        p.stdin.close()
    except OSError:
        pass
    p.stdin = None  # closed above: communicate() must not flush it again
    if detach:
        guard.children.remove(p)  # not ours to kill any more
        return None
    timeout_s = max(1.0, guard.remaining() - 10.0)
    try:
        out, _ = p.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        guard.kill_children()
        p.communicate()
        return {"status": "failed", "error": f"no result within {timeout_s:.0f}s (run deadline)"}
    lines = [ln for ln in out.decode(errors="replace").splitlines() if ln.startswith("PROBE ")]
    if lines:
        return json.loads(lines[-1][len("PROBE "):])
    return {"status": "failed", "error": f"probe exited with {p.returncode} and no result"}


def launch_ranks(a) -> int:
    """`--gpus N` without an external launcher: run N ranks under torch.distributed.run as a CHILD
    process (nothing here has touched the GPU; the parent never execs) and return its exit code."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (the only mode the host driver has)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    vlog("launching: " + " ".join(cmd))
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------- load + bookkeeping
class Driver:
    """Open-loop Poisson load on one request-owning rank, steady-state detection and latency
    bookkeeping."""

    def __init__(self, a, rank: int, vocab: int, qps: float):
        rng = np.random.default_rng(1234 + rank)
        self.qps = qps
        self.horizon = 65536
        self.arrivals = np.cumsum(rng.exponential(1.0 / qps, size=self.horizon))
        self.isl = a.isl
        self.osl = a.osl
        self.vocab = vocab
        self.rng = rng
        self.rank = rank
        self.nxt = 0
        self.t_start = 0.0
        self.arrival_of: dict = {}
        self.first_tok: dict = {}
        self.last_tok: dict = {}
        self.itls: list = []
        self.record_ttft = False  # steady state reached: TTFT samples count from here
        self.record = False  # timed window: tokens + ITL
        self.finished = 0
        self.lifetimes: list = []  # arrival -> last token of finished requests (steady-state test)
        self.warmup_steps = 0
        self.warmup_s = 0.0
        self.steady = False
        self.c = {"ttft": [], "tokens": 0}
        # per-step samples for the steady-state test: (time, running set, arrivals, finished)
        self.hist: list = []
        self.source = None  # ArrivalClient: requests routed here by the node's router (--arrivals router)
        self.load_fn = None
        self.breakdown: list = []  # disagg decode rank: per-request TTFT components (BREAKDOWN_KEYS), seconds

    def attach(self, source, load_fn) -> None:
        self.source, self.load_fn = source, load_fn

    def report(self, force: bool = False) -> None:
        if self.source is not None:
            self.source.report(self.load_fn, force)

    def on_phase(self, phase: str) -> None:
        if self.source is None:
            return
        if phase == "warmup":  # arrivals start once every request-owning rank is here
            self.report(force=True)
            self.source.start()
        elif phase == "stop":
            self.source.stop()

    def prompt(self) -> list:
        return self.rng.integers(100, self.vocab - 100, size=self.isl, dtype=np.int64).tolist()

    def due(self) -> list:
        """(request_id, prompt) for every arrival whose time has come."""
        out = []
        if self.source is not None:
            for rid, t_arr, prompt in self.source.poll():
                self.arrival_of[rid] = t_arr  # the hub's schedule, CLOCK_MONOTONIC = perf_counter's clock
                out.append((rid, prompt.tolist()))
            self.nxt += len(out)
            return out
        now_rel = time.perf_counter() - self.t_start
        while self.nxt < self.horizon and self.arrivals[self.nxt] <= now_rel:
            rid = f"r{self.rank}-{self.nxt}"
            self.arrival_of[rid] = self.t_start + self.arrivals[self.nxt]
            out.append((rid, self.prompt()))
            self.nxt += 1
        return out

    def wait_next(self) -> None:
        if self.source is not None:
            self.source.wait(0.05)
        elif self.nxt < self.horizon:
            time.sleep(max(0.0, min(0.05, self.t_start + self.arrivals[self.nxt] - time.perf_counter())))

    def token(self, rid: str, now: float, finished: bool = False) -> None:
        self.finished += finished
        if finished and rid in self.arrival_of:
            self.lifetimes.append(now - self.arrival_of[rid])
        if rid not in self.first_tok:
            self.first_tok[rid] = now
            if self.record_ttft:
                self.c["ttft"].append(now - self.arrival_of[rid])
        elif self.record:
            self.itls.append(now - self.last_tok[rid])
        self.last_tok[rid] = now
        if self.record:
            self.c["tokens"] += 1

    def sample(self, running: int) -> None:
        now = time.perf_counter()
        self.hist.append((now, running, self.nxt, self.finished))
        if len(self.hist) > 20000:  # the steady-state test reads the last two windows (seconds); bound
            # the list (and is_steady's array of it) when a stalled engine makes step() calls cheap
            import bisect
            cut = bisect.bisect_left(self.hist, (now - 60.0,))
            if cut > 0:
                del self.hist[:min(cut, len(self.hist) - 1000)]

    def is_steady(self, window: float) -> bool:
        """Running set flat over two consecutive windows, completions ~= arrivals in the last, and two
        request lifetimes since the load started (OSL x the current iteration time, or the median
        lifetime of the last 20 finished requests if longer -- not the ramp's short small-batch ones):
        one lifetime in, the running set still holds the ramp's requests, served at the small-batch
        ITL, so it reads flat a few seconds before the system settles (warmups of ~12 s here timed a
        window at ~93 % of the offered rate, ~19 s ones at ~98 %)."""
        if not self.hist or self.finished == 0:
            return False
        t_now = self.hist[-1][0]
        if t_now - self.t_start < 2 * window:
            return False
        h = np.asarray(self.hist, dtype=np.float64)
        # the lifetime a request admitted now will have: OSL iterations at the current iteration time
        # (each engine iteration gives every running request one token), not the ramp's shorter ones
        recent = h[h[:, 0] >= t_now - window]
        if len(recent) >= 2:
            life_now = self.osl * (recent[-1, 0] - recent[0, 0]) / (len(recent) - 1)
            if t_now - self.t_start < 2.0 * max(life_now, float(np.median(self.lifetimes[-20:])) if self.lifetimes else 0.0):
                return False
        a_mask = (h[:, 0] >= t_now - 2 * window) & (h[:, 0] < t_now - window)
        b_mask = h[:, 0] >= t_now - window
        if a_mask.sum() < 5 or b_mask.sum() < 5:
            return False
        ra, rb = h[a_mask, 1].mean(), h[b_mask, 1].mean()
        b = h[b_mask]
        arr = b[-1, 2] - b[0, 2]
        fin = b[-1, 3] - b[0, 3]
        flat = abs(rb - ra) <= 0.08 * rb + 1.0
        balanced = arr > 0 and abs(fin - arr) <= 0.2 * arr + 2
        return bool(flat and balanced)

    def stats(self, dt: float) -> list:
        ttft = np.array(self.c["ttft"]) if self.c["ttft"] else np.array([np.nan])
        itl = np.array(self.itls) if self.itls else np.array([np.nan])
        running = float(np.mean([x[1] for x in self.hist[-200:]])) if self.hist else 0.0
        bd = (np.median(np.asarray(self.breakdown), axis=0).tolist() if self.breakdown
              else [float("nan")] * len(BREAKDOWN_KEYS))
        return [dt, float(self.c["tokens"]), float(np.nanmedian(ttft)), float(np.nanmedian(itl)),
                float(len(self.c["ttft"])), float(self.warmup_steps), float(self.warmup_s), float(self.steady),
                running, float(np.nanpercentile(ttft, 90)), float(np.nanpercentile(itl, 90))] + bd


# disagg TTFT components (decode ranks; columns 11.. of the stat rows): arrival -> sent to a prefill
# rank (decode-side reservation queue), -> first scheduled there (pipe + prefill queue), -> first token
# sampled (prefill compute), -> KV push complete (transfer), -> first token emitted here (admission)
BREAKDOWN_KEYS = ("decode_queue_ms", "to_prefill_ms", "prefill_ms", "transfer_ms", "admit_ms")
_STAT_NAN = [0.0, 0.0, float("nan"), float("nan"), 0.0, float("nan"), float("nan"), float("nan"), float("nan"),
             float("nan"), float("nan")] + [float("nan")] * len(BREAKDOWN_KEYS)


def timed_phases(a, step, barrier, agree, drv, running, on_phase=lambda phase: None) -> float:
    """Warm up to steady state (agreed by every request-owning rank), soak for TTFT samples, then
    exactly K steps between barrier + device sync; returns the timed window."""
    phase_hook = on_phase

    def on_phase(ph):
        phase_hook(ph)
        drv.on_phase(ph)
    on_phase("warmup")
    barrier()
    vlog("warmup")
    drv.t_start = time.perf_counter()
    check_every = 25
    i = 0
    while True:
        step()
        drv.sample(running())
        i += 1
        if i % check_every == 0:
            timed_out = time.perf_counter() - drv.t_start > a.max_warmup_s
            mine = i >= a.warmup * a.iters_per_step and (drv.is_steady(a.steady_window_s) or timed_out)
            if i % 200 == 0:
                vlog(f"warmup step {i}: {drv.nxt} arrivals, {drv.finished} finished, running {running()}")
            if agree(mine):
                drv.steady = not timed_out or drv.is_steady(a.steady_window_s)
                break
    # steady state: count TTFTs from here; soak until this rank has enough samples (bounded)
    drv.record_ttft = True
    t_soak = time.perf_counter()
    soak_cap = max(2.0, 3.0 * a.min_ttft_samples / max(drv.qps, 1e-3))
    while len(drv.c["ttft"]) < a.min_ttft_samples and time.perf_counter() - t_soak < soak_cap:
        step()
        drv.sample(running())
        i += 1
    drv.warmup_steps = i
    drv.warmup_s = time.perf_counter() - drv.t_start
    on_phase("timed")
    barrier()
    vlog(f"timed (warmup {i} steps, {drv.warmup_s:.1f}s, steady={drv.steady})")
    drv.record = True
    t0 = time.perf_counter()
    for i in range(a.steps):
        for _ in range(a.iters_per_step):  # one bench step = a fixed number of engine iterations
            step()
            drv.sample(running())
        if i % 20 == 0:
            vlog(f"timed step {i}: {drv.c['tokens']} tokens")
    on_phase("stop")
    barrier()
    vlog("done")
    return time.perf_counter() - t0


def run_agg(a, eng, sp, drv, barrier, agree) -> float:
    def admit():  # late admission (engine/pacing.py): arrivals due by the time the next step is scheduled
        for rid, toks in drv.due():
            eng.add_request(toks, sp, request_id=rid)
    eng.admit_hook = admit

    def step():
        for rid, toks in drv.due():
            eng.add_request(toks, sp, request_id=rid)
        if not eng.has_unfinished():  # idle: wait for the next arrival
            drv.wait_next()
            for rid, toks in drv.due():
                eng.add_request(toks, sp, request_id=rid)
            if not eng.has_unfinished():
                return
        t0 = time.perf_counter()
        outs = eng.step()
        now = time.perf_counter()
        for o in outs:
            drv.token(o.request_id, now, o.finished)
        drv.report()
        if eng.step_times is not None:
            eng.step_times["engine_step"] = eng.step_times.get("engine_step", 0.0) + now - t0
            eng.step_times["loop"] = eng.step_times.get("loop", 0.0) + time.perf_counter() - t_loop[0]
        t_loop[0] = time.perf_counter()

    t_loop = [time.perf_counter()]
    sch = eng.scheduler
    return timed_phases(a, step, barrier, agree, drv, lambda: len(sch.running) + len(sch.waiting))


def _disagg_conns(rank: int, p: int, world: int, gather) -> list:
    """Host control channels of the disagg phase, one per (prefill rank, decode rank): every decode
    rank (ranks [p, world)) listens on a port of its own choosing (published to all ranks through
    `gather`, so no fixed port can collide) and accepts the p prefill ranks."""
    from multiprocessing.connection import Client, Listener
    lst = None
    if rank >= p:
        lst = Listener(("127.0.0.1", 0), authkey=b"mxs-bench", backlog=max(8, p))
    ports = gather([float(lst.address[1]) if lst is not None else 0.0])[:, 0].astype(int)
    if lst is not None:
        conns = [lst.accept() for _ in range(p)]
        lst.close()
        return conns
    conns = []
    for j in range(p, world):
        for _ in range(600):
            try:
                conns.append(Client(("127.0.0.1", int(ports[j])), authkey=b"mxs-bench"))
                break
            except OSError:
                time.sleep(0.1)
        else:
            raise RuntimeError(f"could not reach decode rank {j}")
    return conns


def run_disagg_decode(a, eng, sp, drv, barrier, agree, conns: list) -> float:
    """Decode rank: its arrivals' prompts go to the prefill rank with the fewest prompts in flight
    (one control channel per prefill rank); the KV lands in this rank's pool before the request
    decodes here."""
    from mxserve.disagg.kv_transfer import KVTransferAgent
    agent = KVTransferAgent(eng.runner, "xgmi")
    desc = agent.descriptor()
    for conn in conns:
        conn.send(("desc", desc))
    arenas = []
    for conn in conns:  # each prefill rank maps the arena now, while this rank idles in a socket wait
        ack = conn.recv()
        assert ack[0] == "mapped", ack
        arenas.append(bool(ack[1]) if len(ack) > 1 else True)
    vlog(f"decode arena mapped by the prefill ranks: {arenas}")
    bs = eng.args.block_size
    backlog: list = []
    inflight: dict = {}
    load = [0] * len(conns)

    def pump():
        """Arrivals due -> reserved and sent to a prefill rank; finished prefills -> landed and admitted.
        Runs every loop pass and, as the engine's late-admission hook, once more right before the next
        step is scheduled: a prefill that finished while a step ran joins the very next step."""
        backlog.extend(drv.due())
        while backlog:
            rid, toks = backlog[0]
            req = eng.reserve_remote_prefill(toks, sp, rid)
            if req is None:  # decode pool or batch full: retry next step
                break
            k = min(range(len(conns)), key=load.__getitem__)
            skip = req.num_cached_tokens // bs
            dst = list(req.block_ids[skip:-(-len(toks) // bs)])
            # GPU arena extent over xGMI, else the page-locked /dev/shm arena, else the pipe
            start = agent.acquire(len(dst)) if arenas[k] else None
            shm_start = agent.acquire_shm(len(dst)) if start is None else None
            backlog.pop(0)
            conns[k].send(("prefill", rid, toks, dst, skip, start, shm_start))
            inflight[rid] = (k, dst, start, shm_start, time.perf_counter())
            load[k] += 1
        for conn in conns:
            while conn.poll():
                _, rid, tok, data, tm = conn.recv()
                k, dst, start, shm_start, t_sent = inflight.pop(rid)
                load[k] -= 1
                if start is not None:  # staging extent -> pool blocks, ordered before the next step
                    agent.land(start, dst)
                elif shm_start is not None:
                    agent.land_shm(shm_start, dst)
                elif data is not None:  # host-staged transfer
                    agent.write_blocks(dst, data)
                out = eng.complete_remote_prefill(rid, tok)
                now = time.perf_counter()
                if drv.record_ttft and rid in drv.arrival_of:
                    # TTFT = decode queue + hand-off to prefill + prefill + KV transfer + admission here
                    t_recv, t_sched, t_first, t_done = tm
                    drv.breakdown.append((t_sent - drv.arrival_of[rid], t_sched - t_sent, t_first - t_sched,
                                          t_done - t_first, now - t_done))
                drv.token(rid, now, out.finished)

    eng.admit_hook = pump

    def step():
        backlog.extend(drv.due())
        if not eng.has_unfinished() and not backlog and not inflight:
            drv.wait_next()
        pump()
        if eng.has_unfinished():
            outs = eng.step()
            now = time.perf_counter()
            for o in outs:
                drv.token(o.request_id, now, o.finished)
        elif inflight:  # nothing to decode yet: wait briefly for a prefill to land (arrivals keep coming)
            if len(conns) == 1:
                conns[0].poll(0.002)
            else:
                time.sleep(0.0005)
        drv.report()

    def on_phase(ph):
        for conn in conns:
            conn.send(("phase", ph))

    sch = eng.scheduler
    return timed_phases(a, step, barrier, agree, drv,
                        lambda: len(sch.running) + len(sch.remote) + len(backlog), on_phase=on_phase)


def run_disagg_prefill(eng, temperature: float, barrier, conns: list) -> int:
    """Prefill rank: serve this rank's decode ranks until they say stop (mxserve/disagg/prefill_loop.py);
    returns blocks moved."""
    from mxserve.disagg.prefill_loop import serve_prefill
    return serve_prefill(eng, temperature, barrier, conns, log=vlog)


# ---------------------------------------------------------------------------- phases
class Ctx:
    """Per-rank process context shared by the phases."""

    def __init__(self, a):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.on_gpu = torch.cuda.is_available() and a.device != "cpu"
        self.ndev = torch.cuda.device_count() if self.on_gpu else 0
        self.shared_gpu = self.on_gpu and self.ndev < self.world
        if self.on_gpu:
            torch.cuda.set_device(self.local % self.ndev)
        self.pg_decode = None
        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # control plane only (barriers, steady-state votes, stats): replicas share no tensors,
            # and the P->D KV moves over IPC, so a CPU group keeps RCCL out of the measurement.
            # A collective a peer never joins raises after the timeout instead of gloo's 30 min.
            from datetime import timedelta
            dist.init_process_group("gloo", timeout=timedelta(seconds=max(60.0, min(300.0, a.time_budget_s))))
            p = disagg_plan(a, self.world)[0]
            self.pg_decode = dist.new_group(list(range(p, self.world)), backend="gloo")
        self.sync = torch.cuda.synchronize if self.on_gpu else (lambda: None)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()
        self.sync()

    def agree_fn(self, group, size: int):
        """All request-owning ranks stop warming up at the same step: every rank votes, MIN wins."""
        torch, dist = self.torch, self.dist

        def agree(flag: bool) -> bool:
            if size <= 1:
                return bool(flag)
            t = torch.tensor([1 if flag else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
            return bool(t.item())
        return agree

    def gather(self, vals: list) -> np.ndarray:
        torch, dist = self.torch, self.dist
        t = torch.tensor(vals, dtype=torch.float64)
        if self.world > 1:
            parts = [torch.zeros_like(t) for _ in range(self.world)]
            dist.all_gather(parts, t)
            return torch.stack(parts).numpy()
        return t.unsqueeze(0).numpy()


def engine_args(a, ctx, **kw):
    from mxserve.config import EngineArgs
    args = EngineArgs(model=a.model, device="cuda" if ctx.on_gpu else "cpu", max_num_seqs=a.max_num_seqs,
                      cuda_graph_max_bs=a.max_num_seqs,
                      max_num_batched_tokens=a.max_num_batched_tokens, max_model_len=a.max_model_len,
                      enforce_eager=a.enforce_eager, seed=a.seed, kv_cache_dtype=a.kv_cache_dtype,
                      itl_target_ms=a.itl_target_ms)
    if kw:
        args = args.replace(**kw)
    if not ctx.on_gpu:  # plumbing run only (CPU container): keep it tiny
        args = args.replace(model="tiny-llama", max_model_len=1024, cpu_num_blocks=4096)
    elif ctx.shared_gpu:  # functional run: ranks share a GPU, split its memory
        blocks = int(os.environ.get("MXS_BENCH_SHARED_BLOCKS", "40000"))
        role = kw.get("disagg_mode")
        if role in ("prefill", "decode"):
            # by role: a decode rank holds the running set of world / D GPUs' arrivals (at 40 req/s a
            # 1P+1D decode rank runs ~140 requests x 282 blocks: 40,000 blocks refused reservations and
            # queued arrivals for ~50 ms); a prefill rank holds only the prompts in flight
            p_ranks, d_ranks, _ = disagg_plan(a, ctx.world)
            blocks = (min(2 * blocks, blocks * ctx.world // max(1, d_ranks)) if role == "decode"
                      else max(8192, blocks // 4))
        args = args.replace(num_gpu_blocks=blocks)
    if a.num_gpu_blocks and ctx.on_gpu:
        args = args.replace(num_gpu_blocks=a.num_gpu_blocks)
    return args


def start_arrivals(a, ctx, owners: list, rate: float, isl: int, vocab: int, eng=None, drv=None):
    """--arrivals router with >= 2 request-owning ranks: rank 0 starts the arrival hub (its own
    process: one Poisson stream at the node's rate, each request routed by mxserve.router.Router from
    the ranks' load reports), every rank learns its port, and each owner's Driver takes its requests
    from the hub.  Collective over all ranks of ctx.  Returns rank 0's hub process (else None)."""
    if a.arrivals != "router" or len(owners) < 2:
        return None
    from mxserve.tools import arrival_hub
    hub, port = None, 0
    if ctx.rank == 0:
        hub, port = arrival_hub.spawn(owners, rate, isl, vocab, seed=4321 + a.seed, mode=a.router_mode)
    port = int(ctx.gather([float(port)])[0, 0])
    if ctx.rank in owners:
        cl = arrival_hub.ArrivalClient(("127.0.0.1", port), ctx.rank, eng.runner.num_blocks, eng.args.block_size)
        drv.attach(cl, eng.scheduler.stats)
    return hub


def finish_arrivals(hub, drv) -> dict | None:
    if drv is not None and drv.source is not None:
        drv.source.close()
    if hub is None:
        return None
    from mxserve.tools import arrival_hub
    return arrival_hub.collect(hub)


def free_engine(eng, ctx) -> None:
    eng.close()
    del eng
    gc.collect()
    if ctx.on_gpu:
        ctx.torch.cuda.synchronize()
        ctx.torch.cuda.empty_cache()


def summarize(col: np.ndarray, steps: int, owners: list) -> dict:
    """Whole-job numbers from the per-rank stat rows of the request-owning ranks."""
    col = col[owners]
    t_max = float(col[:, 0].max())
    value = float(col[:, 1].sum()) / t_max if t_max > 0 else 0.0

    def med(c):
        v = col[:, c][~np.isnan(col[:, c])]
        return float(np.median(v)) * 1e3 if len(v) else None

    r = lambda x, n=2: None if x is None else round(x, n)  # noqa: E731
    ttft, itl = med(2), med(3)
    per_rank = None
    if len(owners) > 1:  # how evenly the node's load landed (routed arrivals) and what each rank saw
        rr = lambda v, n: [None if np.isnan(x) else round(float(x), n) for x in v]  # noqa: E731
        per_rank = {"rank": list(owners), "tok_s": rr(col[:, 1] / np.maximum(col[:, 0], 1e-9), 1),
                    "first_tokens": [int(x) for x in col[:, 4]], "ttft_p50_ms": rr(col[:, 2] * 1e3, 2),
                    "ttft_p90_ms": rr(col[:, 9] * 1e3, 2), "itl_p90_ms": rr(col[:, 10] * 1e3, 3),
                    "running_mean": rr(col[:, 8], 1)}
    return {"value": round(value, 2), "ms_per_step": round(t_max / steps * 1e3, 4), "per_rank": per_rank,
            "ttft_p50_ms": r(ttft), "ttft_p90_ms": r(med(9)), "itl_p50_ms": r(itl, 3), "itl_p90_ms": r(med(10), 3),
            "requests_with_first_token": int(col[:, 4].sum()),
            "warmup_steps_executed": int(np.nanmax(col[:, 5])), "warmup_s": round(float(np.nanmax(col[:, 6])), 1),
            "steady_state": bool(np.all(col[:, 7] > 0)), "running_mean": round(float(np.nanmean(col[:, 8])), 1),
            "sla_isl4000_osl500": {"ttft_ms<=600": ttft is not None and ttft <= 600,
                                   "itl_ms<=25": itl is not None and itl <= 25}}


def phase_agg(a, ctx) -> tuple:
    from mxserve.engine.engine import LLMEngine
    from mxserve.engine.request import SamplingParams
    args = engine_args(a, ctx)
    isl, osl = (a.isl, a.osl) if ctx.on_gpu else (min(a.isl, 200), min(a.osl, 20))
    a2 = argparse.Namespace(**{**vars(a), "isl": isl, "osl": osl})
    vlog("agg: building engine")
    eng = LLMEngine(args)
    vlog(f"agg: engine ready ({eng.runner.num_blocks} KV blocks)")
    sp = SamplingParams(max_tokens=osl, temperature=a.temperature, ignore_eos=True)
    drv = Driver(a2, ctx.rank, eng.model_config.vocab_size, a.qps)
    hub = start_arrivals(a, ctx, list(range(ctx.world)), a.qps * ctx.world, isl, eng.model_config.vocab_size,
                         eng, drv)
    group = None
    agree = ctx.agree_fn(group, ctx.world)
    from mxserve.utils.gcpause import PauseStats
    gcs = PauseStats().install()  # collector passes on this rank's loop (the engine froze its start-up heap)
    st = drv.stats(run_agg(a2, eng, sp, drv, ctx.barrier, agree))
    gcs.remove()
    arrivals = finish_arrivals(hub, drv)
    info = {"kv_blocks": eng.runner.num_blocks, "graphs": sorted(eng.runner.graphs) if ctx.on_gpu else [],
            "preemptions": eng.stats()["num_preemptions"], "model": args.model,
            "kv_cache_dtype": "fp8_e4m3fn" if eng.runner.kv_fp8 else ("bf16" if ctx.on_gpu else "fp32"),
            "isl": isl, "osl": osl,
            "arrivals": arrivals or {"mode": "local" if ctx.world > 1 else "single rank",
                                     "per_rank_rate": a.qps}}
    rep = getattr(eng.runner, "decode_gemm_report", None)
    if rep:  # capture-time choice per (bucket, projection): hand-written MFMA kernels vs hipBLASLt
        info["decode_gemm"] = {"pairs": len(rep), "hand_written": sum(r["chosen"] == "mfma" for r in rep),
                               "mt_kernel": sum(bool(r["cfg"]) and r["cfg"][0] == "mt" for r in rep),
                               "tune_s": round(getattr(eng.runner, "decode_gemm_tune_s", 0.0), 1),
                               "from_table": sum(r.get("source") == "table" for r in rep)}
    rep = getattr(eng.runner, "prefill_pf_report", None)
    if rep:  # start-up choice per (projection, row bucket): stream-K MFMA GEMM vs hipBLASLt
        pf = [r for r in rep if "code" not in r]
        fu = [r for r in rep if "code" in r]  # fused chain (llama.py _forward_pf): gemm_pf forms kept
        info["prefill_gemm"] = {"buckets": len(pf), "gemm_pf": sum(r["chosen"] != "hipblaslt" for r in pf),
                                "by_proj": {p: sum(r["chosen"] != "hipblaslt" for r in pf if r["proj"] == p)
                                            for p in sorted({r["proj"] for r in pf})},
                                "fused": {p: sum(r["chosen"].startswith("gemm_pf") for r in fu if r["proj"] == p)
                                          for p in sorted({r["proj"] for r in fu})},
                                "from_table": sum(r.get("source") == "table" for r in rep)}
    rep = getattr(eng.runner, "prefill_hblt_report", None)
    if rep:  # start-up choice per (projection, form, row bucket): a measured hipBLASLt solution vs its default
        info["prefill_hblt"] = {"buckets": len(rep), "tuned": sum(r["chosen"] != "default" for r in rep),
                                "by_proj": {f"{p}{'+resid' if rs else ''}": sum(r["chosen"] != "default" for r in rep
                                                                          if r["proj"] == p and r["resid"] == rs)
                                            for p, rs in sorted({(r["proj"], r["resid"]) for r in rep})},
                                "from_table": sum(r.get("source") == "table" for r in rep)}
    la = getattr(eng, "_late", None)
    if la is not None:  # engine/pacing.py: how often the host waited for a late admission, and how long
        info["late_admission"] = {"waits": la.waits, "mean_wait_ms": round(1e3 * la.wait_s / max(1, la.waits), 3),
                                  "model_updates": la.model.n, "host_lead_ms": round(1e3 * la.host_lead, 3),
                                  "late_wakes": la.late, "margin_ms": round(1e3 * la.margin, 3)}
    if eng.scheduler.chunk_budget is not None:
        info["chunk_budget"] = eng.scheduler.chunk_budget.stats()
    info["gc"] = gcs.summary()
    host = None
    if eng.step_times is not None and eng.step_times["steps"]:
        n = eng.step_times["steps"]
        host = {k: round(v / n * 1e3, 4) for k, v in eng.step_times.items() if k != "steps"}
    free_engine(eng, ctx)
    return ctx.gather(st), info, host


def phase_served(a, ctx, agg: dict, info: dict, guard) -> dict:
    """The engine-direct phase's workload through the served stack (mxserve/tools/served_phase.py),
    same QPS / ISL / OSL / engine limits, warm-up and window lengths; with the delta against the
    engine-direct numbers."""
    from mxserve.models.config import get_model_config
    from mxserve.tools import served_phase
    model = info["model"]
    isl, osl = info["isl"], info["osl"]
    flags = ["--max-num-seqs", str(a.max_num_seqs), "--max-num-batched-tokens", str(a.max_num_batched_tokens),
             "--max-model-len", str(a.max_model_len), "--seed", str(a.seed)]
    if a.itl_target_ms:
        flags += ["--itl-target-ms", str(a.itl_target_ms)]
    if a.kv_cache_dtype != "auto":
        flags += ["--kv-cache-dtype", a.kv_cache_dtype]
    if a.enforce_eager:
        flags.append("--enforce-eager")
    if a.num_gpu_blocks:
        flags += ["--num-gpu-blocks-override", str(a.num_gpu_blocks)]
    if not ctx.on_gpu:
        flags += ["--device", "cpu", "--num-gpu-blocks-override", "4096"]
    os.environ["MXS_CUDA_GRAPH_MAX_BS"] = str(a.max_num_seqs)  # the engine-direct phase's capture range
    window_s = agg["ms_per_step"] * a.steps / 1e3
    # the engine-direct warm-up ends once its running set is flat; the served stack starts from cold
    # processes and its running set was measured still growing through a window entered after the same
    # time (212 -> 447 requests), so it gets at least MXS_SERVED_MIN_WARMUP_S (two request lifetimes)
    warmup_s = max(float(agg.get("warmup_s") or 10.0),
                   float(os.environ.get("MXS_SERVED_MIN_WARMUP_S", "20")) if ctx.on_gpu else 0.0)
    vlog(f"served: warmup {warmup_s:.1f}s, window {window_s:.1f}s")
    log_dir = os.environ.get("MXS_BENCH_LOG_DIR", "")
    try:
        res = served_phase.run(model, a.qps, isl, osl, warmup_s, window_s, flags,
                               get_model_config(model).vocab_size, a.seed, ctx.on_gpu, guard.deadline - 20, log_dir,
                               guard.children)
    except Exception as e:  # noqa: BLE001 - the engine-direct line stands
        import traceback
        traceback.print_exc()
        return {"status": "failed", "error": repr(e)[:300]}
    if res.get("status") == "ok" and res.get("value"):
        res["vs_engine_direct"] = {"value_ratio": round(res["value"] / agg["value"], 4) if agg["value"] else None,
                                   "ttft_p50_delta_ms": round(res["ttft_p50_ms"] - agg["ttft_p50_ms"], 2)
                                   if res.get("ttft_p50_ms") is not None and agg.get("ttft_p50_ms") is not None
                                   else None,
                                   "itl_p50_delta_ms": round(res["itl_p50_ms"] - agg["itl_p50_ms"], 3)
                                   if res.get("itl_p50_ms") is not None and agg.get("itl_p50_ms") is not None
                                   else None}
        it = (res.get("worker_engine") or {}).get("iteration_ms")
        if it and res.get("itl_req_p50_ms") is not None:  # each running request gets one token per iteration
            res["itl_req_p50_vs_worker_iteration"] = round(res["itl_req_p50_ms"] / it, 3)
    vlog(f"served: {res}")
    return res


def phase_disagg(a, ctx) -> tuple:
    from mxserve.engine.engine import LLMEngine
    from mxserve.engine.request import SamplingParams
    world, rank = ctx.world, ctx.rank
    p, d, qps = disagg_plan(a, world)
    is_prefill = rank < p
    isl, osl = (a.isl, a.osl) if ctx.on_gpu else (min(a.isl, 200), min(a.osl, 20))
    a2 = argparse.Namespace(**{**vars(a), "isl": isl, "osl": osl})
    if is_prefill:  # prefill-only steps never replay decode graphs; no decode rows to pace, so the
        # largest steps (16384 tokens: ~128 req/s against ~120 at 8192, profiles/r3/s3/prefill_capacity)
        args = engine_args(a, ctx, disagg_mode="prefill", enforce_eager=True, itl_target_ms=0.0,
                           max_num_batched_tokens=max(a.max_num_batched_tokens, _PREFILL_STEP_TOKENS))
    else:
        mns = a.disagg_max_num_seqs
        args = engine_args(a, ctx, disagg_mode="decode", max_num_seqs=mns, cuda_graph_max_bs=mns)
    vlog("disagg: building engine")
    eng = LLMEngine(args)
    vlog(f"disagg: engine ready ({eng.runner.num_blocks} KV blocks)")
    conns = _disagg_conns(rank, p, world, ctx.gather)
    drv = None
    if not is_prefill:
        drv = Driver(a2, rank, eng.model_config.vocab_size, qps * world / d)  # the node's rate over D ranks
    hub = start_arrivals(a, ctx, list(range(p, world)), qps * world, isl, eng.model_config.vocab_size, eng, drv)
    if is_prefill:
        run_disagg_prefill(eng, a.temperature, ctx.barrier, conns)
        st = list(_STAT_NAN)
    else:
        sp = SamplingParams(max_tokens=osl, temperature=a.temperature, ignore_eos=True)
        agree = ctx.agree_fn(ctx.pg_decode, d)
        st = drv.stats(run_disagg_decode(a2, eng, sp, drv, ctx.barrier, agree, conns))
    arrivals = finish_arrivals(hub, drv)
    for c in conns:
        c.close()
    info = {"arrivals": arrivals or {"mode": "local" if d > 1 else "single decode rank"},"decode_max_num_seqs": a.disagg_max_num_seqs, "prefill_ranks": p, "decode_ranks": d,
            "qps_per_gpu": round(qps, 2), "qps_node": round(qps * world, 2),
            "qps_per_decode_rank": round(qps * world / d, 2)}
    free_engine(eng, ctx)
    return ctx.gather(st), info


def main():
    a = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and a.gpus > 1:
        return launch_ranks(a)
    world = int(world_env or "1")
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; run `python bench.py --gpus N` "
                         "(it spawns the ranks) or launch exactly N ranks")
    mode = a.mode if a.mode != "auto" else ("agg" if world == 1 else "both")
    if mode in ("disagg", "both") and world < 2:
        raise SystemExit("bench.py: the disagg phase needs at least 2 GPUs (prefill and decode ranks)")
    guard = Guard(a.time_budget_s, int(os.environ.get("RANK", "0"))).arm()
    # the disagg phase runs in the crash-isolated probe processes unless the probe is off
    host_disagg = mode in ("disagg", "both") and a.probe_timeout_s > 0
    probe = start_probe(a, world, guard, host_disagg)  # before Ctx: nothing here has touched the GPU yet
    ctx = Ctx(a)

    agg = dis = info = None
    if mode in ("agg", "both"):
        col, info, host = phase_agg(a, ctx)
        agg = summarize(col, a.steps, list(range(world)))
        if host and ctx.rank == 0:
            print(json.dumps({"host_ms_per_step": host}), file=sys.stderr, flush=True)
        if ctx.rank == 0:  # provisional: what the watchdog prints if the rest runs out of time
            line = build_line(a, ctx, mode, agg, None, info)
            if mode == "both":
                line["disagg"] = {"status": "pending"}
            if probe is not None:
                line["multi_gpu_probe"] = {"status": "pending"}
            guard.pending = line
            vlog(f"agg done: {agg['value']} tok/s; {guard.remaining():.0f}s of the budget left")
    if agg is not None and world == 1 and a.served:
        served = phase_served(a, ctx, agg, info, guard)
        if ctx.rank == 0:
            guard.pending = dict(guard.pending or {}, served=served)
    if mode in ("disagg", "both") and not host_disagg:
        dis = run_guarded(lambda: phase_disagg(a, ctx), min(a.phase_timeout_s, max(1.0, guard.remaining() - 15)),
                          ctx, agg_info=info, agg=agg, a=a, mode=mode, guard=guard)
        dis = disagg_summary(*dis, a, world)
    probe_res = finish_probe(probe, guard, ctx)
    if host_disagg and ctx.rank == 0:
        r = probe_res.pop("disagg_headline", None) if isinstance(probe_res, dict) else None
        if isinstance(r, dict) and "col" in r:
            dis = disagg_summary(np.array(r["col"], dtype=np.float64), r["info"], a, world)
            dis["ran_in"] = "probe processes (crash-isolated)"
        else:
            src = r or probe_res or {}
            err = src.get("error", "no result from the probe processes")
            dis = {"status": "failed", "error": err}
            if src.get("where"):
                dis.update(where=src["where"], rank=src.get("rank"))
            if agg is None:
                raise SystemExit(f"bench.py: disagg phase failed: {err}")
    if mode in ("disagg", "both") and agg is None:
        info = {"kv_blocks": None, "graphs": [], "preemptions": None, "model": a.model,
                "kv_cache_dtype": "bf16", "isl": a.isl, "osl": a.osl}
    if ctx.rank == 0:
        line = build_line(a, ctx, mode, agg, dis, info)
        if isinstance(guard.pending, dict) and "served" in guard.pending:
            line["served"] = guard.pending["served"]
        if probe_res is not None:
            line["multi_gpu_probe"] = probe_res
        line["wall_s"] = round(time.time() - _WALL0, 1)
        guard.emit(line)
    if world > 1:
        if probe is None:  # with a probe, ranks > 0 left at finish_probe: no final barrier
            ctx.dist.barrier()
        ctx.dist.destroy_process_group()
    return 0


def disagg_summary(col_d: np.ndarray, info_d: dict, a, world: int) -> dict:
    p_d = info_d["prefill_ranks"]
    dis = summarize(col_d, a.steps, list(range(p_d, world)))
    dis.update(info_d, parallelism=f"disagg {p_d}P+{world - p_d}D")
    if col_d.shape[1] >= 11 + len(BREAKDOWN_KEYS):  # median over decode ranks of their per-request p50s
        bd = col_d[p_d:, 11:11 + len(BREAKDOWN_KEYS)]
        dis["ttft_breakdown_p50_ms"] = {k: (round(float(np.nanmedian(bd[:, i])) * 1e3, 2)
                                            if not np.all(np.isnan(bd[:, i])) else None)
                                        for i, k in enumerate(BREAKDOWN_KEYS)}
    return dis


def compare_modes(agg: dict, dis: dict, agg_qps: float) -> dict:
    """Agg vs disagg on the same node: the arrival rate each ran at (like-for-like when equal) and
    which mode is better on each serving metric."""
    keys = (("value", True), ("ttft_p50_ms", False), ("ttft_p90_ms", False), ("itl_p50_ms", False),
            ("itl_p90_ms", False))
    out = {"qps_per_gpu": {"agg": agg_qps, "disagg": dis.get("qps_per_gpu")},
           "like_for_like": dis.get("qps_per_gpu") is not None and abs(float(dis["qps_per_gpu"]) - agg_qps) < 0.01}
    for k, higher in keys:
        va, vd = agg.get(k), dis.get(k)
        if va is None or vd is None:
            continue
        out[k] = {"agg": va, "disagg": vd, "better": ("agg" if (va > vd) == higher else "disagg") if va != vd else "tie"}
    return out


def build_line(a, ctx, mode, agg, dis, info) -> dict:
    head = agg if agg is not None else dis
    world = ctx.world
    on_gpu = ctx.on_gpu
    model = info["model"] if on_gpu else a.model
    metric = BASELINE_METRIC
    if model != "meta-llama/Llama-3.2-1B-Instruct":  # a labelled side data point, not the headline
        metric = BASELINE_METRIC.replace("Llama-3.2-1B", model.split("/")[-1])
    line = {
        "metric": metric,
        "value": head["value"],
        "unit": "tok/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": head["ms_per_step"],
        "engine_iterations_per_step": a.iters_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if on_gpu else "fp32",
        "data": "synthetic (random prompt token ids, random-init weights, Poisson arrivals)",
        "config": {"model": info["model"] if on_gpu else "tiny-llama (CPU plumbing run)",
                   "global_batch": int(world * a.max_num_seqs), "seq_len": info["isl"] + info["osl"],
                   "parallelism": f"dp{world}" if agg is not None else (dis or {}).get("parallelism", "disagg"),
                   "mode": mode, "isl": info["isl"], "osl": info["osl"],
                   "qps_per_gpu": a.qps, "qps_node": a.qps * world, "kv_cache_dtype": info["kv_cache_dtype"],
                   "shared_gpu": ctx.shared_gpu, "max_num_batched_tokens": a.max_num_batched_tokens,
                   "itl_target_ms": a.itl_target_ms or None},
    }
    for k in ("ttft_p50_ms", "ttft_p90_ms", "itl_p50_ms", "itl_p90_ms", "requests_with_first_token",
              "warmup_steps_executed", "warmup_s", "steady_state", "running_mean", "sla_isl4000_osl500"):
        line[k] = head[k]
    line["ttft_window"] = "steady state: post-warmup soak + timed steps"
    if on_gpu:  # where the default rate sits (measured, one MI355X per rank; profiles/r5/qps_sweep/)
        line["operating_point"] = {"qps_per_gpu": a.qps, "measured_saturation_qps_per_gpu": SATURATION_QPS,
                                   "headroom": round(1.0 - a.qps / SATURATION_QPS, 3),
                                   "sweep": SATURATION_SWEEP}
    if agg is not None and dis is not None:
        line["agg"] = {k: agg[k] for k in ("value", "ttft_p50_ms", "itl_p50_ms", "ms_per_step")}
        line["agg_vs_disagg"] = compare_modes(agg, dis, a.qps)
    if dis is not None:
        line["disagg"] = dis
    line["per_rank"] = head.get("per_rank")
    if "arrivals" in info:
        line["arrivals"] = info["arrivals"]
    line["engine"] = {"kv_blocks": info["kv_blocks"], "preemptions": info["preemptions"], "graphs": info["graphs"]}
    for k in ("late_admission", "decode_gemm", "prefill_gemm", "prefill_hblt", "chunk_budget", "gc"):
        if k in info:
            line["engine"][k] = info[k]
    return line


def run_guarded(fn, timeout_s: float, ctx, **kw):
    """Run a phase with a watchdog: if it has not returned by timeout_s (e.g. an IPC mapping that
    never completes across GPUs), rank 0 prints the line it has, marking the phase failed, and
    every rank exits instead of hanging the job."""
    done = threading.Event()

    guard = kw["guard"]

    def watchdog():
        if done.wait(timeout_s):
            return
        if ctx.rank == 0 and kw.get("agg") is not None:
            line = build_line(kw["a"], ctx, kw["mode"], kw["agg"], None, kw["agg_info"])
            line["disagg"] = {"status": "failed", "error": f"phase did not finish within {timeout_s:.0f}s"}
            guard.emit(line)
        print(f"bench.py rank {ctx.rank}: disagg phase timed out after {timeout_s:.0f}s", file=sys.stderr, flush=True)
        guard.kill_children()
        os._exit(0 if kw.get("agg") is not None else 3)

    threading.Thread(target=watchdog, daemon=True).start()
    try:
        return fn()
    except BaseException as e:  # noqa: BLE001 - one rank failing must not hang the others in a barrier
        import traceback
        traceback.print_exc()
        if kw.get("agg") is None:
            raise
        if ctx.rank == 0:
            line = build_line(kw["a"], ctx, kw["mode"], kw["agg"], None, kw["agg_info"])
            line["disagg"] = {"status": "failed", "error": repr(e)[:300]}
            guard.emit(line)
        guard.kill_children()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    finally:
        done.set()


if __name__ == "__main__":
    sys.exit(main())
