"""Late admission for async scheduling.

With async scheduling the host schedules and launches step N+1 while the GPU runs step N, so the
GPU never waits for the host.  Launched right after step N, step N+1 is fixed before most of step N's
GPU time has passed: a request that arrives during step N misses N+1 and is prefilled in N+2, one
whole step later than it could be.  At the headline point (Llama-3.2-1B, QPS 42) that step is about
a quarter of the p50 TTFT.

Late admission keeps the GPU queue full but schedules N+1 as LATE as possible: it predicts when the
GPU will finish step N, sleeps (releasing the GIL) until the host's schedule + launch time before
that, admits whatever arrived meanwhile, then schedules and launches N+1.  If step N turns out to be
done earlier (its completion event fires), it proceeds at once.

The prediction is an online exponentially weighted least-squares fit of a step's GPU time on its
composition (prefill tokens, prefill attention work, decode rows, decode context), from completion
times observed whenever the host sees a step finish (see LLMEngine._step).
"""
from __future__ import annotations

import math
import os
import time
from typing import Optional

import numpy as np

try:  # imported with the engine: a first import inside the step loop (the 24th observed step, when the
    # model is first fitted) held the host ~300-400 ms while the GPU queue drained (scripts/
    # prefill_capacity_probe.py: one 330-400 ms step at engine step 25 whatever the step size)
    from scipy.optimize import nnls as _nnls
except Exception:  # noqa: BLE001 - no scipy: no constrained fit
    _nnls = None

NF = 5


def step_features(so) -> np.ndarray:
    """[1, prefill tokens, prefill attention work, decode rows, decode context tokens], scaled."""
    p = pa = 0.0
    for s in so.prefills:
        n = s.num_new_tokens
        p += n
        pa += n * (s.start + 0.5 * n)
    dctx = 0.0
    for s in so.decodes:
        dctx += s.start
    return np.array([1.0, p / 1e3, pa / 1e7, len(so.decodes) / 1e2, dctx / 1e5])


def nonneg_fit(A: np.ndarray, b: np.ndarray) -> Optional[np.ndarray]:
    """argmin_{theta >= 0} theta' A theta - 2 b' theta for the normal equations (A = X'X, b = X'y):
    with A = L L' that is the non-negative least squares problem ||L' theta - L^-1 b||."""
    if _nnls is None:
        return None
    try:
        L = np.linalg.cholesky(A + 1e-9 * np.eye(A.shape[0]))
        theta, _ = _nnls(L.T, np.linalg.solve(L, b))
        return theta
    except Exception:  # noqa: BLE001 - no scipy / not positive definite: no constrained fit
        return None


class StepTimeModel:
    def __init__(self, lam: float = 0.98, warmup: int = 24, nf: int = NF):
        self.lam = lam
        self.warmup = warmup
        self.nf = nf
        self.A = np.eye(nf) * 1e-6
        self.b = np.zeros(nf)
        self.theta: Optional[np.ndarray] = None
        # the same fit with every coefficient >= 0 (a step cannot get faster with more work): prefill
        # tokens and prefill attention work move together, so the unconstrained fit can trade one
        # for the other with a negative sign, which is harmless for predicting a whole step but not
        # for pricing a chunk of a given size (ChunkBudget)
        self.theta_nn: Optional[np.ndarray] = None
        self.n = 0

    def update(self, x: np.ndarray, seconds: float) -> None:
        if not (0.0 < seconds < 5.0):
            return
        self.A = self.lam * self.A + np.outer(x, x)
        self.b = self.lam * self.b + x * seconds
        self.n += 1
        if self.n >= self.warmup and (self.n < 200 or self.n % 8 == 0):
            try:
                self.theta = np.linalg.solve(self.A + 1e-9 * np.eye(self.nf), self.b)
            except np.linalg.LinAlgError:
                self.theta = None
            self.theta_nn = nonneg_fit(self.A, self.b)

    def predict(self, x: np.ndarray) -> Optional[float]:
        if self.theta is None:
            return None
        return max(0.0, float(x @ self.theta))


class ChunkBudget:
    """Decode-aware prefill chunk budget (--itl-target-ms).

    A fixed token budget (max_num_batched_tokens) makes a step that carries a prefill chunk as long
    as the decode rows plus the whole chunk: at 250 decode rows and an 8192-token chunk that step,
    and so every running request's inter-token latency, is ~2.5x a decode-only step.  With a target
    the scheduler prices the step's decode rows and gives prefill chunks only the time left.

    Two non-negative least-squares models, fed with each step's GPU time (runner events):
      * decode: [1, decode rows, decode context] fitted on decode-only steps;
      * prefill: [1, prefill tokens, prefill attention work] fitted on what a mixed step took beyond
        the decode model's price for its decode rows (the constant is the mixed step's fixed extra:
        eager launch, MoE weights streamed again).
    Kept apart because in a loaded closed loop nearly every step carries both, and one joint fit
    then cannot tell decode cost from prefill cost (it settles on pricing prefill tokens at the whole
    step's time and starves prefill).  Guards: the first chunk of a step always gets `min_tokens`;
    when the oldest waiting request has waited `ttft_guard_s` the step is not limited at all, so an
    overloaded worker trades ITL back for TTFT instead of queueing without bound.  Until both models
    are fitted no limit applies.
    """

    def __init__(self, target_ms: float, min_tokens: int = 256, align: int = 64, ttft_guard_s: float = 0.5):
        self.dec = StepTimeModel(nf=3)
        self.pre = StepTimeModel(nf=3)
        self.target = float(target_ms) / 1e3
        self.min_tokens = int(min_tokens)
        self.align = int(align)
        self.ttft_guard_s = float(ttft_guard_s)
        self.steps = 0  # steps that planned with fitted models
        self.limited = 0  # prefill chunks cut short by the budget
        self.cut_tokens = 0
        self.guard_lifts = 0  # steps left unlimited because a request waited too long

    @staticmethod
    def _dec_x(nd: float, dctx: float) -> np.ndarray:
        return np.array([1.0, nd / 1e2, dctx / 1e5])

    def observe(self, x: np.ndarray, seconds: float) -> None:
        """A step of composition x (step_features) took `seconds` of GPU time."""
        if not (0.0 < seconds < 5.0):
            return
        xd = np.array([1.0, x[3], x[4]])
        if x[1] <= 0.0:
            self.dec.update(xd, seconds)
            return
        th = self.dec.theta_nn
        if th is None:
            return
        self.pre.update(np.array([1.0, x[1], x[2]]), seconds - float(xd @ th))

    def begin(self, running, waiting=None) -> Optional[float]:
        """Seconds left for prefill work in the next step (None = no limit)."""
        td, tp = self.dec.theta_nn, self.pre.theta_nn
        if td is None or tp is None or tp[1] + tp[2] <= 0.0:
            return None
        if waiting and time.monotonic() - waiting[0].arrival_time > self.ttft_guard_s:
            self.guard_lifts += 1
            return None
        nd = 0
        dctx = 0
        for r in running:
            c = r.num_computed_tokens
            if r.num_tokens - c == 1 and c >= r.num_prompt_tokens:
                nd += 1
                dctx += c
        self.steps += 1
        return self.target - float(self._dec_x(nd, dctx) @ td) - tp[0]

    def fit(self, left: float, start: int, want: int, first: bool) -> tuple:
        """Largest chunk <= want (tokens from position `start`) whose predicted cost fits in
        `left` seconds; returns (tokens, seconds)."""
        th = self.pre.theta_nn
        c1 = th[1] / 1e3  # s per prefill token
        c2 = max(0.0, th[2] / 1e7)  # s per token x context token (attention)
        b = max(c1 + c2 * start, 1e-9)
        a = 0.5 * c2
        if left <= 0.0:
            n = 0
        elif a > 0.0:
            n = int((-b + math.sqrt(b * b + 4.0 * a * left)) / (2.0 * a) + 1e-6)
        else:
            n = int(left / b + 1e-6)
        if n < want:
            if n > self.align:
                n -= n % self.align
            if first:
                n = max(n, self.min_tokens)
            n = min(n, want)
            if n < want:
                self.limited += 1
                self.cut_tokens += want - n
        else:
            n = want
        return n, n * (b + a * n)

    def stats(self) -> dict:
        ms = lambda t: None if t is None else [round(1e3 * float(v), 4) for v in t]  # noqa: E731
        return {"target_ms": round(self.target * 1e3, 2), "planned_steps": self.steps, "limited_chunks": self.limited,
                "cut_tokens": self.cut_tokens, "guard_lifts": self.guard_lifts,
                "decode_updates": self.dec.n, "prefill_updates": self.pre.n,
                # fitted costs: decode ms per step / per 100 rows / per 1e5 context tokens; prefill ms
                # per mixed step (fixed extra) / per 1k tokens / per 1e7 token x context
                "decode_ms": ms(self.dec.theta_nn), "prefill_ms": ms(self.pre.theta_nn)}


class LateAdmission:
    """Per-engine state: the in-flight step's launch time, predicted completion and features."""

    def __init__(self):
        self.model = StepTimeModel()
        self.host_lead = 1.5e-3  # EMA of admit -> launched host time
        # slack for the prediction error: admitting this much earlier than the host lead requires
        self.margin = float(os.environ.get("MXS_LATE_ADMISSION_MARGIN_MS", "1.5")) / 1e3
        self.margin_min = self.margin
        self.late = 0  # waits the step outlasted (GPU done before the host admitted)
        self.inflight: Optional[dict] = None  # {"x", "t_launch", "est_done", "done"}
        self.last_done: Optional[float] = None  # observed completion of the previous step
        self.waits = 0
        self.wait_s = 0.0

    def wait(self, ev) -> None:
        """Sleep until the in-flight step is predicted to be a host-lead away from done (or done)."""
        st = self.inflight
        if st is None or st["est_done"] is None:
            return
        target = st["est_done"] - self.host_lead - self.margin
        t0 = now = time.perf_counter()
        if ev is not None and ev.query():  # already done when we looked: completion time unknown
            return
        finished = False
        while now < target:
            if ev is not None and ev.query():  # seen finishing: a completion time within one poll
                st["done"] = now
                finished = True
                break
            time.sleep(min(2e-4, target - now))
            now = time.perf_counter()
        # margin control (AIMD): the GPU finishing before the host admits means it idles for the
        # host's schedule + launch time -- widen the slack at once; shrink it slowly while on time
        if finished or (ev is not None and ev.query()):
            self.late += 1
            self.margin = min(self.margin + 5e-4, 8e-3)
        else:
            self.margin = max(self.margin - 2e-5, self.margin_min)
        self.waits += 1
        self.wait_s += time.perf_counter() - t0

    def launched(self, so, t_admit: float, t_launched: float, t_begin: Optional[float] = None) -> None:
        """t_begin: when the host started enqueueing the step.  Its GPU work starts from then (the first
        kernels run while the host still enqueues the rest: an eager Mixtral prefill step takes tens of
        ms to launch), so a step's GPU time is measured from there, not from the end of the launch."""
        self.host_lead = 0.9 * self.host_lead + 0.1 * (t_launched - t_admit)
        x = step_features(so)
        est = self.model.predict(x)
        t0 = t_launched if t_begin is None else t_begin
        prev = self.inflight
        start = t0
        if prev is not None and prev.get("est_done") is not None:
            start = max(start, prev["est_done"])
        self.pending_next = {"x": x, "t_launch": t0, "est_done": None if est is None else start + est,
                             "done": None}

    def rotate(self) -> None:
        """The launched step becomes the in-flight one (called once per engine step)."""
        self.inflight, self.pending_next = getattr(self, "pending_next", None), None

    def observe_done(self, st: Optional[dict], t_done: Optional[float], gpu_s: Optional[float] = None) -> None:
        """A step completed at t_done (None: not observed precisely).  gpu_s: its GPU time from the
        runner's events (start marker -> end marker), which the model then fits on directly;
        without it the GPU time is taken to run from the later of its launch and the previous
        step's completion (host clocks: steps whose neighbours' completions were not seen drop out)."""
        if st is None:
            return
        if gpu_s is not None:
            self.model.update(st["x"], gpu_s)
        if t_done is not None:
            if self.last_done is not None and gpu_s is None:
                begin = max(st["t_launch"], self.last_done)
                self.model.update(st["x"], t_done - begin)
            # re-anchor the step now in flight on this observed completion (it was queued behind it)
            cur = self.inflight
            if cur is not None and cur is not st:
                est = self.model.predict(cur["x"])
                if est is not None:
                    cur["est_done"] = max(cur["t_launch"], t_done) + est
        self.last_done = t_done
