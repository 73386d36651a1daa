"""Decode-aware prefill chunk budget (engine/pacing.py ChunkBudget, --itl-target-ms): the scheduler
caps prefill chunks so a step's predicted time stays under the target, always gives the first
chunk of a step its minimum, and leaves decodes alone.  CPU only."""
import numpy as np
import pytest

from mxserve.engine.kv_manager import KVCacheManager
from mxserve.engine.pacing import ChunkBudget, StepTimeModel, step_features
from mxserve.engine.request import Request, SamplingParams
from mxserve.engine.scheduler import Scheduler


def _budget(target_ms, dec=(2e-3, 4e-3, 0.0), pre=(0.0, 2e-3, 0.0)):
    """A ChunkBudget with fitted models: decode [per step, per 100 rows, per 1e5 context] and prefill
    [fixed extra per mixed step, per 1k tokens, per 1e7 token x context] costs in seconds."""
    cb = ChunkBudget(target_ms)
    cb.dec.theta_nn = np.asarray(dec, dtype=float)
    cb.pre.theta_nn = np.asarray(pre, dtype=float)
    return cb


# 2 ms per step, 4 ms per 100 decode rows; prefill 2 ms per 1000 tokens, no attention term
THETA = [2e-3, 2e-3, 0.0, 4e-3, 0.0]


def _req(i, n_prompt):
    return Request(f"r{i}", list(range(1, n_prompt + 1)), SamplingParams(max_tokens=64, ignore_eos=True))


def _sched(target_ms, pre=(0.0, 2e-3, 0.0), budget=8192):
    s = Scheduler(KVCacheManager(4096, 16, False), max_num_seqs=256, max_num_batched_tokens=budget,
                  max_model_len=8192)
    if target_ms:
        s.chunk_budget = _budget(target_ms, pre=pre)
    return s


def _to_decode(s, n):
    """n requests that have finished their prefill and sit in the running batch as decodes."""
    cb, s.chunk_budget = s.chunk_budget, None
    for i in range(n):
        s.add(_req(1000 + i, 32))
    so = s.schedule()
    s.update(so, {x.req.request_id: 5 for x in so.all() if x.sample})
    s.chunk_budget = cb
    assert all(r.num_computed_tokens >= r.num_prompt_tokens for r in s.running)


def test_no_target_uses_token_budget():
    s = _sched(0)
    s.add(_req(0, 6000))
    so = s.schedule()
    assert so.prefills[0].num_new_tokens == 6000


def test_budget_caps_prefill_chunk():
    s = _sched(20.0)
    s.add(_req(0, 6000))
    so = s.schedule()
    # 20 ms - 2 ms intercept = 18 ms at 2 us/token -> 9000 tokens: whole prompt fits
    assert so.prefills[0].num_new_tokens == 6000
    s = _sched(10.0)
    s.add(_req(0, 6000))
    so = s.schedule()
    # 8 ms / 2 us = 4000 tokens, rounded down to a multiple of 64
    assert so.prefills[0].num_new_tokens == 3968
    assert s.chunk_budget.limited == 1 and s.chunk_budget.cut_tokens == 2032


def test_decodes_take_their_share_first():
    s = _sched(10.0)
    _to_decode(s, 100)  # 100 decode rows: 4 ms
    s.add(_req(0, 6000))
    so = s.schedule()
    assert len(so.decodes) == 100
    # 10 - 2 - 4 = 4 ms -> 2000 tokens -> 1984
    assert so.prefills[0].num_new_tokens == 1984
    x = step_features(so)
    assert float(x @ np.asarray(THETA)) <= 10e-3 + 1e-9


def test_first_chunk_gets_minimum_when_decode_exceeds_target():
    s = _sched(5.0)
    _to_decode(s, 100)  # decode alone: 6 ms > 5 ms
    s.add(_req(0, 6000))
    s.add(_req(1, 3000))
    so = s.schedule()
    assert len(so.decodes) == 100
    assert [p.num_new_tokens for p in so.prefills] == [256]  # min_tokens, and the second waits


def test_running_chunked_prefill_continues_under_budget():
    s = _sched(10.0)
    s.add(_req(0, 8000))
    first = s.schedule()
    assert first.prefills[0].num_new_tokens == 3968
    s.update(first, {})
    second = s.schedule()
    assert second.prefills[0].start == 3968 and second.prefills[0].num_new_tokens == 3968


def test_attention_term_shrinks_late_chunks():
    # attention 1 ms per 1e7 token*context: a chunk deep into a long prompt costs more per token
    cb = _budget(10.0, pre=(0.0, 2e-3, 1e-3))
    n0, c0 = cb.fit(8e-3, 0, 8000, True)
    n1, c1 = cb.fit(8e-3, 6000, 8000, True)
    assert n1 < n0
    assert c0 <= 8e-3 + 1e-9 and c1 <= 8e-3 + 1e-9


def test_unfitted_or_degenerate_model_means_no_limit():
    s = _sched(10.0, pre=(0.0, 0.0, 0.0))
    s.add(_req(0, 6000))
    assert s.schedule().prefills[0].num_new_tokens == 6000
    s = _sched(0)
    s.chunk_budget = ChunkBudget(10.0)  # not fitted yet
    s.add(_req(0, 6000))
    assert s.schedule().prefills[0].num_new_tokens == 6000


def test_engine_wires_target_from_args(monkeypatch):
    """The engine builds the budget from --itl-target-ms and feeds it every step's time.  The fed
    values are wall times of CPU steps, which a loaded test box can stretch past the model's
    5-second outlier cut, so the test checks the calls (a spy), not the fitted model."""
    from mxserve.config import EngineArgs
    from mxserve.engine.engine import LLMEngine
    from mxserve.engine.pacing import ChunkBudget
    seen = []
    orig = ChunkBudget.observe
    monkeypatch.setattr(ChunkBudget, "observe", lambda self, x, sec: (seen.append((tuple(x), sec)), orig(self, x, sec)))
    eng = LLMEngine(EngineArgs(model="tiny-llama", device="cpu", cpu_num_blocks=256, max_model_len=512,
                               itl_target_ms=50.0, async_scheduling=False))
    assert eng.scheduler.chunk_budget is not None
    sp = SamplingParams(max_tokens=4, ignore_eos=True)
    outs = eng.generate([list(range(1, 40)) for _ in range(30)], sp)
    assert all(len(o) == 4 for o in outs)
    assert len(seen) >= 4  # one prefill step and the decode steps, each with its time
    assert any(x[1] > 0 for x, _ in seen) and any(x[1] == 0 and x[3] > 0 for x, _ in seen)
    assert all(sec > 0 for _, sec in seen)
    # the decode-only observations reach the decode model whenever they pass its outlier cut
    cb = eng.scheduler.chunk_budget
    assert cb.dec.n == sum(1 for x, sec in seen if x[1] <= 0 and 0 < sec < 5.0)
    assert eng.stats()["chunk_budget"]["target_ms"] == 50.0


def test_cli_flag():
    from mxserve.worker.args import parse_worker_args
    wa = parse_worker_args(["--model", "tiny-llama", "--itl-target-ms", "25"])
    assert wa.engine.itl_target_ms == 25.0


def test_nonneg_fit_on_collinear_steps():
    """Prefill tokens and prefill attention work move together in real traffic; the constrained fit
    keeps every coefficient >= 0 and still predicts the steps."""
    rng = np.random.default_rng(0)
    m = StepTimeModel()
    true = np.array([3e-3, 2.5e-3, 0.4e-3, 4e-3, 1e-3])
    for _ in range(400):
        p = rng.choice([0, 0, 8192, 4096]) + rng.integers(0, 64)
        start = rng.integers(0, 4000)
        x = np.array([1.0, p / 1e3, p * (start + p / 2) / 1e7, rng.integers(50, 300) / 1e2,
                      rng.integers(50, 300) * 4000 / 1e5])
        m.update(x, float(x @ true) * (1 + 0.02 * rng.standard_normal()))
    assert m.theta_nn is not None and (m.theta_nn >= 0).all()
    x = np.array([1.0, 8.192, 8192 * 6096 / 1e7, 2.0, 8.0])
    assert abs(float(x @ m.theta_nn) - float(x @ true)) < 0.05 * float(x @ true)


def test_step_time_measured_from_launch_start():
    """A long eager step starts on the GPU while the host still enqueues it: its measured time runs
    from the start of the launch (not the end), else the model sees a 100 ms prefill step as a few ms."""
    from types import SimpleNamespace
    from mxserve.engine.pacing import LateAdmission
    la = LateAdmission()
    seen = []
    la.model.update = lambda x, s: seen.append(s)
    so = SimpleNamespace(prefills=[SimpleNamespace(num_new_tokens=8000, start=0)], decodes=[])
    la.last_done = 0.0
    la.launched(so, t_admit=0.0, t_launched=0.060, t_begin=0.001)  # 59 ms to enqueue
    la.rotate()
    la.observe_done(la.inflight, 0.101)
    assert seen and abs(seen[0] - 0.100) < 1e-9


def test_step_time_from_gpu_events_preferred():
    """With the runner's event-measured GPU time the model fits on it, even when the host saw
    neither this step's nor the previous step's completion."""
    from types import SimpleNamespace
    from mxserve.engine.pacing import LateAdmission
    la = LateAdmission()
    seen = []
    la.model.update = lambda x, s: seen.append(s)
    so = SimpleNamespace(prefills=[SimpleNamespace(num_new_tokens=8000, start=0)], decodes=[])
    la.launched(so, t_admit=0.0, t_launched=0.02, t_begin=0.0)
    la.rotate()
    la.observe_done(la.inflight, None, gpu_s=0.095)
    assert seen == [0.095]


def test_separate_models_survive_all_mixed_steps():
    """Decode cost is learned from decode-only steps and kept when (under load) every later step
    carries a chunk; prefill cost is fitted on what mixed steps take beyond it, so a chunk's price is
    per-token prefill work, not the whole step's time (the joint-fit failure that starved prefill)."""
    rng = np.random.default_rng(1)
    cb = ChunkBudget(40.0)

    def step(nd, p, start=0):
        x = np.array([1.0, p / 1e3, p * (start + p / 2) / 1e7, nd / 1e2, nd * 4200 / 1e5])
        t = 0.024 + 0.0001 * nd + ((0.004 + 0.012 * p / 1e3) if p else 0.0)  # Mixtral-like
        return x, t * (1 + 0.01 * rng.standard_normal())

    for _ in range(60):  # decode-only warmup
        cb.observe(*step(rng.integers(60, 90), 0))
    for _ in range(300):  # loaded: every step mixed
        cb.observe(*step(rng.integers(60, 90), rng.integers(300, 2000), rng.integers(0, 3000)))
    assert cb.dec.theta_nn is not None and cb.pre.theta_nn is not None
    assert abs(cb.pre.theta_nn[1] - 0.012) < 0.003, cb.pre.theta_nn  # ~12 ms per 1k tokens
    left = cb.begin([], [])
    n, cost = cb.fit(left, 0, 8192, True)
    assert 500 < n < 1200, n  # (40 - ~32 decode - ~4 extra) ms at ~12 ms / 1k tokens


def test_ttft_guard_lifts_the_limit():
    import time as _t
    s = _sched(10.0)
    old = _req(0, 6000)
    s.add(old)
    old.arrival_time = _t.monotonic() - 5.0  # waited far longer than the guard
    so = s.schedule()
    assert so.prefills[0].num_new_tokens == 6000
    assert s.chunk_budget.guard_lifts == 1


def test_nnls_imported_with_the_module():
    """The first constrained fit must not import scipy inside the step loop (a 330-400 ms host stall at
    engine step 25 that drained the GPU queue): the solver is bound when pacing is imported."""
    import importlib.util

    from mxserve.engine import pacing
    if importlib.util.find_spec("scipy") is None:
        assert pacing._nnls is None
        return
    assert pacing._nnls is not None
    import sys
    mods = set(sys.modules)
    m = pacing.StepTimeModel(nf=3, warmup=2)
    for k in range(4):
        m.update(np.array([1.0, k, k * k]), 0.01 + 0.002 * k)
    assert m.theta_nn is not None
    assert not {x for x in set(sys.modules) - mods if x.startswith("scipy")}
