"""Unit tests: native block pool / hashing / KV indexer, scheduler (chunked prefill, prefix caching,
preemption, invariants), router cost, tokenizer + chat templates, worker flag dialects, SLA planner."""
import random

import pytest

from mxserve import _native
from mxserve.engine.kv_manager import KVCacheManager
from mxserve.engine.request import Request, SamplingParams, Status
from mxserve.engine.scheduler import Scheduler

rt = _native.rt()


# ----------------------------------------------------------------------------- block pool
def test_block_pool_alloc_free_evict():
    p = rt.BlockPool(8, True)
    a = p.allocate(5)
    assert len(set(a)) == 5 and p.num_free() == 3
    with pytest.raises(RuntimeError):
        p.allocate(4)
    p.cache_blocks(a[:2], [11, 22])
    p.free(list(reversed(a)))
    assert p.num_free() == 8 and p.check_invariants()
    hit = p.get_cached_prefix([11, 22, 33])
    assert hit == a[:2] and p.ref_count(a[0]) == 1
    with pytest.raises(RuntimeError):
        p.free([a[4]])  # already free -> double free detected
    p.free(hit)
    # eviction: allocating everything drops the cached hashes
    p.allocate(8)
    assert p.num_cached() == 0
    stored, removed = p.take_events()
    assert stored == [11, 22] and sorted(removed) == [11, 22]
    assert p.check_invariants()


def test_block_pool_random_ops_invariants():
    rng = random.Random(0)
    p = rt.BlockPool(64, True)
    held = []
    for step in range(3000):
        op = rng.random()
        if op < 0.4 and p.num_free() > 0:
            n = rng.randint(1, min(4, p.num_free()))
            blocks = p.allocate(n)
            hs = [rng.randint(1, 200) for _ in blocks]
            p.cache_blocks(blocks, hs)
            held.append(blocks)
        elif op < 0.7 and held:
            p.free(held.pop(rng.randrange(len(held))))
        else:
            hit = p.get_cached_prefix([rng.randint(1, 200) for _ in range(3)])
            if hit:
                held.append(hit)
        if step % 97 == 0:
            assert p.check_invariants()
    assert p.check_invariants()


def test_block_hashes_chained_and_stable():
    toks = list(range(100))
    h = rt.block_hashes(toks, 16)
    assert len(h) == 6
    assert rt.block_hashes(toks[:48], 16) == h[:3]  # prefix property
    other = toks[:]
    other[20] = 999
    h2 = rt.block_hashes(other, 16)
    assert h2[0] == h[0] and all(a != b for a, b in zip(h2[1:], h[1:]))  # chained
    assert rt.block_hashes(toks, 16, 0, 0) == h


def test_kv_indexer():
    ix = rt.KvIndexer()
    h = rt.block_hashes(list(range(64)), 16)
    ix.apply_stored(0, h[:4])
    ix.apply_stored(3, h[:2])
    assert ix.find_matches(h, 4) == [4, 0, 0, 2]
    ix.apply_removed(0, h[1:2])
    assert ix.find_matches(h, 4) == [1, 0, 0, 2]
    ix.remove_worker(3)
    assert ix.find_matches(h, 4) == [1, 0, 0, 0] and ix.num_blocks(0) == 3


# ----------------------------------------------------------------------------- scheduler
def _req(rid, n, max_tokens=4, base=0):
    return Request(rid, [base + i % 50 for i in range(n)], SamplingParams(max_tokens=max_tokens, ignore_eos=True))


def _run(s: Scheduler, steps=200):
    done = []
    for _ in range(steps):
        so = s.schedule()
        if so.is_empty:
            break
        assert s.kv.check_invariants()
        toks = {x.req.request_id: 7 for x in so.all() if x.sample}
        done += [r for r in s.update(so, toks) if r.is_finished]
    return done


def test_chunked_prefill_budget_and_decode_first():
    kv = KVCacheManager(256, 16)
    s = Scheduler(kv, max_num_seqs=8, max_num_batched_tokens=64, max_model_len=2048)
    s.add(_req("b", 10))
    s.add(_req("a", 150))
    so = s.schedule()
    assert so.num_tokens == 64 and so.prefills[1].num_new_tokens == 54 and not so.prefills[1].sample
    finished = [r for r in s.update(so, {x.req.request_id: 7 for x in so.all() if x.sample}) if r.is_finished]
    # a keeps chunking; once b decodes, decodes come first in the batch
    saw_mixed = False
    for _ in range(200):
        so = s.schedule()
        if so.is_empty:
            break
        assert so.num_tokens <= 64
        saw_mixed |= bool(so.decodes and so.prefills)
        finished += [r for r in s.update(so, {x.req.request_id: 7 for x in so.all() if x.sample}) if r.is_finished]
    assert saw_mixed and {r.request_id for r in finished} == {"a", "b"}


def test_prefix_cache_hits_and_first_token_recompute():
    kv = KVCacheManager(64, 16)
    s = Scheduler(kv, max_num_batched_tokens=512, max_model_len=1024)
    s.add(_req("a", 64))
    _run(s)
    b = _req("b", 64)  # identical prompt: 3 full blocks reused, last block recomputed
    s.add(b)
    so = s.schedule()
    assert b.num_cached_tokens == 48 and so.prefills[0].num_new_tokens == 16
    _run(s)
    assert kv.hit_rate() > 0 and kv.check_invariants()


def test_preemption_recompute():
    kv = KVCacheManager(12, 16)  # tiny pool forces preemption
    s = Scheduler(kv, max_num_seqs=4, max_num_batched_tokens=256, max_model_len=1024)
    for i in range(3):
        s.add(_req(f"r{i}", 40, max_tokens=40, base=i * 7))
    done = _run(s, steps=2000)
    assert len(done) == 3 and all(len(r.output_token_ids) == 40 for r in done)
    assert s.num_preemptions > 0 and kv.num_free() == 12 and kv.check_invariants()


def test_stop_conditions():
    r = Request("x", [1, 2], SamplingParams(max_tokens=10, stop_token_ids=[9]), eos_token_ids=(5,))
    r.output_token_ids = [3]
    assert r.check_stop(100) is None
    r.output_token_ids.append(5)
    assert r.check_stop(100) == Status.FINISHED_STOPPED
    r2 = Request("y", [1], SamplingParams(max_tokens=3, ignore_eos=True), eos_token_ids=(5,))
    r2.output_token_ids = [5, 5]
    assert r2.check_stop(100) is None
    r2.output_token_ids.append(5)
    assert r2.check_stop(100) == Status.FINISHED_LENGTH
    r3 = Request("z", [1], SamplingParams(max_tokens=10, min_tokens=3), eos_token_ids=(5,))
    r3.output_token_ids = [5]
    assert r3.check_stop(100) is None


def test_remote_prefill_reserve_and_complete():
    kv = KVCacheManager(32, 16)
    s = Scheduler(kv, max_model_len=1024)
    r = _req("d", 40, max_tokens=3)
    assert s.reserve_remote(r) and len(r.block_ids) == 3 and "d" in s.remote
    assert s.schedule().is_empty  # waits for its KV
    s.complete_remote("d", 11)
    assert r.output_token_ids == [11] and r in s.running
    done = _run(s)
    assert done and done[0].output_token_ids[0] == 11 and kv.num_free() == 32


def test_remote_reservations_count_against_max_num_seqs():
    """A decode worker never holds more than max_num_seqs requests (running + remote-prefill
    reservations): the model runner has max_num_seqs rows."""
    kv = KVCacheManager(256, 16)
    s = Scheduler(kv, max_num_seqs=4, max_model_len=1024)
    reqs = [_req(f"d{i}", 40, max_tokens=3) for i in range(6)]
    ok = [s.reserve_remote(r) for r in reqs]
    assert ok == [True] * 4 + [False] * 2
    assert kv.num_free() == 256 - 4 * 3  # refused reservations hold no blocks
    for r in reqs[:4]:
        s.complete_remote(r.request_id, 7)
    assert len(s.running) == 4
    # local admissions respect the cap too, while reservations are outstanding
    s2 = Scheduler(KVCacheManager(256, 16), max_num_seqs=3, max_model_len=1024)
    assert s2.reserve_remote(_req("x", 40)) and s2.reserve_remote(_req("y", 40))
    for i in range(3):
        s2.add(_req(f"w{i}", 20))
    out = s2.schedule()
    assert len(out.prefills) == 1 and len(s2.waiting) == 2


def test_prefix_registration_stops_at_landed_step():
    """With async scheduling num_computed_tokens already counts the step in flight; landing step N
    must only register blocks whose KV step N wrote."""
    kv = KVCacheManager(64, 16)
    s = Scheduler(kv, max_num_batched_tokens=32, max_model_len=1024)
    s.add(_req("a", 64, max_tokens=2))
    o1 = s.schedule()  # tokens [0, 32)
    o2 = s.schedule()  # tokens [32, 64) scheduled before step 1 lands
    r = o1.prefills[0].req
    assert r.num_computed_tokens == 64
    s.update(o1, {})
    assert r.num_registered_blocks == 2  # not 4: step 2's KV is not written yet
    s.update(o2, {"a": 5})
    assert r.num_registered_blocks == 4


# ----------------------------------------------------------------------------- router
def test_kv_router_prefers_cached_worker():
    from mxserve.router.router import Registry, Router, WorkerInfo
    reg = Registry()
    a = reg.register(WorkerInfo("a", "http://a", "m", kv_total_blocks=1000))
    b = reg.register(WorkerInfo("b", "http://b", "m", kv_total_blocks=1000))
    router = Router(reg, "kv")
    toks = list(range(320))
    reg.heartbeat("b", {"num_running": 5}, stored=router.block_hashes(toks))
    w, ov = router.pick([a, b], toks)
    assert w.worker_id == "b" and ov == 20
    # load balances when nothing is cached
    reg.heartbeat("b", {"kv_total_blocks": 1000, "kv_free_blocks": 100})
    w, ov = router.pick([a, b], list(range(1000, 1100)))
    assert w.worker_id == "a" and ov == 0
    reg.expire()
    assert len(reg.list()) == 2


# ----------------------------------------------------------------------------- tokenizer / templates
def test_byte_tokenizer_and_templates():
    from mxserve.frontend.chat_template import render
    from mxserve.frontend.tokenizer import ByteTokenizer, IncrementalDetokenizer
    from mxserve.models.config import get_model_config
    cfg = get_model_config("meta-llama/Llama-3.2-1B-Instruct")
    tok = ByteTokenizer(cfg)
    text = render("llama3", [{"role": "system", "content": "S"}, {"role": "user", "content": "héllo"}])
    assert text.startswith("<|begin_of_text|><|start_header_id|>system<|end_header_id|>\n\nS<|eot_id|>")
    assert text.endswith("<|start_header_id|>assistant<|end_header_id|>\n\n")
    ids = tok.encode(text)
    assert ids[0] == 128000 and 128009 in ids
    assert tok.decode(ids, skip_special_tokens=False) == text
    assert "héllo" in tok.decode(ids)
    d = IncrementalDetokenizer(tok)
    out = "".join(d.add(t) for t in tok.encode("日本語 ok")) + d.flush()
    assert out == "日本語 ok"
    # windowed decode: same text as one full decode, and the work per token does not grow with n
    long = "streaming détokenizer, ünïcödé 🙂 " * 40
    calls = []

    class _Windowed:  # a tokenizer without context-free pieces: the windowed decode path
        def decode(self, ids, **kw):
            calls.append(len(ids))
            return tok.decode(ids, **kw)
    d = IncrementalDetokenizer(_Windowed(), prompt_tail=tok.encode("prompt "))
    out = "".join(d.add(t) for t in tok.encode(long)) + d.flush()
    assert out == long
    assert max(calls) <= 16, max(calls)
    n_tok = len(tok.encode(long))
    assert len(calls) <= 1.3 * n_tok, (len(calls), n_tok)  # ~one decode per token, not two
    import random
    rng = random.Random(5)
    ids = tok.encode(long)
    for mode in [tok, _Windowed()] * 3:  # random batches, byte mode and window mode: the full decode's text
        d = IncrementalDetokenizer(mode)
        parts, i = [], 0
        while i < len(ids):
            k = rng.randint(1, 6)
            parts.append(d.add_many(ids[i:i + k]) if k > 1 else d.add(ids[i]))
            i += k
        assert "".join(parts) + d.flush() == long
    q = render("chatml", [{"role": "user", "content": "hi"}])
    assert q == "<|im_start|>user\nhi<|im_end|>\n<|im_start|>assistant\n"
    assert render("mistral", [{"role": "user", "content": "x"}]) == "<s>[INST] x [/INST]"


# ----------------------------------------------------------------------------- worker dialects
def test_worker_dialects(tmp_path):
    from mxserve.worker.args import parse_worker_args
    v = parse_worker_args(["--model", "meta-llama/Llama-3.2-1B-Instruct", "--is-prefill-worker"], "vllm")
    assert v.engine.model == "meta-llama/Llama-3.2-1B-Instruct" and v.engine.disagg_mode == "prefill"
    s = parse_worker_args(["--model-path", "m", "--served-model-name", "served", "--page-size", "16", "--tp", "2",
                           "--trust-remote-code", "--skip-tokenizer-init", "--disaggregation-mode", "decode",
                           "--disaggregation-transfer-backend", "nixl", "--disaggregation-bootstrap-port", "12345",
                           "--host", "0.0.0.0"], "sglang")
    assert s.engine.tensor_parallel_size == 2 and s.engine.name == "served" and s.engine.disagg_mode == "decode"
    assert s.engine.kv_transfer_backend == "xgmi" and s.engine.bootstrap_port == 12345
    y = tmp_path / "e.yaml"
    y.write_text("max_batch_size: 64\nmax_num_tokens: 2048\nkv_cache_config:\n  free_gpu_memory_fraction: 0.5\n")
    t = parse_worker_args(["--model-path", "Qwen/Qwen3-0.6B", "--extra-engine-args", str(y),
                           "--max-num-seqs", "32"], "trtllm")
    assert t.engine.max_num_seqs == 32 and t.engine.max_num_batched_tokens == 2048  # CLI beats YAML
    assert t.engine.gpu_memory_utilization == 0.5
    with pytest.raises(ValueError):
        parse_worker_args(["--model", "m", "--page-size", "32"], "sglang")


# ----------------------------------------------------------------------------- SLA planner
def test_sla_plan_meets_targets():
    from mxserve.profiler.sla import plan
    p = plan("Qwen/Qwen3-0.6B", 4000, 500, 600, 25)
    assert p["feasible"]
    d = p["disagg"]
    assert d["prefill"]["ttft_ms"] <= 600 and d["decode"]["itl_ms"] <= 25
    assert d["gpus_used"] <= 8
    big = plan("meta-llama/Meta-Llama-3-70B-Instruct", 2000, 256, 1000, 40)
    assert big["agg"]["tp"] >= 1 and big["feasible"]
    assert not plan("meta-llama/Meta-Llama-3-70B-Instruct", 4000, 500, 1, 1)["feasible"]


# ----------------------------------------------------------------------------- KV transfer staging
def test_ipc_safe_staging_sizes():
    from mxserve.disagg.kv_transfer import ipc_safe_blocks
    gib = 1 << 30
    for bb in (524288, 2 << 20, 32768, 81920, 1835008):
        for g in (0.5, 1, 2, 3, 4, 4.5, 6, 8, 19.53):
            k = int(g * gib) // bb
            kk = ipc_safe_blocks(k, bb)
            alloc = -(-kk * bb // (2 << 20)) * (2 << 20)  # caching-allocator 2 MiB granule
            assert kk <= k and alloc % (4 * gib) < 2 * gib, (bb, g)
    assert ipc_safe_blocks(8192, 524288) == 8192  # 4 GiB exactly is safe


def test_staging_arena_extents():
    import torch
    from mxserve.disagg.kv_transfer import KVTransferAgent

    class R:
        kv_cache = torch.zeros(4, 2, 2, 1, 16, 8)
        block_bytes = kv_cache[0].numel() * 4

    a = KVTransferAgent(R(), "host", max_prompt_tokens=64)
    a.backend = "xgmi"  # exercise the arena bookkeeping without a GPU
    a.arena_blocks = 10
    x = a.acquire(4)
    y = a.acquire(4)
    assert (x, y) == (0, 4) and a.acquire(4) is None
    a.release(x, 4)  # no event: reclaimed at the next acquire
    assert a.acquire(3) == 0 and a.acquire(2) == 8
    a.release(y, 4)
    a.release(0, 3)
    a.release(8, 2)
    assert a.acquire(10) == 0  # all extents merged back


def test_reasoning_splitter_streaming_and_unary():
    """<think> blocks go to reasoning_content; tags split across chunks are held back; deepseek_r1
    starts inside the reasoning block."""
    from mxserve.frontend.reasoning import ReasoningSplitter, split_text
    text = "<think>\nplan: add 2 and 2\n</think>\n\nFINAL: 4"
    assert split_text(text, "qwen3") == ("plan: add 2 and 2", "FINAL: 4")
    assert split_text(text, None) == (None, text)
    assert split_text("no reasoning here", "qwen3") == (None, "no reasoning here")
    assert split_text("thinking...</think>answer", "deepseek_r1") == ("thinking...", "answer")
    for cut in range(1, len(text)):
        sp = ReasoningSplitter("qwen3")
        parts = [sp.feed(text[i:i + cut], final=i + cut >= len(text)) for i in range(0, len(text), cut)]
        r = "".join(p[0] for p in parts)
        c = "".join(p[1] for p in parts)
        assert r == "\nplan: add 2 and 2\n" and c == "\n\nFINAL: 4", cut


def test_debug_kernel_build_compiles(tmp_path):
    """MXS_DEBUG_KERNELS builds (bounds-checked kernels) compile for gfx950: the
    checks are real device code in the debug objects and compiled away in release ones."""
    import os
    import shutil
    import subprocess
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "csrc", "kernels", "ep.hip")
    for mode, flags in (("debug", ["-DMXS_DEBUG_KERNELS"]), ("release", [])):
        out = tmp_path / f"ep_{mode}.s"
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                            *flags, src, "-o", str(out)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        asm = out.read_text()
        assert ("s_trap" in asm) == (mode == "debug"), mode
    shutil.rmtree(tmp_path, ignore_errors=True)


_LLAMA3_JINJA = ("{% set loop_messages = messages %}{% for message in loop_messages %}{% set content = "
                 "'<|start_header_id|>' + message['role'] + '<|end_header_id|>\\n\\n'+ message['content'] | trim + "
                 "'<|eot_id|>' %}{% if loop.index0 == 0 %}{% set content = bos_token + content %}{% endif %}"
                 "{{ content }}{% endfor %}{% if add_generation_prompt %}"
                 "{{ '<|start_header_id|>assistant<|end_header_id|>\\n\\n' }}{% endif %}")
_CHATML_JINJA = ("{% for message in messages %}{{'<|im_start|>' + message['role'] + '\\n' + message['content'] + "
                 "'<|im_end|>' + '\\n'}}{% endfor %}{% if add_generation_prompt %}{{ '<|im_start|>assistant\\n' }}"
                 "{% endif %}")


@pytest.mark.parametrize("form", ["string", "list"])
def test_chat_template_from_tokenizer_config(tmp_path, form):
    """A model directory's own Jinja chat_template (tokenizer_config.json) is what the frontend
    renders; for the public Llama-3 / ChatML templates that equals the built-in renderers."""
    import json

    from mxserve.frontend.chat_template import load_hf_template, render
    msgs = [{"role": "system", "content": "  Be brief. "}, {"role": "user", "content": "héllo"},
            {"role": "assistant", "content": "hi"}, {"role": "user", "content": "again"}]
    for name, tpl, bos, builtin in (("l3", _LLAMA3_JINJA, "<|begin_of_text|>", "llama3"),
                                    ("cm", _CHATML_JINJA, None, "chatml")):
        d = tmp_path / name
        d.mkdir()
        (d / "config.json").write_text("{}")
        cfg = {"bos_token": {"content": bos} if bos else None, "eos_token": "<|eot_id|>"}
        cfg["chat_template"] = tpl if form == "string" else [{"name": "tool_use", "template": "x"},
                                                             {"name": "default", "template": tpl}]
        (d / "tokenizer_config.json").write_text(json.dumps(cfg))
        load_hf_template.cache_clear()
        assert render(builtin, msgs, str(d)) == render(builtin, msgs)
    bad = tmp_path / "bad"
    bad.mkdir()
    (bad / "tokenizer_config.json").write_text(json.dumps(
        {"chat_template": "{{ raise_exception('roles must alternate') }}"}))
    load_hf_template.cache_clear()
    with pytest.raises(ValueError, match="alternate"):
        render("llama3", msgs, str(bad))


def test_step_time_model_learns_step_composition():
    """The late-admission predictor fits a step's GPU time from its composition."""
    import numpy as np
    from mxserve.engine.pacing import StepTimeModel
    m = StepTimeModel(lam=0.99, warmup=10)
    rng = np.random.default_rng(0)
    true = np.array([0.002, 0.0025, 0.001, 0.004, 0.0005])
    for _ in range(200):
        x = np.array([1.0, rng.uniform(0, 8), rng.uniform(0, 3), rng.uniform(0, 3), rng.uniform(0, 9)])
        m.update(x, float(x @ true))
    x = np.array([1.0, 4.0, 0.8, 2.0, 8.5])
    assert abs(m.predict(x) - float(x @ true)) < 1e-4


def test_late_admission_wait_stops_at_target_or_completion():
    import time
    from mxserve.engine.pacing import LateAdmission

    class Ev:
        def __init__(self, t_done):
            self.t_done = t_done

        def query(self):
            return time.perf_counter() >= self.t_done

    la = LateAdmission()
    la.host_lead, la.margin = 0.001, 0.0
    now = time.perf_counter()
    la.inflight = {"x": None, "t_launch": now, "est_done": now + 0.02, "done": None}
    t0 = time.perf_counter()
    la.wait(Ev(now + 1.0))  # predicted done in 20 ms: wake ~1 ms before
    assert 0.015 <= time.perf_counter() - t0 < 0.05 and la.inflight["done"] is None
    now = time.perf_counter()
    la.inflight = {"x": None, "t_launch": now, "est_done": now + 0.5, "done": None}
    t0 = time.perf_counter()
    la.wait(Ev(now + 0.01))  # finishes early: proceed at once, completion time recorded
    assert time.perf_counter() - t0 < 0.1 and la.inflight["done"] is not None
    la.inflight = {"x": None, "t_launch": now, "est_done": now + 0.5, "done": None}
    la.wait(Ev(0.0))  # already done when looked at: no wait, completion time unknown
    assert la.inflight["done"] is None


def test_streamer_ring_stall_is_transient():
    """a stalled output ring (GC pause / slow SSE writer in the streamer) must not drop
    outputs for good.  Held-back messages go out in order once the ring drains; the plane is
    declared dead only when the streamer process has exited (and then /health fails)."""
    import msgpack

    from mxserve.worker.streamer import RingPlane

    class _Ring:
        slot_bytes = 1 << 16

        def __init__(self):
            self.accept = False
            self.got = []

        def push(self, data, timeout):
            if not self.accept:
                return False
            self.got.append(msgpack.unpackb(data, raw=False))
            return True

        def pop(self, i, timeout):
            return None

    class _Proc:
        rc = None

        def poll(self):
            return self.rc

    ring, proc = _Ring(), _Proc()
    rp = RingPlane(worker=None, cmd_ring=ring, out_ring=ring, proc=proc)
    rp.emit_tuples([("a", 1, False, None, 0, 0, None, None, None)])
    rp.emit_tuples([("a", 2, True, "length", 0, 0, None, None, None)])  # the finish marker
    assert not rp.dead and len(rp.backlog) == 2 and rp.stalls >= 1
    ring.accept = True
    assert rp.poll(0.0) is None  # an idle engine loop flushes the backlog
    assert [m[0][1] for m in ring.got] == [1, 2] and not rp.backlog and rp.dropped == 0
    ring.accept = False
    proc.rc = -9  # the streamer died: now the plane is dead
    rp.emit_tuples([("b", 1, False, None, 0, 0, None, None, None)])
    assert rp.dead and rp.streamer_exited() and rp.dropped == 1


def test_meta_ring_push_is_bounded():
    """a TP follower that stops reading makes the driver's metadata push raise after
    MXS_TP_META_TIMEOUT_S instead of retrying forever (the worker then exits and is restarted)."""
    import pytest as _pt

    from mxserve.parallel.comm import MetaRing

    class _Full:
        slot_bytes = 1 << 16
        calls = 0

        def push(self, data, timeout):
            self.calls += 1
            return False

    r = _Full()
    mr = MetaRing(r, 0)
    mr.PUSH_TIMEOUT_S = 30.0
    with _pt.raises(RuntimeError, match="stopped reading"):
        mr.send(("step", 1))
    assert r.calls == 3


def test_ipc_open_deadline(monkeypatch):
    """a hipIpcOpenMemHandle that never returns costs its caller the deadline, not a
    hang: TimeoutError (an OSError, which the KV agent turns into the shm / HTTP path), and every
    later open in the process fails fast (the stuck call still holds the native table's lock)."""
    import threading
    import time as _time

    from mxserve import ops
    release = threading.Event()

    class _Ext:
        calls = 0

        def ipc_open_pool(self, handle, offset):
            _Ext.calls += 1
            if handle == b"hang":
                release.wait(30)
            return 4096 + offset

    monkeypatch.setattr(ops, "ext", lambda: _Ext())
    monkeypatch.setitem(ops.IPC_STATE, "broken", None)
    assert ops.ipc_open(b"ok", 16, timeout_s=5) == 4112
    t0 = _time.time()
    import pytest as _pt
    with _pt.raises(TimeoutError):
        ops.ipc_open(b"hang", 0, timeout_s=0.3)
    assert _time.time() - t0 < 2.0
    with _pt.raises(OSError):  # fails fast from now on, without calling into the native table
        ops.ipc_open(b"ok", 0, timeout_s=5)
    assert _Ext.calls == 2
    release.set()
