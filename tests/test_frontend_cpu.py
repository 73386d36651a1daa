"""OpenAI frontend + workers over real HTTP on localhost, CPU engines (BASELINE config 1 plumbing,
SURVEY.md §4.2 T4/T5): /v1/models, chat + completions (unary and SSE), error shapes, metrics
names from the reference dashboard, aggregated and disaggregated (host-staged KV) serving."""
import json

import httpx
import pytest

from mxserve.config import EngineArgs
from mxserve.frontend.app import Frontend
from mxserve.worker.args import WorkerArgs
from mxserve.worker.server import Worker
from tests.serving_utils import FrontendServer, Server, wait_for

MODEL = "tiny-llama"


def _worker(frontend_url, role="agg", seed=7):
    ea = EngineArgs(model=MODEL, device="cpu", cpu_num_blocks=256, max_model_len=1024, max_num_batched_tokens=64,
                    disagg_mode=role, load_format="random", seed=seed)
    wa = WorkerArgs(engine=ea, host="127.0.0.1", frontend_url=frontend_url, worker_id=f"{role}-w")
    w = Worker(wa)
    srv = Server(w.app)
    w.url = srv.url
    return w, srv


@pytest.fixture(scope="module")
def agg_stack():
    fe = Frontend(router_mode="kv", ttl=30)
    fs = FrontendServer(fe).start()  # httpd + push fast path, as `python -m mxserve.frontend` serves
    w, ws = _worker(fs.url)
    ws.start()
    wait_for(lambda: len(fe.registry.list()) == 1)
    yield fe, fs, w
    ws.stop()
    fs.stop()
    w.aeng.shutdown()


def test_models(agg_stack):
    fe, fs, _ = agg_stack
    d = httpx.get(fs.url + "/v1/models").json()
    assert d["object"] == "list" and d["data"][0]["id"] == MODEL and d["data"][0]["object"] == "model"
    assert httpx.get(fs.url + "/health").status_code == 200


def test_chat_unary(agg_stack):
    _, fs, _ = agg_stack
    r = httpx.post(fs.url + "/v1/chat/completions", headers={"Authorization": "Bearer dummy"},
                   json={"model": MODEL, "messages": [{"role": "user", "content": "hi there"}], "max_tokens": 7,
                         "temperature": 0}, timeout=60)
    assert r.status_code == 200
    d = r.json()
    assert d["object"] == "chat.completion"
    assert isinstance(d["choices"][0]["message"]["content"], str)
    assert d["usage"]["completion_tokens"] <= 7 and d["usage"]["prompt_tokens"] > 0
    assert d["choices"][0]["finish_reason"] in ("stop", "length")


def test_chat_stream_matches_unary(agg_stack):
    _, fs, _ = agg_stack
    body = {"model": MODEL, "messages": [{"role": "system", "content": "be brief"},
                                         {"role": "user", "content": "count"}], "max_tokens": 9, "temperature": 0,
            "ignore_eos": True}
    unary = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=60).json()
    text, reasons, saw_done = "", [], False
    with httpx.stream("POST", fs.url + "/v1/chat/completions", json=dict(body, stream=True,
                                                                        stream_options={"include_usage": True}),
                      timeout=60) as r:
        assert r.headers["content-type"].startswith("text/event-stream")
        for line in r.iter_lines():
            if not line.startswith("data: "):
                continue
            payload = line[6:]
            if payload == "[DONE]":
                saw_done = True
                break
            ch = json.loads(payload)
            if ch["choices"]:
                text += ch["choices"][0]["delta"].get("content") or ""
                if ch["choices"][0]["finish_reason"]:
                    reasons.append(ch["choices"][0]["finish_reason"])
            else:
                assert ch["usage"]["completion_tokens"] == 9
    assert saw_done and reasons == ["length"]
    assert text == unary["choices"][0]["message"]["content"]


def test_completions_and_prefix_routing(agg_stack):
    fe, fs, w = agg_stack
    prompt = "the same long prefix " * 8
    for _ in range(2):
        r = httpx.post(fs.url + "/v1/completions", json={"model": MODEL, "prompt": prompt, "max_tokens": 3,
                                                         "temperature": 0}, timeout=60)
        assert r.status_code == 200 and r.json()["object"] == "text_completion"
    # the worker published its cached blocks; the router's index now holds them
    wait_for(lambda: fe.registry.indexer.size() > 0, timeout=10)


def test_errors(agg_stack):
    _, fs, _ = agg_stack
    r = httpx.post(fs.url + "/v1/chat/completions", json={"model": "nope", "messages": [{"role": "user",
                                                                                       "content": "x"}]})
    assert r.status_code == 404 and "message" in r.json()["error"]
    r = httpx.post(fs.url + "/v1/chat/completions", json={"model": MODEL})
    assert r.status_code == 400 and "message" in r.json()["error"]
    r = httpx.post(fs.url + "/v1/chat/completions", content=b"{not json")
    assert r.status_code == 400


def test_metrics_names(agg_stack):
    _, fs, _ = agg_stack
    httpx.post(fs.url + "/v1/chat/completions", json={"model": MODEL, "messages": [{"role": "user", "content": "m"}],
                                                      "max_tokens": 2}, timeout=60)
    text = httpx.get(fs.url + "/metrics").text
    for name in ("dynamo_frontend_requests_total", "dynamo_frontend_time_to_first_token_seconds_sum",
                 "dynamo_frontend_time_to_first_token_seconds_count", "dynamo_frontend_inter_token_latency_seconds_sum",
                 "dynamo_frontend_request_duration_seconds_sum", "dynamo_frontend_input_sequence_tokens_sum",
                 "dynamo_frontend_output_sequence_tokens_sum", "dynamo_frontend_inflight_requests"):
        assert name in text, name
    assert 'request_type="unary"' in text and 'status="success"' in text


def test_stop_strings(agg_stack):
    _, fs, _ = agg_stack
    body = {"model": MODEL, "messages": [{"role": "user", "content": "x"}], "max_tokens": 30, "temperature": 0,
            "ignore_eos": True}
    full = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=60).json()["choices"][0]["message"]["content"]
    if len(full) < 4:
        pytest.skip("generated text too short to cut")
    stop = full[2:4]
    cut = httpx.post(fs.url + "/v1/chat/completions", json=dict(body, stop=[stop]), timeout=60).json()
    assert cut["choices"][0]["message"]["content"] == full[:full.find(stop)]
    assert cut["choices"][0]["finish_reason"] == "stop"


def test_logprobs_chat_and_completions(agg_stack):
    """OpenAI logprobs: chat (`logprobs` + `top_logprobs`, unary and SSE) and completions
    (`logprobs: k`); greedy picks are the top-1 alternative and log-probs are <= 0."""
    _, fs, _ = agg_stack
    body = {"model": MODEL, "messages": [{"role": "user", "content": "logprobs please"}], "max_tokens": 6,
            "temperature": 0, "ignore_eos": True, "logprobs": True, "top_logprobs": 3}
    d = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=60).json()
    content = d["choices"][0]["logprobs"]["content"]
    assert len(content) == 6
    for e in content:
        assert e["logprob"] <= 1e-6 and isinstance(e["token"], str) and isinstance(e["bytes"], list)
        tops = e["top_logprobs"]
        assert len(tops) == 3 and tops[0]["logprob"] >= tops[1]["logprob"] >= tops[2]["logprob"]
        assert abs(tops[0]["logprob"] - e["logprob"]) < 1e-4  # greedy: the sampled token is the best
    assert "".join(e["token"] for e in content) == d["choices"][0]["message"]["content"]
    streamed = []
    with httpx.stream("POST", fs.url + "/v1/chat/completions", json=dict(body, stream=True), timeout=60) as r:
        for line in r.iter_lines():
            if line.startswith("data: ") and line != "data: [DONE]":
                ch = json.loads(line[6:])["choices"][0]
                if ch.get("logprobs"):
                    streamed += ch["logprobs"]["content"]
    assert [e["logprob"] for e in streamed] == pytest.approx([e["logprob"] for e in content], abs=1e-5)
    c = httpx.post(fs.url + "/v1/completions", json={"model": MODEL, "prompt": "abc", "max_tokens": 4,
                                                     "temperature": 0, "ignore_eos": True, "logprobs": 2},
                   timeout=60).json()
    lp = c["choices"][0]["logprobs"]
    assert len(lp["tokens"]) == len(lp["token_logprobs"]) == len(lp["top_logprobs"]) == len(lp["text_offset"]) == 4
    assert all(len(t) <= 2 for t in lp["top_logprobs"]) and lp["text_offset"][0] == 0
    r = httpx.post(fs.url + "/v1/chat/completions", json=dict(body, logprobs=False), timeout=60)
    assert r.status_code == 400  # top_logprobs without logprobs
    plain = httpx.post(fs.url + "/v1/chat/completions", json=dict(body, logprobs=None, top_logprobs=None),
                       timeout=60).json()
    assert plain["choices"][0].get("logprobs") is None


def test_n_choices_unary_and_stream(agg_stack):
    """`n` > 1: one choice per index, seeds offset per choice, usage sums every choice; SSE chunks
    carry the choice index and every choice ends with its own finish_reason."""
    _, fs, _ = agg_stack
    body = {"model": MODEL, "messages": [{"role": "user", "content": "several"}], "max_tokens": 5,
            "temperature": 0.9, "seed": 11, "ignore_eos": True, "n": 3}
    d = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=60).json()
    assert [c["index"] for c in d["choices"]] == [0, 1, 2]
    assert d["usage"]["completion_tokens"] == 15
    greedy = httpx.post(fs.url + "/v1/chat/completions", json=dict(body, temperature=0, n=2), timeout=60).json()
    a, b = (c["message"]["content"] for c in greedy["choices"])
    assert a == b
    texts, reasons = {}, {}
    with httpx.stream("POST", fs.url + "/v1/completions",
                      json={"model": MODEL, "prompt": "abc", "max_tokens": 4, "temperature": 0, "ignore_eos": True,
                            "n": 2, "stream": True}, timeout=60) as r:
        for line in r.iter_lines():
            if line.startswith("data: ") and line != "data: [DONE]":
                for ch in json.loads(line[6:])["choices"]:
                    texts[ch["index"]] = texts.get(ch["index"], "") + ch["text"]
                    if ch["finish_reason"]:
                        reasons[ch["index"]] = ch["finish_reason"]
    assert reasons == {0: "length", 1: "length"} and texts[0] == texts[1]
    assert httpx.post(fs.url + "/v1/chat/completions", json=dict(body, n=0)).status_code == 400


def test_penalty_params(agg_stack):
    _, fs, _ = agg_stack
    body = {"model": MODEL, "messages": [{"role": "user", "content": "repeat"}], "max_tokens": 12, "temperature": 0,
            "ignore_eos": True, "presence_penalty": 2.0, "frequency_penalty": 0.5, "repetition_penalty": 1.2}
    r = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=60)
    assert r.status_code == 200 and r.json()["usage"]["completion_tokens"] == 12
    assert httpx.post(fs.url + "/v1/chat/completions", json=dict(body, presence_penalty=3.0)).status_code == 400
    assert httpx.post(fs.url + "/v1/chat/completions", json=dict(body, repetition_penalty=0)).status_code == 400


def test_reasoning_parser_fields(agg_stack):
    """With a reasoning parser the <think> part goes to message.reasoning_content (unary) and
    delta.reasoning_content (SSE).  deepseek_r1 starts in reasoning mode, so a completion without
    </think> is all reasoning: the plumbing is visible with any model."""
    fe, fs, _ = agg_stack
    body = {"model": MODEL, "messages": [{"role": "user", "content": "think"}], "max_tokens": 6, "temperature": 0,
            "ignore_eos": True}
    plain = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=60).json()["choices"][0]["message"]
    fe.reasoning_parser = "deepseek_r1"
    try:
        msg = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=60).json()["choices"][0]["message"]
        assert msg["content"] == "" and msg["reasoning_content"] == plain["content"].strip("\n")
        rs, cs = "", ""
        with httpx.stream("POST", fs.url + "/v1/chat/completions", json=dict(body, stream=True), timeout=60) as r:
            for line in r.iter_lines():
                if line.startswith("data: ") and line != "data: [DONE]":
                    d = json.loads(line[6:])["choices"][0]["delta"]
                    rs += d.get("reasoning_content") or ""
                    cs += d.get("content") or ""
        assert rs == plain["content"] and cs == ""
    finally:
        fe.reasoning_parser = None


@pytest.mark.parametrize("via", ["shm", "host"])
@pytest.mark.parametrize("streamer", [False, True])
def test_disaggregated_matches_aggregated(via, streamer, monkeypatch):
    """Prefill worker + decode worker give the agg result token for token, with the KV moved
    through the decode worker's /dev/shm staging arena (same host) or, without one, in the HTTP
    body; with the decode worker's token plane in its own or in a streamer process."""
    from mxserve.disagg import kv_transfer
    if via == "host":
        monkeypatch.setattr(kv_transfer, "SHM_BYTES", 0)
    fe = Frontend(router_mode="round_robin", ttl=30)
    fs = Server(fe.app).start()
    pw, ps = _worker(fs.url, role="prefill")
    dw, ds = _worker(fs.url, role="decode")
    sproc = None
    if streamer:
        from mxserve.worker.streamer import start_streamer
        from tests.serving_utils import free_port
        sport = free_port()
        sproc, cmd, out = start_streamer("127.0.0.1", sport, 1024)
        dw.attach_streamer(cmd, out, f"http://127.0.0.1:{sport}")

        def up():
            try:
                return httpx.get(f"http://127.0.0.1:{sport}/health", timeout=2).status_code == 200
            except httpx.HTTPError:
                return False
        wait_for(up, timeout=60)
    ps.start()
    ds.start()
    try:
        wait_for(lambda: len(fe.registry.list()) == 2)
        body = {"model": MODEL, "messages": [{"role": "user", "content": "disaggregate me " * 5}], "max_tokens": 8,
                "temperature": 0, "ignore_eos": True}
        r = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=120)
        assert r.status_code == 200, r.text
        disagg = r.json()["choices"][0]["message"]["content"]
        assert pw.agent.backend == "host"
        # the decode worker really received the prompt's KV from the prefill worker
        assert dw.metrics.kv_xfer_bytes.labels(MODEL, via)._value.get() > 0
        # the request trace carries the disaggregated spans: remote prefill + KV transfer by path
        tr = httpx.get(fs.url + "/debug/traces").json()["traces"][-1]
        wm = tr["worker_ms"]
        assert wm["kv_path"] == via and wm["kv_transfer_ms"] >= 0 and wm["remote_prefill_ms"] >= 0
        assert wm["prefill_worker_prefill_ms"] >= 0
        if via == "shm":  # every staging extent came back once the copies landed
            assert dw.agent._shm_ext.free_blocks() == dw.agent.shm_blocks
        # aggregated reference with the same weights (same seed)
        agg, ags = _worker(None, role="agg")
        ags.start()
        fe2 = Frontend(router_mode="round_robin")
        fe2.registry.register(__import__("mxserve.router.router", fromlist=["WorkerInfo"]).WorkerInfo(
            worker_id="a", url=ags.url, model=MODEL))
        fs2 = Server(fe2.app).start()
        ref = httpx.post(fs2.url + "/v1/chat/completions", json=body, timeout=120).json()
        assert disagg == ref["choices"][0]["message"]["content"]
        fs2.stop()
        ags.stop()
        agg.aeng.shutdown()
    finally:
        ps.stop()
        ds.stop()
        fs.stop()
        pw.aeng.shutdown()
        dw.aeng.shutdown()
        pw.agent.close()
        dw.agent.close()
        if sproc is not None:
            sproc.terminate()
            sproc.wait(timeout=20)


def test_request_trace_by_x_request_id(agg_stack):
    _, fs, _ = agg_stack
    r = httpx.post(fs.url + "/v1/chat/completions", headers={"x-request-id": "trace-me-1"},
                   json={"model": MODEL, "messages": [{"role": "user", "content": "t"}], "max_tokens": 3}, timeout=60)
    assert r.status_code == 200
    tr = [t for t in httpx.get(fs.url + "/debug/traces").json()["traces"] if t["request_id"] == "trace-me-1"]
    assert tr and tr[0]["status"] == "success"
    spans = tr[0]["spans_ms"]
    # receive -> tokenize -> route -> (worker: queue -> prefill) -> first token -> done
    assert spans["received"] <= spans["tokenized"] <= spans["routed"] <= spans["first_token"] <= spans["done"]
    wm = tr[0]["worker_ms"]
    assert wm["queue_ms"] >= 0 and wm["prefill_ms"] >= 0 and tr[0]["worker"] == "agg-w"


def test_retry_on_dead_worker_before_first_token(agg_stack):
    """A registered worker that refuses connections is skipped (and dropped) before the first token."""
    from mxserve.router.router import WorkerInfo
    from tests.serving_utils import free_port
    _, _, w = agg_stack
    fe = Frontend(router_mode="round_robin", ttl=30)
    fe.registry.register(WorkerInfo(worker_id="dead", url=f"http://127.0.0.1:{free_port()}", model=MODEL))
    fe.registry.register(WorkerInfo(worker_id="live", url=w.url, model=MODEL))
    fs = Server(fe.app).start()
    try:
        for _ in range(2):
            r = httpx.post(fs.url + "/v1/chat/completions",
                           json={"model": MODEL, "messages": [{"role": "user", "content": "r"}], "max_tokens": 2},
                           timeout=60)
            assert r.status_code == 200, r.text
        assert [x.worker_id for x in fe.registry.list()] == ["live"]
    finally:
        fs.stop()


def test_disagg_prefill_failure_falls_back_to_local():
    """Fault injection: the prefill worker rejects every /prefill; the decode worker
    prefills locally and the answer is unchanged."""
    from mxserve.utils.tracing import FAULTS
    fe = Frontend(router_mode="round_robin", ttl=30)
    fs = Server(fe.app).start()
    pw, ps = _worker(fs.url, role="prefill")
    dw, ds = _worker(fs.url, role="decode")
    ps.start()
    ds.start()
    body = {"model": MODEL, "messages": [{"role": "user", "content": "fallback " * 4}], "max_tokens": 6,
            "temperature": 0, "ignore_eos": True}
    try:
        wait_for(lambda: len(fe.registry.list()) == 2)
        ok = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=120).json()
        FAULTS.p = {"fail_prefill": 1.0}
        r = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=120)
        assert r.status_code == 200, r.text
        assert r.json()["choices"][0]["message"]["content"] == ok["choices"][0]["message"]["content"]
        assert dw.engine.kv.check_invariants() and pw.engine.kv.check_invariants()
    finally:
        FAULTS.p = {}
        ps.stop()
        ds.stop()
        fs.stop()
        pw.aeng.shutdown()
        dw.aeng.shutdown()


@pytest.mark.parametrize("together", [False, True])
def test_mid_stream_migration_keeps_greedy_output(monkeypatch, together):
    """a worker that drops the stream after its first token; the frontend re-prefills
    prompt + generated tokens on the other worker and the client sees the same greedy text.
    together: the first token and the drop marker reach the frontend in one channel write (a loaded
    worker: two steps' outputs before the channel drains) -- the token still counts as generated."""
    from mxserve.utils.tracing import Faults
    if together:
        from mxserve.engine.engine import StepOutput
        from mxserve.worker import server as wsrv
        held: dict = {}

        def put_nowait(self, o):
            self.n += 1
            if self.n == 1:
                held[id(self)] = o
            elif self.n == 2:
                self.ch.pending.append(held.pop(id(self)))
                self.ch.pending.append(StepOutput(o.request_id, -2, True, "abort", 0, 0, 0))
                self.ch.wake.set()
                self.on_drop(o.request_id)
        monkeypatch.setattr(wsrv._DropSink, "put_nowait", put_nowait)
    fe = Frontend(router_mode="round_robin", ttl=30)
    fs = Server(fe.app).start()
    a, as_ = _worker(fs.url, role="agg")
    b, bs_ = _worker(fs.url, role="agg")
    a.worker_id, b.worker_id = "flaky", "healthy"
    a.faults = Faults("drop_stream:1.0")
    as_.start()
    bs_.start()
    body = {"model": MODEL, "messages": [{"role": "user", "content": "migrate me"}], "max_tokens": 12,
            "temperature": 0, "ignore_eos": True}
    forgot = []
    real_forget = fe.router.forget
    fe.router.forget = lambda w, rid: forgot.append((w.worker_id, rid)) or real_forget(w, rid)
    try:
        wait_for(lambda: len(fe.registry.list()) == 2)
        outs = [httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=120).json() for _ in range(2)]
        texts = {o["choices"][0]["message"]["content"] for o in outs}
        assert len(texts) == 1, outs  # one request hit the flaky worker first, the other did not
        # the flaky worker queued the request (it streamed a token), so its routed entry is
        # retired by the worker's num_added, not forgotten (that would retire a later request's)
        assert not forgot, forgot
        assert all(o["usage"]["completion_tokens"] == 12 for o in outs)
        text = httpx.get(fs.url + "/metrics").text
        assert "dynamo_frontend_request_migrations_total" in text
        assert any(ln.startswith("dynamo_frontend_request_migrations_total") and not ln.endswith(" 0.0")
                   for ln in text.splitlines())
    finally:
        as_.stop()
        bs_.stop()
        fs.stop()
        a.aeng.shutdown()
        b.aeng.shutdown()


def test_remote_prefill_cancel_releases_reservation():
    """A client that goes away while the decode worker awaits the prefill POST (CancelledError)
    must not leak the reserved KV blocks, the remote slot or the token queue -- and must not free
    the blocks while the prefill worker may still push into them: they are held until its reply,
    or (the POST failing without one, as here) the quarantine delay."""
    import asyncio
    import socket
    import threading
    import time

    lst = socket.socket()
    lst.bind(("127.0.0.1", 0))
    lst.listen(4)
    held = []
    threading.Thread(target=lambda: held.append(lst.accept()), daemon=True).start()  # accepts, never answers
    w, _ = _worker(None, role="decode")
    w.QUARANTINE_S = 0.5
    eng = w.engine
    free0 = eng.kv.num_free()

    async def go():
        from mxserve.engine.request import SamplingParams
        t = asyncio.ensure_future(w._remote_prefill("rq", list(range(40)), SamplingParams(max_tokens=4),
                                                   f"http://127.0.0.1:{lst.getsockname()[1]}"))
        for _ in range(200):
            await asyncio.sleep(0.01)
            if held:
                break
        assert "rq" in eng.scheduler.remote and eng.kv.num_free() < free0
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        await asyncio.sleep(0.1)
        assert "rq" not in eng.scheduler.remote and eng.kv.num_free() < free0  # detached, still held
        if w._http is not None:
            await w._http.close()  # the POST fails without a reply: quarantine, then free
        for _ in range(100):
            if w.kv_quarantined == 0:
                break
            await asyncio.sleep(0.05)

    try:
        asyncio.run(go())
        for _ in range(200):  # the abort runs on the engine thread
            if not eng.scheduler.remote and eng.kv.num_free() == free0:
                break
            time.sleep(0.01)
        assert not eng.scheduler.remote and eng.kv.num_free() == free0
        assert "rq" not in w.aeng._queues and "rq" not in eng.requests
    finally:
        w.aeng.shutdown()
        lst.close()


def test_batched_ndjson_token_lines():
    """A worker that writes several tokens per NDJSON line (a consumer fell behind) is parsed
    token by token: same completion text, usage and finish reason as one token per line."""
    from fastapi import FastAPI
    from fastapi.responses import StreamingResponse

    from mxserve.engine.engine import StepOutput
    from mxserve.router.router import WorkerInfo
    from mxserve.worker.server import _batch_line
    toks = [ord(c) for c in "hello batched world"]  # byte tokenizer ids (tiny-llama vocab covers ASCII)
    outs = [StepOutput("x", t, i == len(toks) - 1, "length" if i == len(toks) - 1 else None, 7, 0, i + 1)
            for i, t in enumerate(toks)]
    app = FastAPI()

    @app.post("/generate")
    async def gen():
        async def body():
            yield _batch_line(outs[:1])
            yield _batch_line(outs[1:6])
            yield _batch_line(outs[6:])
        return StreamingResponse(body(), media_type="application/x-ndjson")

    ws = Server(app).start()
    fe = Frontend(router_mode="round_robin")
    fs = Server(fe.app).start()
    try:
        fe.registry.register(WorkerInfo(worker_id="fake", url=ws.url, model=MODEL))
        r = httpx.post(fs.url + "/v1/completions", json={"model": MODEL, "prompt": "p", "max_tokens": len(toks)},
                       timeout=30)
        assert r.status_code == 200, r.text
        d = r.json()
        assert d["usage"]["completion_tokens"] == len(toks)
        assert d["choices"][0]["finish_reason"] == "length"
        tok = fe.tokenizer(MODEL)
        assert d["choices"][0]["text"] == tok.decode(toks)
    finally:
        fs.stop()
        ws.stop()


def test_mux_plane_client_disconnect_aborts(agg_stack):
    """On the multiplexed request plane a client that goes away mid-stream makes the frontend POST
    /abort: the worker drops the request (engine, channel membership, sink)."""
    import time
    fe, fs, w = agg_stack
    with httpx.Client(timeout=60) as c:
        with c.stream("POST", fs.url + "/v1/completions",
                      json={"model": MODEL, "prompt": "tell me", "max_tokens": 400, "stream": True,
                            "ignore_eos": True}) as r:
            n = 0
            for line in r.iter_lines():
                if line.startswith("data: {"):
                    n += 1
                if n >= 3:
                    break
    for _ in range(300):
        if not w.engine.requests and not w.aeng._queues and all(not ch.rids for ch in w._channels.values()):
            break
        time.sleep(0.02)
    assert not w.engine.requests and not w.aeng._queues
    assert w._channels and all(not ch.rids for ch in w._channels.values())


def test_stream_plane_fallback(agg_stack, monkeypatch):
    """MXS_REQUEST_PLANE=stream: one /generate NDJSON response per request (the pre-mux protocol,
    also what the frontend falls back to for a worker without /mux)."""
    from mxserve.frontend import app as app_mod
    monkeypatch.setattr(app_mod, "REQUEST_PLANE", "stream")
    _, fs, _ = agg_stack
    body = {"model": MODEL, "prompt": "same prompt", "max_tokens": 6, "temperature": 0}
    a = httpx.post(fs.url + "/v1/completions", json=body, timeout=60).json()
    monkeypatch.setattr(app_mod, "REQUEST_PLANE", "mux")
    b = httpx.post(fs.url + "/v1/completions", json=body, timeout=60).json()
    assert a["choices"][0]["text"] == b["choices"][0]["text"]
    assert a["usage"]["completion_tokens"] == b["usage"]["completion_tokens"] == 6


def test_multiprocess_frontend_shares_discovery_and_metrics(tmp_path):
    """`--num-procs 2`: both processes serve the port, a worker registered through one of them is
    routable from either, and /metrics sums the processes' counters."""
    import os
    import subprocess
    import sys
    import time
    from tests.serving_utils import free_port
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    env.pop("PROMETHEUS_MULTIPROC_DIR", None)
    fp, wp = free_port(), free_port()
    fe = subprocess.Popen([sys.executable, "-m", "mxserve.frontend", "--http-host", "127.0.0.1", "--http-port", str(fp),
                           "--num-procs", "2"], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    wk = subprocess.Popen([sys.executable, os.path.join(root, "scripts", "frontend_cpu_probe.py"), "--role", "worker",
                           "--port", str(wp), "--frontend", f"http://127.0.0.1:{fp}", "--step-ms", "2"], env=env,
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    url = f"http://127.0.0.1:{fp}"
    model = "meta-llama/Llama-3.2-1B-Instruct"
    try:
        seen = 0
        for _ in range(300):  # fresh connections land on either process; all must know the worker
            try:
                ok = all(model in httpx.get(url + "/v1/models", timeout=2).text for _ in range(8))
            except httpx.HTTPError:
                ok = False
            seen = seen + 1 if ok else 0
            if seen >= 3:
                break
            time.sleep(0.1)
        assert seen >= 3, "worker not visible from every frontend process"
        for i in range(8):
            r = httpx.post(url + "/v1/completions", json={"model": model, "prompt": [1, 2, 3], "max_tokens": 5},
                           timeout=30)
            assert r.status_code == 200, r.text
            assert r.json()["usage"]["completion_tokens"] == 5
        from mxserve.planner.planner import parse_prometheus
        m = parse_prometheus(httpx.get(url + "/metrics", timeout=5).text)
        total = sum(v for k, v in m.items() if k.startswith("dynamo_frontend_requests_total"))
        assert total == 8, m
    finally:
        wk.terminate()
        fe.terminate()
        wk.wait(timeout=20)
        fe.wait(timeout=30)


@pytest.fixture(scope="module")
def streamer_stack():
    """Agg worker whose token request plane runs in a streamer process (worker/streamer.py)."""
    from mxserve.worker.streamer import start_streamer
    from tests.serving_utils import free_port
    sport = free_port()
    proc, cmd, out = start_streamer("127.0.0.1", sport, 1024)
    fe = Frontend(router_mode="kv", ttl=30)
    fs = Server(fe.app).start()
    w, ws = _worker(fs.url)
    w.attach_streamer(cmd, out, f"http://127.0.0.1:{sport}")
    def up():
        try:
            return httpx.get(f"http://127.0.0.1:{sport}/health", timeout=2).status_code == 200
        except httpx.HTTPError:
            return False
    wait_for(up, timeout=60)
    ws.start()
    wait_for(lambda: len(fe.registry.list()) == 1)
    yield fe, fs, w
    ws.stop()
    fs.stop()
    w.aeng.shutdown()
    proc.terminate()
    proc.wait(timeout=20)


def test_streamer_process_serves_the_token_plane(streamer_stack, agg_stack):
    """Greedy completions through the streamer process equal the in-worker plane's; streaming
    works; the worker registered its stream_url and its own /mux channels stay unused."""
    fe, fs, w = streamer_stack
    assert fe.registry.list()[0].stream_url.endswith(str(w.stream_url.rsplit(":", 1)[1]))
    body = {"model": MODEL, "prompt": "same prompt again", "max_tokens": 9, "temperature": 0}
    a = httpx.post(fs.url + "/v1/completions", json=body, timeout=60).json()
    b = httpx.post(agg_stack[1].url + "/v1/completions", json=body, timeout=60).json()
    assert a["choices"][0]["text"] == b["choices"][0]["text"] and a["usage"]["completion_tokens"] == 9
    chunks = []
    with httpx.stream("POST", fs.url + "/v1/completions", json=dict(body, stream=True), timeout=60) as r:
        for line in r.iter_lines():
            if line.startswith("data: {"):
                chunks.append(json.loads(line[6:])["choices"][0]["text"])
    assert "".join(chunks) == a["choices"][0]["text"]
    assert not w._channels and w._ring_plane is not None and w._ring_plane.dropped == 0


def test_streamer_client_disconnect_aborts(streamer_stack):
    import time
    fe, fs, w = streamer_stack
    with httpx.Client(timeout=60) as c:
        with c.stream("POST", fs.url + "/v1/completions",
                      json={"model": MODEL, "prompt": "go on", "max_tokens": 400, "stream": True,
                            "ignore_eos": True}) as r:
            n = 0
            for line in r.iter_lines():
                n += line.startswith("data: {")
                if n >= 3:
                    break
    for _ in range(300):
        if not w.engine.requests and not w.aeng._queues:
            break
        time.sleep(0.02)
    assert not w.engine.requests and not w.aeng._queues


def test_mux_channel_reconnects_after_worker_restart():
    """The frontend's channel to a worker breaks when the worker restarts on the same address; the
    next request opens a new channel (the worker answers /submit for an unknown channel with 404,
    or the dead reader is noticed first) and completes."""
    from tests.serving_utils import free_port
    fe = Frontend(router_mode="round_robin", ttl=30)
    fs = Server(fe.app).start()
    port = free_port()
    body = {"model": MODEL, "prompt": "restart me", "max_tokens": 5, "temperature": 0}
    w1, _ = _worker(None)
    s1 = Server(w1.app, port=port).start()
    from mxserve.router.router import WorkerInfo
    fe.registry.register(WorkerInfo(worker_id="w", url=s1.url, model=MODEL))
    try:
        a = httpx.post(fs.url + "/v1/completions", json=body, timeout=60).json()
        assert a["usage"]["completion_tokens"] == 5
        s1.stop()
        w1.aeng.shutdown()
        w2, _ = _worker(None)
        s2 = Server(w2.app, port=port).start()
        try:
            b = httpx.post(fs.url + "/v1/completions", json=body, timeout=60)
            assert b.status_code == 200, b.text
            assert b.json()["choices"][0]["text"] == a["choices"][0]["text"]
            assert w2._channels  # a new channel was opened on the restarted worker
        finally:
            s2.stop()
            w2.aeng.shutdown()
    finally:
        fs.stop()


def _sse_events(url: str, path: str, body: dict) -> list:
    out = []
    with httpx.stream("POST", url + path, json=body, timeout=60) as r:
        assert r.status_code == 200 and r.headers["content-type"].startswith("text/event-stream")
        for line in r.iter_lines():
            if line.startswith("data: "):
                out.append(line[6:])
    return out


def _normalize(events: list) -> dict:
    """What a stream says, independent of how tokens were grouped into chunks (a consumer that falls
    behind legitimately merges deltas): the text, the finish reasons, the usage, the chunk schema
    and the terminator."""
    text, reasons, usage, shapes, roles = "", [], None, set(), 0
    for p in events:
        if p == "[DONE]":
            continue
        d = json.loads(p)
        shapes.add((d["object"], d["model"], tuple(sorted(d))))
        if not d["choices"]:
            usage = d.get("usage")
            continue
        ch = d["choices"][0]
        shapes.add(tuple(sorted(ch)))
        delta = ch.get("delta")
        if delta is not None:
            roles += "role" in delta
            text += delta.get("content") or ""
        else:
            text += ch.get("text") or ""
        if ch.get("finish_reason"):
            reasons.append(ch["finish_reason"])
    return {"text": text, "reasons": reasons, "usage": usage, "shapes": shapes, "roles": roles,
            "done": events[-1] == "[DONE]"}


@pytest.mark.parametrize("path,extra", [
    ("/v1/chat/completions", {"stream_options": {"include_usage": True}}),
    ("/v1/chat/completions", {"stop": ["\n", "e"]}),
    ("/v1/completions", {"stop": "a"}),
    ("/v1/completions", {}),
])
def test_push_fast_path_matches_fastapi_path(agg_stack, monkeypatch, path, extra):
    """The httpd push path (frontend/fastpath.py) streams exactly what the FastAPI route streams:
    same chunks (content deltas, finish reasons, usage), same [DONE].  The FastAPI side is served
    by uvicorn from the same Frontend; the fast side must really be the push path."""
    from mxserve.frontend import fastpath
    fe, fs, w = agg_stack
    body = {"model": MODEL, "max_tokens": 12, "temperature": 0, "ignore_eos": True, "stream": True, **extra}
    if path.endswith("chat/completions"):
        body["messages"] = [{"role": "user", "content": "push path parity"}]
    else:
        body["prompt"] = "push path parity"
    used = []
    orig = fastpath.PushStream.head
    monkeypatch.setattr(fastpath.PushStream, "head", lambda self: (used.append(1), orig(self))[1])
    fast = _normalize(_sse_events(fs.url, path, body))
    assert used, "the push fast path did not serve the request"
    fe2 = Frontend(router_mode="kv", ttl=30)  # its own loop-bound sessions: a second Frontend
    slow_srv = Server(fe2.app).start()  # uvicorn: the FastAPI route only
    try:
        assert httpx.post(slow_srv.url + "/internal/register", json=w.registration(), timeout=10).status_code == 200
        slow = _normalize(_sse_events(slow_srv.url, path, body))
    finally:
        slow_srv.stop()
    assert fast == slow
    assert fast["done"] and len(fast["reasons"]) == 1


def test_httpd_keep_alive_errors_and_bridge(agg_stack):
    """One connection, several requests: JSON routes through the ASGI bridge, an error in the app's
    shape from the fast path, a streamed response, and the connection stays usable throughout."""
    _, fs, _ = agg_stack
    with httpx.Client(base_url=fs.url, timeout=60) as c:
        assert c.get("/v1/models").json()["object"] == "list"
        r = c.post("/v1/chat/completions", json={"model": "nope", "messages": [], "stream": True})
        assert r.status_code == 404 and "error" in r.json() and r.json()["error"]["message"]
        r = c.post("/v1/chat/completions", json={"model": MODEL, "stream": True})
        assert r.status_code == 400 and "messages" in r.json()["error"]["message"]
        r = c.post("/v1/chat/completions", content=b"{not json", headers={"content-type": "application/json"})
        assert r.status_code == 400
        with c.stream("POST", "/v1/completions", json={"model": MODEL, "prompt": "x", "max_tokens": 3,
                                                       "stream": True, "temperature": 0}) as s:
            lines = [ln for ln in s.iter_lines() if ln.startswith("data: ")]
        assert lines[-1] == "data: [DONE]" and len(lines) >= 2
        assert c.get("/health").status_code == 200
        assert "dynamo_frontend_requests_total" in c.get("/metrics").text


def test_httpd_rejects_bad_lengths_times_out_slow_heads_and_continues(monkeypatch):
    """Content-Length is digits only and repeated values must agree (400 otherwise); a
    request head that does not complete within the header timeout gets 408 and a close; an idle
    keep-alive connection is closed; Expect: 100-continue gets an interim 100 before the body."""
    import asyncio
    import socket as _socket
    import threading
    import time

    from mxserve.frontend import httpd

    monkeypatch.setattr(httpd, "HEADER_TIMEOUT_S", 0.5)
    monkeypatch.setattr(httpd, "IDLE_TIMEOUT_S", 0.8)

    async def app(scope, receive, send):
        if scope["type"] == "lifespan":
            while True:
                m = await receive()
                await send({"type": m["type"] + ".complete"})
                if m["type"] == "lifespan.shutdown":
                    return
        msg = await receive()
        body = b"got %d" % len(msg["body"])
        await send({"type": "http.response.start", "status": 200, "headers": [(b"content-type", b"text/plain")]})
        await send({"type": "http.response.body", "body": body})

    sock = httpd.listen("127.0.0.1", 0)
    port = sock.getsockname()[1]
    loop = asyncio.new_event_loop()
    stop = asyncio.Event()
    srv = httpd.Server(app)
    th = threading.Thread(target=lambda: loop.run_until_complete(srv.serve(sock, stop)), daemon=True)
    th.start()

    def talk(data: bytes, wait: float = 0.3, read_until_close: bool = False) -> bytes:
        c = _socket.create_connection(("127.0.0.1", port), timeout=5)
        c.sendall(data)
        time.sleep(wait)
        out = b""
        c.settimeout(3)
        try:
            while True:
                b = c.recv(65536)
                if not b:
                    break
                out += b
                if not read_until_close and b"\r\n\r\n" in out and out.count(b"HTTP/1.1") >= 1 and b"got" in out:
                    break
        except _socket.timeout:
            pass
        c.close()
        return out

    try:
        time.sleep(0.3)
        ok = talk(b"POST / HTTP/1.1\r\nhost: x\r\ncontent-length: 3\r\n\r\nabc")
        assert ok.startswith(b"HTTP/1.1 200") and b"got 3" in ok
        for bad in (b"-5", b"+3", b"1_0", b"3 3", b""):
            r = talk(b"POST / HTTP/1.1\r\nhost: x\r\ncontent-length: " + bad + b"\r\n\r\nabc", read_until_close=True)
            assert r.startswith(b"HTTP/1.1 400"), (bad, r)
        r = talk(b"POST / HTTP/1.1\r\ncontent-length: 3\r\ncontent-length: 4\r\n\r\nabcd", read_until_close=True)
        assert r.startswith(b"HTTP/1.1 400") and b"conflicting" in r
        r = talk(b"POST / HTTP/1.1\r\ncontent-length: 3\r\ncontent-length: 3\r\n\r\nabc")
        assert r.startswith(b"HTTP/1.1 200")
        # slowloris: half a head, then nothing -> 408 and the connection is closed
        r = talk(b"POST / HTTP/1.1\r\nhost: x\r\n", wait=1.0, read_until_close=True)
        assert r.startswith(b"HTTP/1.1 408"), r
        # idle keep-alive connection: closed by the server
        c = _socket.create_connection(("127.0.0.1", port), timeout=5)
        t0 = time.time()
        c.settimeout(5)
        assert c.recv(10) == b""  # EOF from the idle timeout
        assert time.time() - t0 < 4
        c.close()
        # Expect: 100-continue -> interim response, then the real one after the body
        c = _socket.create_connection(("127.0.0.1", port), timeout=5)
        c.sendall(b"POST / HTTP/1.1\r\nhost: x\r\nexpect: 100-continue\r\ncontent-length: 5\r\n\r\n")
        c.settimeout(3)
        assert c.recv(100).startswith(b"HTTP/1.1 100 Continue")
        c.sendall(b"hello")
        out = b""
        while b"got 5" not in out:
            out += c.recv(1000)
        assert b"HTTP/1.1 200" in out
        c.close()
        # a body that keeps arriving is never cut off by the header timeout (0.5 s here:
        # the upload takes ~1.2 s in 0.2 s chunks) ...
        c = _socket.create_connection(("127.0.0.1", port), timeout=5)
        c.sendall(b"POST / HTTP/1.1\r\nhost: x\r\ncontent-length: 60\r\n\r\n")
        for _ in range(6):
            time.sleep(0.2)
            c.sendall(b"x" * 10)
        c.settimeout(3)
        out = b""
        while b"got 60" not in out:
            b = c.recv(1000)
            assert b, out
            out += b
        assert out.startswith(b"HTTP/1.1 200"), out
        c.close()
        # ... but a body that stops arriving gets 408
        r = talk(b"POST / HTTP/1.1\r\nhost: x\r\ncontent-length: 60\r\n\r\nxxxx", wait=1.0, read_until_close=True)
        assert r.startswith(b"HTTP/1.1 408"), r
    finally:
        loop.call_soon_threadsafe(stop.set)
        th.join(timeout=10)
