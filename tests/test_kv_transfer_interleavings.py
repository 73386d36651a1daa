"""Randomized interleavings of the disaggregated KV-transfer state machine: many
requests move through reserve -> extent acquire (GPU-arena and shm extents) -> push -> land ->
complete, or are cancelled / fail at any point, in random orders.  Invariants checked after every
event: live extents never overlap, a landed request's pool blocks hold exactly its prompt KV, the
block pool stays consistent, and once everything drains every extent and block is free again."""
import random

import pytest
import torch

from mxserve.disagg.kv_transfer import Extents, KVTransferAgent
from mxserve.engine.kv_manager import KVCacheManager
from mxserve.engine.request import Request, SamplingParams
from mxserve.engine.scheduler import Scheduler


class _Runner:  # the parts of ModelRunner the agent touches
    def __init__(self, nb: int):
        self.kv_cache = torch.zeros(nb, 2, 2, 1, 16, 4)
        self.block_bytes = self.kv_cache[0].numel() * self.kv_cache.element_size()
        self.args = type("A", (), {"block_size": 16, "max_model_len": 512})()


@pytest.mark.parametrize("seed", range(12))
def test_extents_random_interleavings(seed):
    rng = random.Random(seed)
    ext = Extents(300)
    live = {}
    for step in range(2000):
        op = rng.random()
        if op < 0.55:
            k = rng.randint(1, 40)
            start = ext.acquire(k)
            if start is not None:
                rng_ = range(start, start + k)
                for o in live.values():
                    assert not (set(rng_) & set(o)), "overlapping live extents"
                assert 0 <= start and start + k <= 300
                live[step] = rng_
        elif live:
            key = rng.choice(list(live))
            r = live.pop(key)
            ext.release(r.start, len(r))
    for r in live.values():
        ext.release(r.start, len(r))
    assert ext.free_blocks() == 300
    assert ext.acquire(300) == 0  # fully coalesced again


@pytest.mark.parametrize("seed", range(8))
def test_kv_transfer_random_interleavings(seed, monkeypatch):
    from mxserve.disagg import kv_transfer
    monkeypatch.setattr(kv_transfer, "SHM_BYTES", 64 * 2048)  # a small shm arena: fills up, falls back
    rng = random.Random(seed)
    torch.manual_seed(seed)
    NB = 400
    dec_runner, pre_runner = _Runner(NB), _Runner(NB)
    dec_agent = KVTransferAgent(dec_runner, "xgmi")  # CPU: host backend + shm arena
    pre_agent = KVTransferAgent(pre_runner, "xgmi")
    target = dec_agent.descriptor()
    assert target["backend"] == "host" and target.get("shm_name")
    kvm = KVCacheManager(NB, 16, enable_prefix_caching=False)
    sched = Scheduler(kvm, max_num_seqs=24, max_model_len=512)
    pending = {}  # rid -> (req, dst blocks, shm extent start, prefill-side src block ids)
    pre_free = list(range(NB))  # the prefill worker's own pool: a block holds one request's KV
    done = 0
    try:
        for step in range(600):
            ev = rng.random()
            if ev < 0.4:  # a new request arrives at the decode worker
                rid = f"r{step}"
                n = rng.randint(1, 120)
                req = Request(rid, [rng.randint(3, 500) for _ in range(n)], SamplingParams(max_tokens=3),
                              disagg_role="remote_prefill")
                if not sched.reserve_remote(req):
                    continue
                dst = list(req.block_ids[: -(-n // 16)])
                if len(dst) > len(pre_free):
                    sched.cancel_remote(rid)
                    continue
                start = dec_agent.acquire_shm(len(dst))
                # the prefill worker's blocks (random, owned by this request) with recognisable content
                rng.shuffle(pre_free)
                src = [pre_free.pop() for _ in dst]
                for j, b in enumerate(src):
                    pre_runner.kv_cache[b].fill_(float(hash((rid, j)) % 1000))
                pending[rid] = (req, dst, start, src)
            elif ev < 0.75 and pending:  # a prefill finishes: push, land, complete
                rid = rng.choice(list(pending))
                req, dst, start, src = pending.pop(rid)
                if start is not None:
                    pre_agent.push_shm(src, target, start)
                    dec_agent.land_shm(start, dst)
                else:  # shm arena full: host-staged bytes
                    dec_agent.write_blocks(dst, pre_agent.read_blocks(src))
                for j, b in enumerate(dst):
                    assert torch.all(dec_runner.kv_cache[b] == float(hash((rid, j)) % 1000)), "wrong KV landed"
                pre_free.extend(src)
                sched.complete_remote(rid, 7)
                done += 1
            elif ev < 0.85 and pending:  # client goes away / prefill fails before the KV lands
                rid = rng.choice(list(pending))
                req, dst, start, src = pending.pop(rid)
                if start is not None:
                    dec_agent.release_shm(start, len(dst))
                pre_free.extend(src)
                sched.cancel_remote(rid)
            else:  # the decode engine runs a step: running requests make progress and finish
                so = sched.schedule()
                if not so.is_empty:
                    sched.update(so, {s.req.request_id: 9 for s in so.all() if s.sample})
            assert kvm.check_invariants()
            assert len(sched.running) + len(sched.remote) <= 24
        # drain
        for rid in list(pending):
            req, dst, start, src = pending.pop(rid)
            if start is not None:
                dec_agent.release_shm(start, len(dst))
            sched.cancel_remote(rid)
        while sched.has_work():
            so = sched.schedule()
            sched.update(so, {s.req.request_id: 9 for s in so.all() if s.sample})
        assert done > 20
        assert kvm.num_free() == NB and kvm.check_invariants()
        assert dec_agent._shm_ext.free_blocks() == dec_agent.shm_blocks
    finally:
        pre_agent.close()
        dec_agent.close()


@pytest.mark.parametrize("reply", ["ok", "reset"])
def test_cancelled_remote_prefill_holds_kv_until_prefill_side_is_done(reply, monkeypatch):
    """the decode side's /prefill POST is cancelled (the client left) while the
    prefill worker is still pushing.  The request id is freed at once (a local-prefill fallback can
    reuse it), but its pool blocks and staging extents stay allocated until the prefill worker has
    replied -- or, for a reply-less failure, the quarantine delay -- so a late push never lands in
    blocks or extents another request owns."""
    import asyncio

    from mxserve.config import EngineArgs
    from mxserve.disagg import kv_transfer
    from mxserve.worker.args import WorkerArgs
    from mxserve.worker.server import Worker
    monkeypatch.setattr(kv_transfer, "SHM_BYTES", 256 * 2048)
    ea = EngineArgs(model="tiny-llama", device="cpu", cpu_num_blocks=256, max_model_len=1024, disagg_mode="decode",
                    load_format="random", seed=7)
    w = Worker(WorkerArgs(engine=ea, host="127.0.0.1", worker_id="dec"))
    w.QUARANTINE_S = 0.5
    kv = w.engine.scheduler.kv
    posted = []

    class _Resp:
        status = 200

        async def json(self):
            return {"first_token": 5, "via": "shm", "transfer_s": 0.0}

    class _Post:
        def __init__(self, gate):
            self.gate = gate

        async def __aenter__(self):
            posted.append(True)
            await self.gate.wait()  # the prefill worker is still computing / pushing
            if reply == "reset":
                raise ConnectionResetError("prefill worker connection reset")
            return _Resp()

        async def __aexit__(self, *exc):
            return False

    async def main():
        gate = asyncio.Event()

        class _Sess:
            def post(self, url, json=None):
                return _Post(gate)

        async def http():
            return _Sess()
        w.http = http
        free0, shm0 = kv.num_free(), w.agent._shm_ext.free_blocks()
        toks = list(range(3, 103))  # 100 tokens = 7 blocks
        t = asyncio.ensure_future(w._remote_prefill("r1", toks, SamplingParams(max_tokens=4), "http://prefill"))
        while not posted:
            await asyncio.sleep(0.01)
        assert kv.num_free() == free0 - 7 and w.agent._shm_ext.free_blocks() == shm0 - 7
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        for _ in range(100):  # the engine thread runs the detach
            if "r1" not in w.engine.requests:
                break
            await asyncio.sleep(0.01)
        assert "r1" not in w.engine.requests and "r1" not in w.engine.scheduler.remote
        await asyncio.sleep(0.2)
        # still held: the prefill worker may push into them at any moment
        assert kv.num_free() == free0 - 7 and w.agent._shm_ext.free_blocks() == shm0 - 7
        assert w.kv_quarantined == 1
        # the id is reusable right away (the local fallback path re-adds it)
        await w.aeng.submit(w.engine.add_request, toks, SamplingParams(max_tokens=1), "r1")
        gate.set()  # the prefill side replies (or its connection drops)
        for _ in range(300):
            if w.kv_quarantined == 0:
                break
            await asyncio.sleep(0.01)
        assert w.kv_quarantined == 0
        for _ in range(300):  # the fallback request finishes; then everything is free again
            if not w.engine.has_unfinished() and kv.num_free() == free0:
                break
            await asyncio.sleep(0.02)
        assert w.agent._shm_ext.free_blocks() == shm0
        assert kv.num_free() == free0

    try:
        asyncio.run(main())
    finally:
        w.aeng.shutdown()
        w.agent.close()
