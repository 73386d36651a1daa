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
