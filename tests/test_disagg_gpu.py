"""Disaggregated KV transfer over HIP IPC between two processes (the xgmi backend of
mxserve/disagg/kv_transfer.py): the decode process exports its staging arena, the
prefill process maps it and pushes a request's blocks with the copy kernel, the decode process lands
them in its (serving-sized) pool.  Both processes share GPU 0 on
the 1-GPU test box (same code path as two GPUs: IPC mapping + device-side copy; xGMI is only the
wire).  The parent never initialises HIP: it only spawns the two ranks."""
import multiprocessing as mp
import os
import traceback

import pytest

pytestmark = pytest.mark.gpu

SMALL = (64, 4, 2, 2, 16, 64)  # [blocks, layers, K/V, kv heads, 16, D]
LARGE = (40000, 16, 2, 8, 16, 64)  # Llama-3.2-1B layout, 21 GB: a serving-sized pool


class _Runner:
    def __init__(self, kv):
        self.kv_cache = kv
        self.block_bytes = kv[0].numel() * kv.element_size()


def _decode_rank(q_out, q_in, SHAPE):
    try:
        import torch
        from mxserve.disagg.kv_transfer import KVTransferAgent
        torch.cuda.set_device(0)
        kv = torch.zeros(SHAPE, dtype=torch.bfloat16, device="cuda:0")
        agent = KVTransferAgent(_Runner(kv), "xgmi")
        desc = agent.descriptor("http://decode")
        dst = [10, 0, 41, 5, SHAPE[0] - 2]
        start = agent.acquire(len(dst))
        assert start is not None
        q_out.put(("desc", desc, start))
        msg = q_in.get(timeout=120)
        assert msg[0] == "done", msg
        expect = msg[1]
        red = tuple(range(1, kv.dim()))
        staged = agent.staging[start:start + len(dst)].float().sum(dim=red).cpu().tolist()
        agent.land(start, dst)
        torch.cuda.synchronize()
        got = kv[dst].float().sum(dim=red).cpu().tolist()
        assert got == staged, f"landing copy lost data: staged {staged} landed {got}"
        untouched = [b for b in range(min(SHAPE[0], 64)) if b not in dst]
        q_out.put(("result", got, expect, float(kv[untouched].float().abs().sum())))
    except BaseException:  # noqa: BLE001
        q_out.put(("error", traceback.format_exc()))


def _prefill_rank(q_out, q_in, SHAPE):
    try:
        import torch
        from mxserve.disagg.kv_transfer import KVTransferAgent
        torch.cuda.set_device(0)
        g = torch.Generator(device="cuda:0").manual_seed(5)
        kv = torch.randn(SHAPE, generator=g, device="cuda:0").to(torch.bfloat16)
        agent = KVTransferAgent(_Runner(kv), "xgmi")
        desc, start = q_in.get(timeout=120)
        src = [3, 7, 8, 20, SHAPE[0] - 1]
        agent.connect(desc)
        secs = agent.push_xgmi(src, desc, start)
        expect = kv[src].float().sum(dim=tuple(range(1, kv.dim()))).cpu().tolist()
        q_out.put(("done", expect, secs))
    except BaseException:  # noqa: BLE001
        q_out.put(("error", traceback.format_exc()))




@pytest.mark.parametrize("shape", [SMALL, LARGE], ids=["small", "21GB"])
def test_ipc_block_push_between_processes(shape):
    import torch
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in the test process; run this file on its own")
    ctx = mp.get_context("spawn")
    env_before = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    d_out, d_in, p_out, p_in = ctx.Queue(), ctx.Queue(), ctx.Queue(), ctx.Queue()
    dec = ctx.Process(target=_decode_rank, args=(d_out, d_in, shape))
    pre = ctx.Process(target=_prefill_rank, args=(p_out, p_in, shape))
    dec.start()
    pre.start()
    try:
        m = d_out.get(timeout=120)
        assert m[0] == "desc", m
        assert m[1]["backend"] == "xgmi" and "handle" in m[1]
        p_in.put((m[1], m[2]))
        done = p_out.get(timeout=120)
        assert done[0] == "done", done
        d_in.put(done)
        res = d_out.get(timeout=120)
        assert res[0] == "result", res
        _, got, expect, untouched = res
        assert got == pytest.approx(expect, rel=1e-3, abs=1e-2)
        assert untouched == 0.0
    finally:
        for p in (dec, pre):
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
        if env_before is None:
            os.environ.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
        else:
            os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = env_before
    assert dec.exitcode == 0 and pre.exitcode == 0
