"""Tensor parallelism on CPU (gloo, world size 2): a TP=2 engine (driver + follower process) must
produce the same greedy tokens as TP=1 with the same unsharded weights."""
import os

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    from tests.serving_utils import free_port
    return free_port()


PROMPTS = [[5, 9, 13, 200, 31, 7, 77, 8, 100, 3] * 3, [44, 45, 46], list(range(60, 140))]


def _args(model, tp, moe_dispatch="allreduce"):
    from mxserve.config import EngineArgs
    return EngineArgs(model=model, device="cpu", tensor_parallel_size=tp, cpu_num_blocks=128, max_model_len=512,
                      max_num_batched_tokens=48, load_format="random_full", seed=3, moe_dispatch=moe_dispatch)


def _rank(rank, world, port, model, q, moe_dispatch="allreduce"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from mxserve.engine.request import SamplingParams
    from mxserve.parallel.comm import init_distributed
    init_distributed(world, backend="gloo")
    if rank == 0:
        from mxserve.engine.engine import LLMEngine
        eng = LLMEngine(_args(model, world, moe_dispatch))
        out = eng.generate(PROMPTS, SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))
        eng.shutdown()
        from mxserve.parallel.comm import get_tp
        ring = get_tp().meta_ring
        q.put((out, ring.steps if ring else 0, ring.gloo_fallbacks if ring else -1))
    else:
        from mxserve.engine.model_runner import ModelRunner
        from mxserve.models.config import get_model_config
        runner = ModelRunner(_args(model, world, moe_dispatch), get_model_config(model))
        runner.follower_loop()
    # tear the gloo group down before the interpreter exits (its threads otherwise can abort at exit)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("model,moe_dispatch", [("tiny-llama", "allreduce"), ("tiny-mixtral", "allreduce"),
                                                ("tiny-mixtral", "a2a")])
def test_tp2_matches_tp1(model, moe_dispatch):
    from mxserve.engine.engine import LLMEngine
    from mxserve.engine.request import SamplingParams
    ref = LLMEngine(_args(model, 1)).generate(PROMPTS, SamplingParams(max_tokens=6, temperature=0.0,
                                                                      ignore_eos=True))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, model, q, moe_dispatch)) for r in range(2)]
    for p in procs:
        p.start()
    out, ring_steps, fallbacks = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out == ref
    # every step's inputs went to the follower through the /dev/shm ring, none over gloo
    assert ring_steps > 6 and fallbacks == 0


def _ar_norm_rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from mxserve.ops import reference as ref
    from mxserve.parallel.comm import init_distributed, tp_add_rms_norm, tp_linear_add_rms_norm
    init_distributed(world, backend="gloo")
    g = torch.Generator().manual_seed(7)
    x_all = torch.randn(world, 5, 64, generator=g)
    w_all = torch.randn(world, 64, 32, generator=g) * 0.2
    a_all = torch.randn(world, 5, 32, generator=g)
    res0 = torch.randn(5, 64, generator=g)
    nw = 1 + 0.1 * torch.randn(64, generator=g)
    h, res = tp_add_rms_norm(x_all[rank].clone(), res0.clone(), nw, 1e-5)
    want_h, want_res = ref.fused_add_rms_norm(x_all.sum(0), res0.clone(), nw, 1e-5)
    h2, res2 = tp_linear_add_rms_norm(a_all[rank].clone(), w_all[rank], res0.clone(), nw, 1e-5)
    y = sum(a_all[r] @ w_all[r].T for r in range(world))
    want_h2, want_res2 = ref.fused_add_rms_norm(y, res0.clone(), nw, 1e-5)
    ok = all(torch.allclose(u, v, atol=1e-4, rtol=1e-4) for u, v in
             ((h, want_h), (res, want_res), (h2, want_h2), (res2, want_res2)))
    # collectives_local (the per-rank warm-up before collective warm-ups): no peer is involved
    # (every collective call raises here) and each epilogue uses this rank's partial alone
    import torch.distributed as dist
    from mxserve.parallel import comm
    real = (dist.all_reduce, dist.all_gather)

    def boom(*a, **k):
        raise AssertionError("collective called in local mode")
    dist.all_reduce = dist.all_gather = boom
    try:
        with comm.collectives_local():
            hl, resl = tp_add_rms_norm(x_all[rank].clone(), res0.clone(), nw, 1e-5)
            hl2, _ = tp_linear_add_rms_norm(a_all[rank].clone(), w_all[rank], res0.clone(), nw, 1e-5)
            ar = comm.tp_all_reduce(x_all[rank].clone())
            ag = comm.tp_all_gather(a_all[rank], dim=-1)
    finally:
        dist.all_reduce, dist.all_gather = real
    wl, wresl = ref.fused_add_rms_norm(x_all[rank], res0.clone(), nw, 1e-5)
    wl2, _ = ref.fused_add_rms_norm(a_all[rank] @ w_all[rank].T, res0.clone(), nw, 1e-5)
    ok = ok and all(torch.allclose(u, v, atol=1e-4, rtol=1e-4) for u, v in
                    ((hl, wl), (resl, wresl), (hl2, wl2), (ar, x_all[rank])))
    ok = ok and ag.shape == (5, 32 * world) and torch.equal(ag[:, :32], a_all[rank])
    q.put((rank, ok))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_tp_add_rms_norm_gloo():
    """comm.tp_add_rms_norm / tp_linear_add_rms_norm (the TP > 1 residual epilogues: one fused
    all-reduce + add + RMSNorm kernel on the GPU) reduce the row-parallel partials over the group and
    match the unsharded add + RMSNorm (CPU, gloo, 2 ranks)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_ar_norm_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
    assert res == {0: True, 1: True}
