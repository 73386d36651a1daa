"""Expert parallelism with all-to-all dispatch (mxserve/parallel/expert.py) on
CPU/gloo: every rank's MoE output must equal the unsharded reference MoE over the whole batch, for
both dispatch layouts (fixed-capacity / exact counts), world sizes 1, 2 and 4, and batches smaller
than the world (empty token slices)."""
import os

import pytest
import torch
import torch.multiprocessing as mp

E, K, H, I = 8, 2, 32, 48


def _port():
    from tests.serving_utils import free_port
    return free_port()


def _weights():
    g = torch.Generator().manual_seed(0)
    gate = torch.randn(E, H, generator=g)
    w13 = torch.randn(E, 2 * I, H, generator=g) / H ** 0.5
    w2 = torch.randn(E, H, I, generator=g) / I ** 0.5
    return gate, w13, w2


def _reference(h):
    from mxserve.ops import reference as ref
    gate, w13, w2 = _weights()
    tw, tid = ref.moe_topk_softmax(h @ gate.t(), K)
    return ref.moe_experts(h, w13, w2, tw, tid, 0)


def _run(rank, world, port, Ts, layout, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from mxserve.parallel.expert import moe_a2a
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gate, w13, w2 = _weights()
    el = E // world
    res = []
    for T in Ts:
        h = torch.randn(T, H, generator=torch.Generator().manual_seed(T))
        out = moe_a2a(h, gate, w13[rank * el:(rank + 1) * el], w2[rank * el:(rank + 1) * el], K, rank, world,
                      dist.group.WORLD, force_layout=layout)
        res.append(out.numpy())  # by value: a shared-fd tensor dies with this process
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("layout", ["fixed", "variable"])
def test_moe_a2a_matches_reference(world, layout):
    Ts = [1, 3, 16, 37]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_run, args=(r, world, port, Ts, layout, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i, T in enumerate(Ts):
        h = torch.randn(T, H, generator=torch.Generator().manual_seed(T))
        want = _reference(h)
        for r in range(world):
            torch.testing.assert_close(torch.from_numpy(got[r][i]), want, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("layout", ["fixed", "variable"])
def test_moe_a2a_single_rank(layout):
    from mxserve.parallel.expert import moe_a2a
    gate, w13, w2 = _weights()
    for T in (1, 5, 64):
        h = torch.randn(T, H)
        torch.testing.assert_close(moe_a2a(h, gate, w13, w2, K, 0, 1, None, force_layout=layout), _reference(h),
                                   rtol=1e-4, atol=1e-4)


def test_moe_dispatch_flag():
    from mxserve.worker.args import parse_worker_args
    wa = parse_worker_args(["--model", "tiny-mixtral", "--tp", "2", "--moe-dispatch", "a2a"])
    assert wa.engine.moe_dispatch == "a2a"
    with pytest.raises(ValueError):
        from mxserve.models.config import get_model_config
        from mxserve.models.llama import build_model
        build_model(get_model_config("tiny-mixtral"), "cpu", torch.float32, "bogus")
