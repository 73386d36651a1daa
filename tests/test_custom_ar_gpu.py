"""Custom IPC all-reduce (K18) between ranks that share GPU 0 (the 1-GPU test box): each rank is a
process with its own buffers, exported and mapped over hipIpc exactly as across xGMI peers.  Checks
exact sums for several sizes back to back (parity reuse across calls of different sizes), in place
and out of place, and inside a captured hipGraph (device-side epochs).  The parent never
initialises HIP."""
import multiprocessing as mp
import os
import traceback

import pytest

pytestmark = pytest.mark.gpu

SIZES = [8, 2048, 4096 * 8, 1 << 20, 4096 * 8 + 8, 8, 24, 1 << 21]


def _rank(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        from mxserve.parallel.custom_allreduce import CustomAllReduce
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        car = CustomAllReduce.create(dist.group.WORLD, torch.device("cuda:0"), max_bytes=4 << 20)
        assert car.world == world
        errs = []

        def inp(n, call):  # exact in bf16: small integers
            return ((torch.arange(n, device="cuda:0") % 13) + rank * 3 + call).to(torch.bfloat16)

        def want(n, call):
            return sum(((torch.arange(n, device="cuda:0") % 13) + r * 3 + call) for r in range(world)).float()

        # pass 0: default choice (one-shot below 512 KiB, two-shot above for world > 2);
        # pass 1: two-shot for every size (world > 2), interleaved epochs with pass 0's calls
        calls = [(n, 0) for n in SIZES] + [(n, 1) for n in SIZES]
        for call, (n, forced) in enumerate(calls):
            car.two_shot_min_bytes = 0 if forced else 512 << 10
            x = inp(n, call)
            if call % 2:
                out = torch.empty_like(x)
                car.all_reduce(x, out)
            else:
                out = car.all_reduce(x)
            torch.cuda.synchronize()
            if not torch.equal(out.float(), want(n, call)):
                errs.append(f"call {call} n={n}: max err {(out.float() - want(n, call)).abs().max().item()}")
        # equal-split IPC all-to-all (EP dispatch), interleaved with all-reduces: bf16 segments of
        # 16-byte multiples and int32 segments of 4-byte multiples
        for call, (seg, dt) in enumerate([(24, torch.bfloat16), (3, torch.int32), (4096, torch.bfloat16), (5, torch.int32)]):
            x = torch.cat([torch.arange(seg, device="cuda:0") + 1000 * rank + d for d in range(world)]).to(dt)
            out = torch.empty_like(x)
            assert car.can_all_to_all(x)
            car.all_to_all(out, x)
            car.all_reduce(inp(64, call))
            torch.cuda.synchronize()
            exp = torch.cat([torch.arange(seg, device="cuda:0") + 1000 * r + rank for r in range(world)]).to(dt)
            if not torch.equal(out, exp):
                errs.append(f"a2a call {call} seg={seg} {dt}")
        # hipGraph: 3 captured all-reduces (one two-shot when world > 2), replayed twice
        car.two_shot_min_bytes = 512 << 10
        xs = [inp(4096 if i != 1 else 1 << 19, 20 + i) for i in range(3)]
        bufs = [x.clone() for x in xs]
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for b in bufs:
                    car.all_reduce(b)
        for rep in range(2):
            for b, x in zip(bufs, xs):
                b.copy_(x)
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            for i, b in enumerate(bufs):
                if not torch.equal(b.float(), want(b.numel(), 20 + i)):
                    errs.append(f"graph rep {rep} buf {i}")
        # a KV transfer agent in the same process maps a peer's arena and closes it (engine teardown):
        # only that mapping goes; the all-reduce's peer slots (same IPC table) must stay mapped
        from mxserve import ops
        ext = ops.ext()
        arena = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda:0")
        handle, off = ext.ipc_export_pool(arena)
        handles = [None] * world
        dist.all_gather_object(handles, (bytes(handle), int(off)))
        peer_h, peer_off = handles[(rank + 1) % world]
        ext.ipc_open_pool(peer_h, peer_off)
        # a second user of the same mapping in this process takes a reference of its own: one
        # user's close leaves the mapping in place for the other (comm.cpp refcount)
        p2 = ext.ipc_open_pool(peer_h, peer_off)
        if ext.ipc_open_refs(peer_h) != 2:
            errs.append(f"refs after two opens: {ext.ipc_open_refs(peer_h)}")
        ext.ipc_close(peer_h)
        if ext.ipc_open_refs(peer_h) != 1:
            errs.append(f"refs after one close: {ext.ipc_open_refs(peer_h)}")
        torch.cuda.synchronize()
        del p2
        dist.barrier()
        ext.ipc_close(peer_h)
        if ext.ipc_open_refs(peer_h) != 0:
            errs.append("mapping still referenced after the last close")
        x = inp(4096, 40)
        out = car.all_reduce(x)
        torch.cuda.synchronize()
        if not torch.equal(out.float(), want(4096, 40)):
            errs.append("all-reduce after an agent's ipc_close")
        dist.barrier()
        assert car.check(), ("error word raised", car.diagnose())
        dist.barrier()
        q.put((rank, errs))
    except BaseException:  # noqa: BLE001
        q.put((rank, [traceback.format_exc()]))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_custom_allreduce_ranks_on_one_gpu(world):
    import socket
    import torch
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in the test process; run this file on its own")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=180) for _ in range(world))
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res[r] == [], res[r]
