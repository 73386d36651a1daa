"""Llama-3-70B tensor parallelism (BASELINE config 4) rehearsed on the 1-GPU test box:
  * 8 TP ranks share GPU 0 with the real 70B layer shapes (H 8192, 64 q / 8 kv heads of 128,
    FFN 28672, vocab 128256; 2 layers): each rank holds its TP=8 shard (1 KV head per rank) and the
    logits must match the unsharded model.  The group is gloo (RCCL refuses ranks on one device);
    the attention / MLP all-reduces run the custom IPC all-reduce kernel (on by default for TP <= 8),
    two-shot at these message sizes.
  * a TP=4 engine started the way a worker starts it (start_tp_group: rank 0 + `python -m
    mxserve.worker.tp` followers, per-step inputs through the /dev/shm ring, decode hipGraphs that
    capture the custom all-reduce) generates the same greedy tokens as TP=1.
On an 8-GPU node the same code runs one rank per GPU over RCCL + xGMI."""
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import traceback

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODEL_70B_2L = "meta-llama/Meta-Llama-3-70B-Instruct@layers=2"
MIXTRAL_2L = "mistralai/Mixtral-8x7B-Instruct-v0.1@layers=2"


def _md(n, dev):
    import torch
    from mxserve.models.llama import AttnMetadata
    nb = (n + 15) // 16
    pos = torch.arange(n, device=dev)
    qsl = torch.tensor([0, n], dtype=torch.int32, device=dev)
    return AttnMetadata(positions=pos, slot_mapping=pos.clone(), block_tables=torch.arange(
        nb, dtype=torch.int32, device=dev).unsqueeze(0), seq_lens=torch.tensor([n], dtype=torch.int32, device=dev),
        query_start_loc=qsl, logits_indices=torch.arange(n, device=dev), num_decodes=0, num_prefills=1,
        num_prefill_tokens=n, max_query_len=n, max_seq_len=n, prefill_query_start_loc=qsl)


def _logits(full, n=40, model=MODEL_70B_2L, moe_dispatch="allreduce"):
    import torch
    from mxserve.models.config import get_model_config
    from mxserve.models.llama import build_model
    cfg = get_model_config(model)
    m = build_model(cfg, torch.device("cuda:0"), torch.bfloat16, moe_dispatch)
    m.load_full_state(full)
    ids = torch.randint(3, cfg.vocab_size, (n,), generator=torch.Generator().manual_seed(2)).to("cuda:0")
    kv = torch.zeros(4, cfg.num_layers, 2, m.nkv, 16, cfg.head_dim, dtype=torch.bfloat16, device="cuda:0")
    from mxserve.parallel import comm
    if comm.get_tp().tp_size > 1 and not cfg.is_moe:  # first-call loads before any peer waits (comm.py)
        with torch.inference_mode(), comm.collectives_local():
            m.compute_logits(m.forward(ids, _md(n, "cuda:0"), kv))
    with torch.inference_mode():
        out = m.compute_logits(m.forward(ids, _md(n, "cuda:0"), kv)).float().cpu()
    del m
    return out


def _rank(rank, world, port, q, model=MODEL_70B_2L, moe_dispatch="allreduce"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        os.environ.pop("MXS_CUSTOM_AR", None)  # the default
        import torch
        torch.cuda.set_device(0)
        from mxserve.models.config import get_model_config
        from mxserve.models.weights import random_full_state
        from mxserve.parallel import comm
        st = comm.init_distributed(world, backend="gloo", device=torch.device("cuda:0"))
        assert st.custom_ar is not None, "custom all-reduce should be on by default for TP <= 8"
        cfg = get_model_config(model)
        full = random_full_state(cfg, seed=4, std=0.02, dtype=torch.bfloat16, device="cuda:0")
        got = _logits(full, model=model, moe_dispatch=moe_dispatch)
        assert st.custom_ar.check(), ("custom all-reduce timed out", st.custom_ar.diagnose())
        ref = None
        if rank == 0:
            comm.set_tp(comm.ParallelState())  # the same weights unsharded, in this process
            ref = _logits(full, model=model, moe_dispatch="allreduce")
            comm.set_tp(st)
        del full
        torch.distributed.barrier()
        q.put((rank, got.numpy(), None if ref is None else ref.numpy(), None))
    except BaseException:  # noqa: BLE001
        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("model,moe_dispatch", [(MODEL_70B_2L, "allreduce"), (MIXTRAL_2L, "a2a")])
def test_tp8_shapes_on_one_gpu_match_tp1(model, moe_dispatch):
    """Llama-3-70B TP=8 (1 KV head per rank) and Mixtral-8x7B EP=8 (one expert per rank, tokens
    dispatched by the device-side IPC all-to-all) with the real layer shapes, 2 layers."""
    import torch
    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in the test process")
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q, model, moe_dispatch)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = {}
        for _ in range(world):
            r, g, ref, err = q.get(timeout=300)
            res[r] = (g, ref, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res[r][2] is None, res[r][2]
    ref = torch.from_numpy(res[0][1])
    scale = ref.abs().max().item()
    for r in range(world):
        got = torch.from_numpy(res[r][0])
        row_err = (got - ref).abs().amax(-1)
        # bf16: 8-way sharded GEMMs + the all-reduce sum order vs one unsharded GEMM (MoE: a near-tied
        # router score may pick another expert for a token)
        assert (row_err < 0.05 * scale).float().mean().item() > (0.9 if moe_dispatch == "a2a" else 0.99), row_err
        assert (got.argmax(-1) == ref.argmax(-1)).float().mean().item() > 0.9


def _ep_rank(rank, world, port, q, T):
    """One EP rank of a Mixtral-shaped MoE layer (H 4096, I 14336, 8 experts, top-2): this rank owns
    expert `rank`; the reference (rank 0) recomputes every slice's routing with the very same router
    call the rank made (same rows, same kernel), so routing is identical by construction and the only
    differences left are bf16 expert GEMMs vs an fp32 reference."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        os.environ.pop("MXS_CUSTOM_AR", None)
        import torch
        import torch.nn.functional as F
        torch.cuda.set_device(0)
        from mxserve import ops
        from mxserve.parallel import comm
        from mxserve.parallel.expert import moe_a2a
        st = comm.init_distributed(world, backend="gloo", device=torch.device("cuda:0"))
        assert st.custom_ar is not None
        H, I, E, K = 4096, 14336, 8, 2
        g = torch.Generator(device="cuda:0").manual_seed(11)
        x = (torch.randn(T, H, device="cuda:0", generator=g) * 0.5).to(torch.bfloat16)
        gate = (torch.randn(E, H, device="cuda:0", generator=g) * H ** -0.5).to(torch.bfloat16)

        def expert(e):
            ge = torch.Generator(device="cuda:0").manual_seed(100 + e)
            w13 = (torch.randn(2 * I, H, device="cuda:0", generator=ge) * H ** -0.5).to(torch.bfloat16)
            w2 = (torch.randn(H, I, device="cuda:0", generator=ge) * I ** -0.5).to(torch.bfloat16)
            return w13, w2

        w13, w2 = expert(rank)
        with torch.inference_mode():
            got = moe_a2a(x, gate, w13.unsqueeze(0).contiguous(), w2.unsqueeze(0).contiguous(), K, rank, world,
                          st.group)
        torch.cuda.synchronize()
        assert st.custom_ar.check(), ("custom all-reduce timed out", st.custom_ar.diagnose())
        ref = None
        if rank == 0:
            S = (T + world - 1) // world
            tws, tids = [], []
            with torch.inference_mode():
                for r in range(world):  # the router exactly as each rank ran it on its padded slice
                    lo, hi = min(T, r * S), min(T, r * S + S)
                    hs = torch.zeros(S, H, dtype=x.dtype, device=x.device)
                    hs[:hi - lo] = x[lo:hi]
                    tw, tid = ops.moe_topk_softmax(F.linear(hs, gate), K)
                    tws.append(tw[:hi - lo].float())
                    tids.append(tid[:hi - lo].long())
                tw, tid = torch.cat(tws), torch.cat(tids)
                ref = torch.zeros(T, H, device=x.device)
                xf = x.float()
                for e in range(E):
                    rows, j = (tid == e).nonzero(as_tuple=True)
                    if rows.numel() == 0:
                        continue
                    a, b = expert(e)
                    hgu = xf[rows] @ a.float().t()
                    act = F.silu(hgu[:, :I]) * hgu[:, I:]
                    ref.index_add_(0, rows, (act @ b.float().t()) * tw[rows, j].unsqueeze(1))
                ref = ref.cpu().numpy()
        torch.distributed.barrier()
        q.put((rank, got.float().cpu().numpy(), ref, None))
    except BaseException:  # noqa: BLE001
        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("T", [600, 6000])
def test_ep8_moe_layer_identical_routing(T):
    """Mixtral EP = 8 MoE layer (8 ranks on GPU 0, device-side IPC dispatch): with routing identical
    by construction every row must match the fp32 reference within bf16 GEMM error -- no row may be
    off (a misrouted row is off by O(1)).  T = 6000 puts 750 tokens in each rank's slice: two
    slot-sized dispatch chunks (the prefill path above 4,096 tokens)."""
    import numpy as np
    import torch
    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in the test process")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ep_rank, args=(r, world, port, q, T)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = {}
        for _ in range(world):
            r, g, ref, err = q.get(timeout=300)
            res[r] = (g, ref, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res[r][2] is None, res[r][2]
    ref = res[0][1]
    scale = np.abs(ref).max()
    for r in range(world):
        got = res[r][0]
        assert got.shape == ref.shape
        row_err = np.abs(got - ref).max(-1)
        assert row_err.max() < 0.02 * scale, (r, float(row_err.max() / scale), int(row_err.argmax()))


_ENGINE_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, os.environ["MXS_ROOT"])
tp = int(sys.argv[1])
from mxserve.config import EngineArgs
args = EngineArgs(model="small-llama", device="cuda", tensor_parallel_size=tp, num_gpu_blocks=2048,
                  max_model_len=1024, max_num_seqs=16, cuda_graph_max_bs=8, load_format="random_full", seed=5)
if tp > 1:
    from mxserve.worker.tp import start_tp_group, stop_tp_group
    start_tp_group(args)
from mxserve.engine.engine import LLMEngine
from mxserve.engine.request import SamplingParams
from mxserve.parallel.comm import get_tp
eng = LLMEngine(args)
prompts = [list(range(100, 160)), [7, 8, 9] * 11, list(range(1000, 1300))]
out = eng.generate(prompts, SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True))
st = get_tp()
info = {"tokens": out, "graphs": sorted(eng.runner.graphs), "ring_steps": st.meta_ring.steps if st.meta_ring else 0,
        "ring_fallbacks": st.meta_ring.gloo_fallbacks if st.meta_ring else -1,
        "custom_ar": bool(st.custom_ar is not None and not st.custom_ar.disabled)}
eng.shutdown()
if tp > 1:
    stop_tp_group()
print("RESULT " + json.dumps(info), flush=True)
"""


def _run_engine(tp: int, tmp_path, fused_tp1: bool = False) -> dict:
    # the decode-GEMM tuner picks kernels by timing (noise-dependent per run); both sides stay on
    # hipBLASLt so the comparison isolates the TP path (the kernel has its own numerics tests).  The
    # TP = 1 fused prefill chain (llama.py _forward_pf: residual added inside the o / down GEMM, one
    # bf16 rounding instead of two) is off for the same reason: it has its own test
    # (test_engine_gpu.py test_fused_prefill_chain_matches_unfused)
    env = dict(os.environ, MXS_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT, MXS_DECODE_GEMM="off",
               MXS_PF_FUSED="0")
    if fused_tp1:  # the default TP = 1 chain (fused prefill on)
        env.pop("MXS_PF_FUSED", None)
    env.pop("MXS_CUSTOM_AR", None)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", _ENGINE_SCRIPT, str(tp)], capture_output=True, text=True, timeout=300,
                       env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_tp4_engine_on_one_gpu_matches_tp1(tmp_path):
    ref = _run_engine(1, tmp_path)
    got = _run_engine(4, tmp_path)
    assert got["graphs"] and got["custom_ar"], got
    assert got["ring_steps"] >= 12 and got["ring_fallbacks"] == 0, got
    same = sum(a == b for ra, rb in zip(ref["tokens"], got["tokens"]) for a, b in zip(ra, rb))
    total = sum(len(x) for x in ref["tokens"])
    # greedy bf16: a 4-way sharded reduction order may flip a near-tied argmax late in a sequence
    assert all(ra[:4] == rb[:4] for ra, rb in zip(ref["tokens"], got["tokens"])), (ref, got)
    assert same >= 0.9 * total, (ref, got)


def test_tp4_engine_matches_the_default_tp1_chain(tmp_path):
    """TP = 4 against the TP = 1 engine as it runs by default (fused prefill chain
    on: RMSNorm inside the consumer GEMMs, residual adds inside o / down).  The two differ in bf16
    rounding order on both sides, so the check is on greedy tokens: every prompt's first tokens agree
    and most of the rest."""
    ref = _run_engine(1, tmp_path, fused_tp1=True)
    got = _run_engine(4, tmp_path)
    same = sum(a == b for ra, rb in zip(ref["tokens"], got["tokens"]) for a, b in zip(ra, rb))
    total = sum(len(x) for x in ref["tokens"])
    assert all(ra[:2] == rb[:2] for ra, rb in zip(ref["tokens"], got["tokens"])), (ref, got)
    assert same >= 0.8 * total, (ref, got)
