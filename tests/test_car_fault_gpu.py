"""Custom all-reduce fault handling on the GPU (VERDICT r4 "next round" #1):
  * a TP=4 engine (4 ranks sharing GPU 0, per-step inputs over the /dev/shm ring, decode hipGraphs
    holding the custom all-reduce) whose rank 2 -- or the driver rank 0 -- stalls for 1.5 s before
    one step while the wait budget is 0.3 s: the peers give up, the step is detected as faulted,
    and no request receives a token from it.  Every stream must equal the fault-free TP=4 run token
    for token (greedy), the fault is counted, the path is re-armed (graphs kept) -- or, with
    MXS_CAR_MAX_FAULTS=1, turned off for good and decode continues on the fallback path;
  * the give-up record names the kernel, the block and the peer whose flag was missing.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, os.environ["MXS_ROOT"])
from mxserve.config import EngineArgs
args = EngineArgs(model="small-llama", device="cuda", tensor_parallel_size=4, num_gpu_blocks=2048,
                  max_model_len=1024, max_num_seqs=16, cuda_graph_max_bs=8, load_format="random_full", seed=5)
from mxserve.worker.tp import start_tp_group, stop_tp_group
start_tp_group(args)
from mxserve.engine.engine import LLMEngine
from mxserve.engine.request import SamplingParams
from mxserve.parallel.comm import get_tp
eng = LLMEngine(args)
prompts = [list(range(100, 160)), [7, 8, 9] * 11, list(range(1000, 1300))]
out = eng.generate(prompts, SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True))
st = get_tp()
info = {"tokens": out, "graphs": sorted(eng.runner.graphs), "faults": eng.stats()["custom_ar_timeouts"],
        "custom_ar": bool(st.custom_ar is not None and not st.custom_ar.disabled),
        "last_fault": getattr(eng.runner, "last_collective_fault", None)}
eng.shutdown()
stop_tp_group()
print("RESULT " + json.dumps(info), flush=True)
"""


def _run(tmp_path, **extra) -> dict:
    # the two runs must match token for token: no start-up tuner may pick kernels by timing on either
    # side (small-llama's shapes are in no packaged table, so each process would measure afresh and a
    # different prefill GEMM solution rounds differently -- a late near-tie flip, not a fault effect)
    env = dict(os.environ, MXS_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT, MXS_DECODE_GEMM="off",
               MXS_PF_FUSED="0", MXS_HBLT="off", MXS_GEMM_PF="off", MXS_MPLAN="0", **extra)
    env.pop("MXS_CUSTOM_AR", None)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", _SCRIPT], capture_output=True, text=True, timeout=300, env=env,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


@pytest.mark.parametrize("stall_rank,max_faults", [(2, "3"), (0, "3"), (0, "1")])
def test_injected_timeout_never_emits_tokens(tmp_path, stall_rank, max_faults):
    ref = _run(tmp_path)
    assert ref["faults"] == 0 and ref["custom_ar"] and ref["graphs"], ref
    got = _run(tmp_path, MXS_FAULT=f"car_delay:rank={stall_rank}:step=6:ms=1500", MXS_CAR_TIMEOUT_MS="300",
               MXS_CAR_MAX_FAULTS=max_faults)
    assert got["faults"] == 1, got
    if max_faults == "1":  # turned off for good: gloo groups cannot capture, decode runs eagerly
        assert not got["custom_ar"] and not got["graphs"], got
        # the fallback all-reduce rounds differently (gloo sums bf16 partials pairwise): tokens up
        # to the fault are identical, later ones may take the other side of a near-tied argmax
        assert all(a[:4] == b[:4] for a, b in zip(ref["tokens"], got["tokens"])), (ref, got)
        same = sum(x == y for a, b in zip(ref["tokens"], got["tokens"]) for x, y in zip(a, b))
        assert same >= 0.8 * sum(len(a) for a in ref["tokens"]), (ref, got)
    else:  # re-armed: the same graphs keep running the custom kernels -- and the same tokens
        assert got["custom_ar"] and got["graphs"] == ref["graphs"], got
        assert got["tokens"] == ref["tokens"], (ref, got)
    ranks = got["last_fault"]["ranks"]
    gave_up = [r for r in ranks if "gave_up" in r]
    assert gave_up, got["last_fault"]
    for r in gave_up:
        g = r["gave_up"]
        assert r["rank"] != stall_rank and g["missing_peer"] == stall_rank, got["last_fault"]
        assert 0 <= g["block"] < 64 and g["waited_ms"] >= 250, got["last_fault"]
