"""End-to-end disaggregated serving on the GPU: the OpenAI frontend (this process,
CPU only) + a prefill worker and a decode worker started exactly as the manifests start them
(`python -m dynamo.vllm --is-prefill-worker / --is-decode-worker`), both on GPU 0.  The decode
worker reserves blocks and an extent of its IPC staging arena, the prefill worker computes the
prompt and pushes the KV blocks with the copy kernel, the decode worker lands them and streams the
rest.  Runs first in the GPU suite (file name) because the parent must not have initialised HIP
before it starts GPU child processes."""
import os
import subprocess
import sys
import time

import httpx
import pytest

from mxserve.frontend.app import Frontend
from tests.serving_utils import Server, free_port, wait_for

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODEL = "small-llama"


def _worker(role: str, fe_url: str, port: int, log):
    flag = [] if role == "agg" else [f"--is-{role}-worker"]
    cmd = [sys.executable, "-m", "dynamo.vllm", "--model", MODEL] + flag + ["--frontend-url", fe_url,
           "--host", "127.0.0.1", "--port", str(port), "--num-gpu-blocks-override", "4096", "--max-model-len",
           "4096", "--max-num-seqs", "16", "--enforce-eager", "--worker-id", f"{role}-0"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MXS_KV_STAGING_BYTES=str(1 << 30),
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    return subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT)


def test_disaggregated_chat_over_ipc(tmp_path):
    import torch
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in the test process; run this file on its own")
    fe = Frontend(router_mode="kv", ttl=60)
    fs = Server(fe.app).start()
    fe_agg = Frontend(router_mode="kv", ttl=60)  # an aggregated worker (same seed) for greedy parity
    fs_agg = Server(fe_agg.app).start()
    logs = {r: open(tmp_path / f"{r}.log", "w") for r in ("prefill", "decode", "agg")}
    ports = {r: free_port() for r in logs}
    procs = {r: _worker(r, fs_agg.url if r == "agg" else fs.url, ports[r], logs[r]) for r in logs}
    try:
        def ready():
            for r, p in procs.items():
                if p.poll() is not None:
                    raise RuntimeError(f"{r} worker exited:\n" + (tmp_path / f"{r}.log").read_text()[-4000:])
            return len(fe.registry.list()) == 2 and len(fe_agg.registry.list()) == 1
        wait_for(ready, timeout=240, interval=1.0)
        body = {"model": MODEL, "messages": [{"role": "user", "content": "disaggregated " * 40}], "max_tokens": 24,
                "temperature": 0, "ignore_eos": True}
        r = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=120)
        assert r.status_code == 200, r.text
        d = r.json()
        assert d["usage"]["completion_tokens"] == 24
        # the prompt's KV came from the prefill worker over the IPC staging arena (not host-staged)
        m = httpx.get(f"http://127.0.0.1:{ports['decode']}/metrics", timeout=10).text
        moved = [ln for ln in m.splitlines()
                 if ln.startswith("dynamo_component_kv_transfer_bytes_total") and 'backend="xgmi"' in ln]
        assert moved and float(moved[0].split()[-1]) > 0, m[-2000:]
        # greedy parity: the disaggregated answer (prefill GPU -> KV over IPC -> decode) is token for
        # token the aggregated one
        ra = httpx.post(fs_agg.url + "/v1/chat/completions", json=body, timeout=120)
        assert ra.status_code == 200, ra.text
        assert ra.json()["choices"][0]["message"]["content"] == d["choices"][0]["message"]["content"]
        # streaming through the same path, several requests at once
        t0 = time.time()
        outs = []
        for i in range(4):
            b = dict(body, messages=[{"role": "user", "content": f"request {i} " * 30}], max_tokens=8)
            outs.append(httpx.post(fs.url + "/v1/chat/completions", json=b, timeout=120))
        assert all(o.status_code == 200 and o.json()["usage"]["completion_tokens"] == 8 for o in outs)
        assert time.time() - t0 < 120
    finally:
        for p in procs.values():
            p.terminate()
        for p in procs.values():
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        fs.stop()
        fs_agg.stop()
        for f in logs.values():
            f.close()


@pytest.mark.parametrize("form", ["pair", "group"])
def test_pd_pair_pod_launcher(tmp_path, form):
    """The P/D group pod the operator renders: `python -m mxserve.worker.pair` runs the decode and
    prefill workers in one container (pair: MXS_PAIR_*_CMD, one of each; group: MXS_GROUP_SPEC, here
    1 decode + 2 prefill); all register under one group id, the frontend sends the decode worker a
    prefill worker of its own group and the KV moves over IPC."""
    import json
    import torch
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    if torch.cuda.is_initialized():
        pytest.skip("HIP already initialised in the test process")
    fe = Frontend(router_mode="kv", ttl=60)
    fs = Server(fe.app).start()
    common = ["--model", MODEL, "--frontend-url", fs.url, "--host", "127.0.0.1", "--num-gpu-blocks-override", "4096",
              "--max-model-len", "4096", "--max-num-seqs", "16", "--enforce-eager"]
    port = free_port()  # the decode worker's; the prefill worker takes port + 1
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MXS_KV_STAGING_BYTES=str(1 << 30), DYN_SYSTEM_PORT=str(port),
               POD_NAME="pairpod-0", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
               MXS_PAIR_DECODE_CMD=json.dumps([sys.executable, "-m", "dynamo.vllm", "--is-decode-worker"] + common),
               MXS_PAIR_PREFILL_CMD=json.dumps([sys.executable, "-m", "dynamo.vllm", "--is-prefill-worker"] + common))
    env.pop("MXS_WORKER_ID", None)
    n_workers = 2
    if form == "group":
        pre = {"role": "prefill", "cmd": [sys.executable, "-m", "dynamo.vllm", "--is-prefill-worker"] + common, "gpus": 1}
        env["MXS_GROUP_SPEC"] = json.dumps(
            [{"role": "decode", "cmd": [sys.executable, "-m", "dynamo.vllm", "--is-decode-worker"] + common, "gpus": 1},
             pre, pre])
        n_workers = 3
    log = open(tmp_path / "pair.log", "w")
    proc = subprocess.Popen([sys.executable, "-m", "mxserve.worker.pair"], cwd=ROOT, env=env, stdout=log,
                            stderr=subprocess.STDOUT)
    try:
        def ready():
            if proc.poll() is not None:
                raise RuntimeError("pair launcher exited:\n" + (tmp_path / "pair.log").read_text()[-4000:])
            return len(fe.registry.list()) == n_workers
        wait_for(ready, timeout=240, interval=1.0)
        ws = fe.registry.list()
        assert {w.role for w in ws} == {"prefill", "decode"} and {w.pair for w in ws} == {"pairpod-0"}
        assert len({w.worker_id for w in ws}) == n_workers
        for i in range(2 if form == "group" else 1):
            body = {"model": MODEL, "messages": [{"role": "user", "content": f"pair pod {i} " * 50}],
                    "max_tokens": 12, "temperature": 0, "ignore_eos": True}
            r = httpx.post(fs.url + "/v1/chat/completions", json=body, timeout=120)
            assert r.status_code == 200 and r.json()["usage"]["completion_tokens"] == 12, r.text
        m = httpx.get(f"http://127.0.0.1:{port}/metrics", timeout=10).text
        moved = [ln for ln in m.splitlines()
                 if ln.startswith("dynamo_component_kv_transfer_bytes_total") and 'backend="xgmi"' in ln]
        assert moved and float(moved[0].split()[-1]) > 0, m[-2000:]
    finally:
        proc.terminate()
        try:
            proc.wait(timeout=60)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
        fs.stop()
        log.close()
