"""Tensor-parallel worker groups: one process per GPU.

The worker's main process is TP rank 0: it runs the scheduler, the HTTP server and its shard of the
model; `start_tp_group` spawns ranks 1..N-1 as child processes (`python -m mxserve.worker.tp`) that
join the same torch.distributed group (RCCL over xGMI for the collectives inside the model, gloo
for the per-step host metadata broadcast) and mirror every step (ModelRunner.follower_loop).
"""
from __future__ import annotations

import dataclasses
import json
import logging
import os
import socket
import subprocess
import sys

log = logging.getLogger(__name__)
_children: list = []


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def start_tp_group(args, device_ids=None) -> None:
    """Called in the rank-0 process before the engine is built."""
    import torch

    from ..parallel.comm import init_distributed
    n = args.tensor_parallel_size
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    os.environ["WORLD_SIZE"] = str(n)
    os.environ["RANK"] = "0"
    os.environ.setdefault("LOCAL_RANK", "0")
    payload = json.dumps(dataclasses.asdict(args))
    for r in range(1, n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), MXS_TP_ARGS=payload)
        _children.append(subprocess.Popen([sys.executable, "-m", "mxserve.worker.tp"], env=env))
    use_gpu = args.resolved_device() == "cuda"
    dev = None
    if use_gpu:  # GPUs [offset, offset + n): offset > 0 for the prefill half of a P/D pair pod
        off = int(os.environ.get("MXS_DEVICE_OFFSET", "0"))
        torch.cuda.set_device(off)
        dev = torch.device("cuda", off)
    init_distributed(n, backend=_backend(use_gpu, n), device=dev)
    log.info("TP group of %d ranks up", n)


def _backend(use_gpu: bool, n: int) -> str:
    """RCCL when every rank has its own GPU.  Ranks that must share a device (a functional run on a
    box with fewer GPUs than ranks; RCCL refuses duplicate devices) use gloo, with the custom IPC
    all-reduce carrying the model's collectives."""
    import torch
    if not use_gpu:
        return "gloo"
    return "nccl" if torch.cuda.device_count() >= n + int(os.environ.get("MXS_DEVICE_OFFSET", "0")) else "gloo"


def stop_tp_group() -> None:
    for p in _children:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()


def follower_main() -> None:
    import torch

    from ..config import EngineArgs
    from ..engine.model_runner import ModelRunner
    from ..models.config import get_model_config
    from ..parallel.comm import init_distributed
    from ..utils.logs import setup_logging
    setup_logging()
    args = EngineArgs(**json.loads(os.environ["MXS_TP_ARGS"]))
    rank = int(os.environ["RANK"])
    use_gpu = args.resolved_device() == "cuda"
    dev = None
    if use_gpu:
        off = int(os.environ.get("MXS_DEVICE_OFFSET", "0"))
        torch.cuda.set_device((off + int(os.environ.get("LOCAL_RANK", rank))) % torch.cuda.device_count())
        dev = torch.device("cuda", torch.cuda.current_device())
    init_distributed(args.tensor_parallel_size, backend=_backend(use_gpu, args.tensor_parallel_size), device=dev)
    runner = ModelRunner(args, get_model_config(args.model))
    runner.follower_loop()


if __name__ == "__main__":
    follower_main()
