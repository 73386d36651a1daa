"""Process-group state for tensor / expert parallelism.

One process per GPU: ranks of a TP group live in the same worker pod and talk
over `torch.distributed` - backend "nccl" is RCCL on ROCm, riding xGMI between MI355X GPUs.  Small
decode all-reduces can go through the custom IPC all-reduce (`custom_allreduce.py`) which reads
all 7 peers' buffers concurrently instead of walking a ring one link at a time.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    tp_rank: int = 0
    tp_size: int = 1
    group: Optional[object] = None
    custom_ar: Optional[object] = None  # CustomAllReduce when enabled
    cpu_group: Optional[object] = None  # gloo group for host-side metadata

    @property
    def is_first(self) -> bool:
        return self.tp_rank == 0


_STATE = ParallelState()


def get_tp() -> ParallelState:
    return _STATE


def set_tp(state: ParallelState) -> None:
    global _STATE
    _STATE = state


def init_distributed(tp_size: int, backend: Optional[str] = None, device: Optional[torch.device] = None,
                     enable_custom_ar: bool = True) -> ParallelState:
    """Initialise the default process group from torchrun-style env (RANK/WORLD_SIZE/MASTER_*).
    The whole world is one TP group (one worker = one TP group)."""
    if tp_size <= 1 and not dist.is_initialized():
        set_tp(ParallelState())
        return _STATE
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl" and device is not None:
            kw["device_id"] = device
        dist.init_process_group(backend=backend, **kw)
    world = dist.get_world_size()
    if world != tp_size:
        raise ValueError(f"world size {world} != tp_size {tp_size}")
    st = ParallelState(tp_rank=dist.get_rank(), tp_size=world, group=dist.group.WORLD)
    # scheduler metadata goes rank0 -> TP ranks over a CPU (gloo) group, never a GPU collective
    st.cpu_group = dist.new_group(backend="gloo") if backend != "gloo" else st.group
    # custom IPC all-reduce: validated between processes sharing one GPU (tests/test_custom_ar_gpu.py,
    # tests/test_tp_gpu.py, where the ranks' group is gloo); opt-in until it has run across a real
    # xGMI mesh
    on_gpu = backend == "nccl" or (device is not None and torch.device(device).type == "cuda")
    if enable_custom_ar and on_gpu and os.environ.get("MXS_CUSTOM_AR", "0") == "1":
        try:
            from .custom_allreduce import CustomAllReduce
            st.custom_ar = CustomAllReduce.create(st.group, device, cpu_group=st.cpu_group)
        except Exception as e:  # noqa: BLE001 - RCCL remains correct
            import logging
            logging.getLogger(__name__).warning("custom all-reduce disabled: %r", e)
    set_tp(st)
    return st


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    st = _STATE
    if st.tp_size == 1:
        return x
    if st.custom_ar is not None and st.custom_ar.should_use(x):
        return st.custom_ar.all_reduce(x)
    dist.all_reduce(x, group=st.group)
    return x


def tp_all_gather(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    st = _STATE
    if st.tp_size == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(st.tp_size)]
    dist.all_gather(parts, x.contiguous(), group=st.group)
    return torch.cat(parts, dim=dim)


def tp_broadcast_object(obj, src: int = 0):
    st = _STATE
    if st.tp_size == 1:
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src=src, group=st.cpu_group or st.group)
    return box[0]
