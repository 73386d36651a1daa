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
    meta_ring: Optional[object] = None  # MetaRing: per-step metadata over /dev/shm

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
                     enable_custom_ar: bool = True, timeout_s: Optional[float] = None) -> ParallelState:
    """Initialise the default process group from torchrun-style env (RANK/WORLD_SIZE/MASTER_*).
    The whole world is one TP group (one worker = one TP group).  timeout_s bounds a collective that
    some rank never joins (gloo raises after it; default: torch's 30 min)."""
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
        if timeout_s:
            from datetime import timedelta
            kw["timeout"] = timedelta(seconds=timeout_s)
        dist.init_process_group(backend=backend, **kw)
    world = dist.get_world_size()
    if world != tp_size:
        raise ValueError(f"world size {world} != tp_size {tp_size}")
    st = ParallelState(tp_rank=dist.get_rank(), tp_size=world, group=dist.group.WORLD)
    # scheduler metadata goes rank0 -> TP ranks over a CPU (gloo) group, never a GPU collective
    if backend != "gloo":
        from datetime import timedelta
        st.cpu_group = dist.new_group(backend="gloo", **({"timeout": timedelta(seconds=timeout_s)} if timeout_s else {}))
    else:
        st.cpu_group = st.group
    # custom IPC all-reduce (one-shot / two-shot over peer-mapped buffers, bounded spins, RCCL
    # fallback on a peer timeout): on by default for TP <= 8 (its rank limit); validated with 2-8
    # ranks sharing one GPU (tests/test_custom_ar_gpu.py, tests/test_b_tp_gpu.py); MXS_CUSTOM_AR=0
    # keeps every all-reduce on RCCL
    on_gpu = backend == "nccl" or (device is not None and torch.device(device).type == "cuda")
    if enable_custom_ar and on_gpu and os.environ.get("MXS_CUSTOM_AR", "1" if world <= 8 else "0") == "1":
        try:
            from .custom_allreduce import CustomAllReduce
            st.custom_ar = CustomAllReduce.create(st.group, device, cpu_group=st.cpu_group)
        except Exception as e:  # noqa: BLE001 - RCCL remains correct
            import logging
            logging.getLogger(__name__).warning("custom all-reduce disabled: %r", e)
    set_tp(st)
    return st


_LOCAL = [False]


class collectives_local:
    """Context manager: every TP collective of this process becomes a local stand-in (all-reduce ->
    this rank's partial, all-gather -> its shard tiled).  A dense model's forward then runs every
    kernel and library GEMM of the real one without waiting for a peer: a local warm-up pays the
    first-call costs (hipBLASLt solution and code-object loads from a cold page cache took one rank
    seconds longer than its peers, profiles/r5/car_timeout/README.md) at each rank's own pace, before
    the collective warm-up.  Numbers computed inside are meaningless."""

    def __enter__(self):
        _LOCAL[0] = True
        return self

    def __exit__(self, *exc):
        _LOCAL[0] = False
        return False


def tp_barrier() -> None:
    """CPU-group barrier of the TP group (no-op at TP 1)."""
    st = _STATE
    if st.tp_size > 1:
        dist.barrier(group=st.cpu_group or st.group)


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    st = _STATE
    if st.tp_size == 1 or _LOCAL[0]:
        return x
    if st.custom_ar is not None and st.custom_ar.should_use(x):
        return st.custom_ar.all_reduce(x)
    dist.all_reduce(x, group=st.group)
    return x


def tp_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float) -> tuple:
    """(RMSNorm(residual + AllReduce(x)) * w, new residual) for a TP-partial projection output x that
    feeds the residual stream.  With the custom all-reduce: one kernel (exchange + add + norm); else
    the all-reduce and then the fused add + RMSNorm kernel.  TP = 1: just the add + norm."""
    from .. import ops
    st = _STATE
    if st.tp_size > 1 and not _LOCAL[0]:
        car = st.custom_ar
        if car is not None and x.is_contiguous() and x.dtype == residual.dtype and car.can_add_rms_norm(residual):
            return car.add_rms_norm(residual, w, eps, x=x)
        x = tp_all_reduce(x)
    return ops.fused_add_rms_norm(x, residual, w, eps)


def tp_linear_add_rms_norm(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor,
                           eps: float) -> tuple:
    """The projection x @ w.T (o_proj / down_proj, row-parallel: a TP-partial sum) + all-reduce +
    residual add + RMSNorm.  TP = 1: ops.linear_add_rms_norm.  TP > 1 with the custom all-reduce:
    when the decode table runs the shard split-K, its fp32 slabs go straight into the fused
    all-reduce kernel (no split-K reduce kernel, no bf16 partial); otherwise the bf16 partial does."""
    from .. import ops
    st = _STATE
    if st.tp_size == 1:
        return ops.linear_add_rms_norm(x, w, residual, norm_w, eps)
    if _LOCAL[0]:
        return ops.fused_add_rms_norm(ops.linear(x, w), residual, norm_w, eps)
    car = st.custom_ar
    if car is not None and car.can_add_rms_norm(residual) and x.is_cuda and x.dim() == 2 \
            and 0 < x.shape[0] <= ops._decode_max_m():
        from ..ops.decode_gemm import TABLE
        M, N = x.shape[0], w.shape[0]
        cfg = TABLE.lookup(M, N, w.shape[1], 0)
        if cfg is not None and TABLE.splitk(cfg) > 1:
            S = TABLE.splitk(cfg)
            if TABLE.run(residual, x, w, cfg, 0, reduce=False):  # no output written: reduce skipped
                return car.add_rms_norm(residual, norm_w, eps, part=TABLE.part[:S * M * N])
    return tp_add_rms_norm(ops.linear(x, w), residual, norm_w, eps)


def tp_all_gather(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    st = _STATE
    if st.tp_size == 1:
        return x
    if _LOCAL[0]:
        return torch.cat([x] * st.tp_size, dim=dim)
    car = st.custom_ar
    if car is not None and x.is_cuda and dim in (0, -1, x.dim() - 1):
        # every rank pushes its shard to every peer through the IPC all-to-all (one xGMI hop per
        # link, graph-capturable whatever the process group's backend)
        rep = x.contiguous().unsqueeze(0).expand(st.tp_size, *x.shape).contiguous()
        if car.can_all_to_all(rep):
            out = torch.empty_like(rep)
            car.all_to_all(out, rep)  # out[r] = rank r's shard
            if dim == 0:
                return out.reshape(st.tp_size * x.shape[0], *x.shape[1:])
            return out.movedim(0, -2).reshape(*x.shape[:-1], st.tp_size * x.shape[-1])
    parts = [torch.empty_like(x) for _ in range(st.tp_size)]
    dist.all_gather(parts, x.contiguous(), group=st.group)
    return torch.cat(parts, dim=dim)


class MetaRing:
    """Per-step scheduler metadata rank 0 -> TP ranks through the native /dev/shm ring
    (csrc/runtime/shm_ring.cpp) instead of a pickled gloo broadcast per step.
    A message larger than a slot, or a node without usable /dev/shm, goes over gloo."""

    _GLOO = b"\x00mxs-gloo"

    def __init__(self, ring, rank: int):
        self.ring, self.rank = ring, rank
        self.steps = 0
        self.gloo_fallbacks = 0

    def send(self, obj) -> None:
        import pickle
        data = pickle.dumps(obj, protocol=5)
        self.steps += 1
        if len(data) > self.ring.slot_bytes:
            self.gloo_fallbacks += 1
            self._push(self._GLOO)
            _gloo_broadcast(obj)
            return
        self._push(data)

    # a follower that has not taken a step for this long is dead or wedged: fail the driver's engine
    # (the worker exits non-zero and gets restarted) instead of serving nothing while looking alive
    PUSH_TIMEOUT_S = float(os.environ.get("MXS_TP_META_TIMEOUT_S", "120"))

    def _push(self, data: bytes) -> None:
        import logging
        waited = 0.0
        while not self.ring.push(data, 10.0):  # a follower is still busy with an old step
            waited += 10.0
            if waited >= self.PUSH_TIMEOUT_S:
                raise RuntimeError(f"TP metadata ring full for {waited:.0f}s: a follower rank stopped reading")
            logging.getLogger(__name__).warning("TP metadata ring full for %.0f s; waiting for followers", waited)

    def recv(self):
        import pickle
        ppid = os.getppid()
        while True:
            data = self.ring.pop(self.rank - 1, 1.0)
            if data is not None:
                break
            if os.getppid() != ppid:  # the driver rank (our parent) is gone
                return ("shutdown", None, None)
        self.steps += 1
        if data == self._GLOO:
            return _gloo_broadcast(None)
        return pickle.loads(data)


def setup_meta_ring(slot_bytes: int, nslots: int = 2) -> Optional[MetaRing]:
    """Collective over the TP group's CPU group: rank 0 creates the ring, every rank attaches, then
    the name is unlinked (nothing stays in /dev/shm whatever happens to the processes later)."""
    st = _STATE
    if st.tp_size == 1 or os.environ.get("MXS_TP_META_RING", "1") != "1":
        return None
    from .. import _native
    rt = _native.rt()
    name = None
    ring = None
    if st.tp_rank == 0:
        name = f"/mxs-tp-{os.getpid()}-{int.from_bytes(os.urandom(4), 'little'):08x}"
        try:
            ring = rt.ShmRing(name, True, int(slot_bytes), int(nslots), st.tp_size - 1)
        except Exception as e:  # noqa: BLE001 - no /dev/shm (or too small): stay on gloo
            import logging
            logging.getLogger(__name__).warning("TP metadata ring unavailable (%r); using gloo", e)
            name = None
    name = _gloo_broadcast(name)
    ok = 1
    if name is not None and st.tp_rank > 0:
        try:
            ring = rt.ShmRing(name, False)
        except Exception:  # noqa: BLE001
            ok = 0
    t = torch.tensor([ok], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=st.cpu_group or st.group)
    if st.tp_rank == 0 and ring is not None:
        ring.unlink()
    if name is None or not int(t.item()):
        st.meta_ring = None
        return None
    st.meta_ring = MetaRing(ring, st.tp_rank)
    return st.meta_ring


def _gloo_broadcast(obj, src: int = 0):
    st = _STATE
    box = [obj]
    dist.broadcast_object_list(box, src=src, group=st.cpu_group or st.group)
    return box[0]


def collectives_capturable(max_message_bytes: int) -> bool:
    """Can a hipGraph capture this group's collectives for messages up to max_message_bytes?  RCCL
    is capturable; a gloo group (ranks sharing a GPU in functional runs) only through the custom
    IPC kernels, within their slot size."""
    st = _STATE
    if st.tp_size == 1:
        return True
    if dist.get_backend(st.group) == "nccl":
        return True
    car = st.custom_ar
    return car is not None and not car.disabled and max_message_bytes <= car.max_bytes


def tp_broadcast_object(obj, src: int = 0):
    st = _STATE
    if st.tp_size == 1:
        return obj
    if st.meta_ring is not None and src == 0:
        if st.tp_rank == 0:
            st.meta_ring.send(obj)
            return obj
        return st.meta_ring.recv()
    return _gloo_broadcast(obj, src)
