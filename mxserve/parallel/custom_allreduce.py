"""Custom IPC all-reduce for tensor-parallel decode.

Kernels: csrc/kernels/custom_allreduce.hip.  One-shot (push the whole input into every peer's
receive slot over the xGMI mesh, flag, sum locally) for small messages; two-shot (reduce-scatter
by push, all-gather by push: each link carries 2/N of the message, one more flag round trip) from
`two_shot_min_bytes` up when there are more than 2 ranks (MXS_CAR_TWO_SHOT_MIN_BYTES, default
512 KiB: 70B TP8 decode at batch >= 32).  This module owns the buffers: each rank allocates uncached receive slots
(2 parities x N ranks x max_bytes) and a 64 KiB signal page, exports both with hipIpc, exchanges
the handles over the CPU group and maps every peer's.  All sizes stay far below 2 GiB (the
dmabuf IPC size rule in mxserve/disagg/kv_transfer.py).

Used for bf16 tensors up to `max_bytes` (decode-sized: 70B TP8 at batch 256 is 4 MiB); larger
all-reduces go to RCCL.  Graph-safe: the per-call epoch lives on the device.  A rank whose peer
never arrives gives up after ~2 s and raises the error word; `check()` (called by the engine between
steps) then turns the path off for good and every later all-reduce uses RCCL.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

SIGNAL_BYTES = 64 << 10
_FLAGS_OFF, _EPOCHS_OFF, _ERR_OFF = 0, 4096, 8192


def _ipc_stalled(err) -> bool:
    """A timed-out open still holds the native IPC table's lock: touch nothing IPC after it."""
    return isinstance(err, TimeoutError)


class CustomAllReduce:
    def __init__(self, rank: int, world: int, max_bytes: int, recv_ptrs: list, flag_ptrs: list, own: tuple,
                 device: torch.device):
        self.rank, self.world = rank, world
        self.max_bytes = max_bytes
        self.slot_elems = max_bytes // 2
        self.recv_ptrs, self.flag_ptrs = recv_ptrs, flag_ptrs
        self._own = own  # (recv_ptr, signal_ptr) allocated by this rank
        sig = flag_ptrs[rank]
        self.epochs_ptr = sig + _EPOCHS_OFF
        self.err_ptr = sig + _ERR_OFF
        self.device = device
        self.disabled = False
        self.two_shot_min_bytes = int(os.environ.get("MXS_CAR_TWO_SHOT_MIN_BYTES", str(512 << 10)))

    @classmethod
    def create(cls, group, device: Optional[torch.device] = None, max_bytes: int = 8 << 20,
               cpu_group=None) -> "CustomAllReduce":
        from .. import ops
        ext = ops.ext()
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        if world > 8:
            raise ValueError("custom all-reduce supports up to 8 ranks (one xGMI mesh)")
        recv_ptr, recv_h = ext.car_alloc(2 * world * max_bytes)
        sig_ptr, sig_h = ext.car_alloc(SIGNAL_BYTES)
        handles = [None] * world
        dist.all_gather_object(handles, (recv_h, sig_h), group=cpu_group or group)
        recv_ptrs, flag_ptrs = [], []
        err = None
        try:  # each open has a deadline (ops.ipc_open): a hung peer mapping fails this rank, not the job
            for r, (rh, sh) in enumerate(handles):
                if r == rank:
                    recv_ptrs.append(recv_ptr)
                    flag_ptrs.append(sig_ptr)
                else:
                    recv_ptrs.append(ops.ipc_open(rh, 0))
                    flag_ptrs.append(ops.ipc_open(sh, 0))
        except (RuntimeError, OSError) as e:
            err = e
        # every rank agrees: one rank that could not map its peers turns the custom path off for all
        ok = torch.tensor([0 if err else 1], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=cpu_group or group)
        if not int(ok.item()):
            if not _ipc_stalled(err):
                for r, (rh, sh) in enumerate(handles):
                    if r != rank and r < len(recv_ptrs):
                        ext.ipc_close(rh)
                    if r != rank and r < len(flag_ptrs):
                        ext.ipc_close(sh)
                ext.car_free(recv_ptr)
                ext.car_free(sig_ptr)
            raise RuntimeError(f"custom all-reduce: peer mapping failed on some rank ({err!r} here)")
        log.info("custom all-reduce ready: rank %d/%d, %d MiB slots", rank, world, max_bytes >> 20)
        return cls(rank, world, max_bytes, recv_ptrs, flag_ptrs, (recv_ptr, sig_ptr), device)

    def should_use(self, x: torch.Tensor) -> bool:
        return (not self.disabled and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % 8 == 0 and x.numel() * 2 <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Sum of x over the group (in place unless `out` is given)."""
        from .. import ops
        out = x if out is None else out
        two_shot = self.world > 2 and x.numel() * 2 >= self.two_shot_min_bytes
        ops.ext().custom_allreduce(out, x, self.recv_ptrs, self.flag_ptrs, self.rank, self.slot_elems,
                                   self.epochs_ptr, self.err_ptr, two_shot)
        return out

    def can_add_rms_norm(self, residual: torch.Tensor) -> bool:
        return (not self.disabled and residual.is_cuda and residual.dtype == torch.bfloat16 and residual.dim() == 2
                and residual.shape[1] % 8 == 0 and residual.shape[1] <= 16384
                and residual.numel() * 2 <= self.max_bytes)

    def add_rms_norm(self, residual: torch.Tensor, w: torch.Tensor, eps: float, x: Optional[torch.Tensor] = None,
                     part: Optional[torch.Tensor] = None) -> tuple:
        """(RMSNorm(residual + AllReduce(partial)) * w, residual updated in place) in one kernel
        (custom_allreduce.hip car_add_rmsnorm_kernel).  The partial is x (bf16, residual's shape) or
        part (fp32 split-K slabs [S, M, H] of the projection, summed and rounded here)."""
        from .. import ops
        h = torch.empty_like(residual)
        two_shot = self.world > 2 and residual.numel() * 2 >= self.two_shot_min_bytes
        ops.ext().car_add_rms_norm(h, residual, x, part, w, eps, self.recv_ptrs, self.flag_ptrs, self.rank,
                                   self.slot_elems, self.epochs_ptr, self.err_ptr, two_shot)
        return h, residual

    def can_all_to_all(self, x: torch.Tensor) -> bool:
        nbytes = x.numel() * x.element_size()
        return (not self.disabled and x.is_cuda and x.is_contiguous() and nbytes % self.world == 0
                and (nbytes // self.world) % 4 == 0 and nbytes // self.world <= self.max_bytes)

    def all_to_all(self, out: torch.Tensor, x: torch.Tensor, push_rows: Optional[torch.Tensor] = None,
                   row_bytes: int = 0) -> torch.Tensor:
        """Equal-split all-to-all (segment d of x -> rank d; segment r of out <- rank r) by direct
        peer pushes into the IPC slots (EP dispatch / combine, graph-capturable).  With push_rows
        (int32 [world] on the device) only the first push_rows[d] rows of segment d cross the link:
        the rest of each segment is capacity (its content in `out` is unspecified)."""
        from .. import ops
        ops.ext().ipc_all_to_all(out, x, self.recv_ptrs, self.flag_ptrs, self.rank, self.max_bytes,
                                 self.epochs_ptr, self.err_ptr, push_rows, row_bytes)
        return out

    def check(self) -> bool:
        """True while healthy.  Reads every rank's error word (all signal pages are mapped here); a
        timed-out peer disables the path (RCCL from then on)."""
        if self.disabled:
            return False
        from .. import ops
        if any(ops.ext().car_read_u32(p + _ERR_OFF) != 0 for p in self.flag_ptrs):
            log.error("custom all-reduce: a peer timed out; falling back to RCCL")
            self.disabled = True
        return not self.disabled
