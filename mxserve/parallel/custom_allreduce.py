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
all-reduces go to RCCL.  Graph-safe: the per-call epoch lives on the device.

Failure handling (round-4 driver failure: GPUTEST_r04.json, profiles/r5/car_timeout/README.md):
  * every wait is bounded by WALL-CLOCK time (MXS_CAR_TIMEOUT_MS, default 10 s, on the device's
    constant 100 MHz counter) instead of a spin count, and a rank that gives up writes a record
    (which kernel / phase, block, which peer's flag it missed, the epoch it expected and the value
    it saw, device timestamps) and raises the error word of every rank;
  * the first collective after creation (or after a reset) is preceded by a device synchronize and
    a CPU-group barrier, so ranks whose start-up work (weight init, graph warm-up) is still queued on
    the GPU do not spend the wait budget on each other's start-up skew;
  * the engine polls every rank's error word at the end of each TP step (`poll_into`, on the step's
    stream, no host sync); a faulted step and the one in flight behind it are discarded and
    recomputed (engine.py), then `reset()` re-arms the path on every rank.  After
    MXS_CAR_MAX_FAULTS faults the path is turned off and decode graphs are re-captured on RCCL.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

SIGNAL_BYTES = 64 << 10
# byte offsets in a rank's signal page (csrc/kernels/custom_allreduce.hip kSig*)
_FLAGS_OFF, _EPOCHS_OFF, _ERR_OFF, _DIAG_OFF, _FIRST_OFF = 0, 4096, 8192, 12288, 12416
_CLEAR_BYTES = 16 << 10  # flags, epochs, error word and records
_KINDS = {1: "one-shot", 2: "two-shot/reduce-scatter", 3: "two-shot/all-gather", 4: "add-rmsnorm/one-shot",
          5: "add-rmsnorm/two-shot reduce-scatter", 6: "add-rmsnorm/two-shot all-gather", 7: "all-to-all"}


def timeout_ms() -> float:
    return float(os.environ.get("MXS_CAR_TIMEOUT_MS", "10000"))


class CollectiveFault(RuntimeError):
    """A TP step whose custom collective gave up on some rank: its results are not to be used."""

    def __init__(self, words: list):
        super().__init__(f"custom all-reduce fault (error words {words})")
        self.words = words


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
        from .. import ops
        self.tick_khz = int(ops.ext().car_wall_clock_khz())
        self.timeout_ticks = max(1, int(timeout_ms() * self.tick_khz))
        self.cpu_group = None
        self.faults = 0  # faults seen (and recovered from) by this process
        self.armed = False  # False until the first collective's synchronize + barrier
        self.first_host_time: Optional[float] = None

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
        car = cls(rank, world, max_bytes, recv_ptrs, flag_ptrs, (recv_ptr, sig_ptr), device)
        car.cpu_group = cpu_group or group
        return car

    def _arm(self) -> None:
        """Before the first collective (and the first after a reset): drain this rank's queued GPU
        work and meet every rank on the CPU group, so the device wait budget covers only the
        collective itself, never start-up skew (weights still initialising on one rank's queue)."""
        import time
        # MXS_CAR_ARM=0 (diagnosis only: mxserve/tools/car_skew_probe.py) measures the skew the
        # barrier removes
        if os.environ.get("MXS_CAR_ARM", "1") != "0":
            if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
                torch.cuda.synchronize()
            dist.barrier(group=self.cpu_group)
        self.first_host_time = time.time()
        self.armed = True
        log.info("custom all-reduce: rank %d armed at host time %.6f", self.rank, self.first_host_time)

    def should_use(self, x: torch.Tensor) -> bool:
        return (not self.disabled and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % 8 == 0 and x.numel() * 2 <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Sum of x over the group (in place unless `out` is given)."""
        from .. import ops
        if not self.armed:
            self._arm()
        out = x if out is None else out
        two_shot = self.world > 2 and x.numel() * 2 >= self.two_shot_min_bytes
        ops.ext().custom_allreduce(out, x, self.recv_ptrs, self.flag_ptrs, self.rank, self.slot_elems,
                                   self.epochs_ptr, self.timeout_ticks, two_shot)
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
        if not self.armed:
            self._arm()
        h = torch.empty_like(residual)
        two_shot = self.world > 2 and residual.numel() * 2 >= self.two_shot_min_bytes
        ops.ext().car_add_rms_norm(h, residual, x, part, w, eps, self.recv_ptrs, self.flag_ptrs, self.rank,
                                   self.slot_elems, self.epochs_ptr, self.timeout_ticks, two_shot)
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
        if not self.armed:
            self._arm()
        ops.ext().ipc_all_to_all(out, x, self.recv_ptrs, self.flag_ptrs, self.rank, self.max_bytes,
                                 self.epochs_ptr, self.timeout_ticks, push_rows, row_bytes)
        return out

    # ------------------------------------------------------------------ health
    def poll_into(self, out: torch.Tensor) -> None:
        """Enqueue a copy of every rank's error word into `out` (pinned int32 [>= world]) on the
        current stream: read it on the host once the step's completion event has fired."""
        from .. import ops
        ops.ext().car_poll_err(out, self.recv_ptrs, self.flag_ptrs)

    def error_words(self) -> list:
        """Every rank's error word, read synchronously (0 = healthy, else 1 + the rank that gave up)."""
        from .. import ops
        return [int(ops.ext().car_read_words(p + _ERR_OFF, 1)[0]) for p in self.flag_ptrs]

    def diagnose(self) -> list:
        """Per rank: its error word, its give-up record (if it gave up) and the device time of its
        first collective since the last reset (ranks sharing one GPU share the clock: their arrival
        skew is exact; on separate GPUs compare records only within a rank)."""
        from .. import ops
        ext = ops.ext()
        out = []
        for r, p in enumerate(self.flag_ptrs):
            err = int(ext.car_read_words(p + _ERR_OFF, 1)[0])
            d = ext.car_read_words(p + _DIAG_OFF, 16)
            first = ext.car_read_words(p + _FIRST_OFF, 2)
            ent = {"rank": r, "err": err, "first_collective_tick": first[0] | (first[1] << 32)}
            if d[0]:
                t0, t1 = d[8] | (d[9] << 32), d[10] | (d[11] << 32)
                ent["gave_up"] = {"kernel": _KINDS.get(d[1], str(d[1])), "epoch": d[2], "flag_seen": d[3],
                                  "block": d[4], "missing_peer": d[5], "waited_ms": (t1 - t0) / self.tick_khz,
                                  "wait_start_tick": t0, "give_up_tick": t1}
            out.append(ent)
        firsts = [e["first_collective_tick"] for e in out if e["first_collective_tick"]]
        if firsts:
            for e in out:
                if e["first_collective_tick"]:
                    e["first_collective_skew_ms"] = (e["first_collective_tick"] - min(firsts)) / self.tick_khz
        return out

    def check(self) -> bool:
        """True while no rank has given up (a synchronous read of every rank's error word; tests and
        fault handling -- the engine polls asynchronously with poll_into).  Logs the diagnosis."""
        if self.disabled:
            return False
        if any(self.error_words()):
            log.error("custom all-reduce fault: %s", self.diagnose())
            return False
        return True

    def reset(self) -> None:
        """Re-arm after a fault.  Collective: call on every rank once each has quiesced (the engine
        does it from _reset_collectives with CPU-group barriers on both sides): zero this rank's
        flags, epochs, error word and records, so every rank restarts at epoch 1."""
        from .. import ops
        ops.ext().car_clear(self._own[1], _CLEAR_BYTES)
        self.armed = False
