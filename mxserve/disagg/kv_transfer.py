"""KV transfer agent for disaggregated prefill -> decode (replaces NIXL).

Backends
  xgmi  the decode worker owns a STAGING ARENA of KV blocks (4 GiB by default: 8,192 Llama-3.2-1B
        blocks, i.e. 32 concurrent 4k-token prompts) allocated once and exported with
        hipIpcGetMemHandle; the prefill worker maps it once (hipIpcOpenMemHandle, lazy peer
        access).  Per request:
          decode   reserve a contiguous extent of the arena, send its offset with the request;
          prefill  ONE copy kernel writes the request's blocks into that extent -- the stores travel
                   over xGMI into the decode GPU's HBM (or stay on-chip when both share a GPU);
          decode   ONE copy kernel on its compute stream scatters extent -> the reserved pool blocks
                   (ordered before the next step); the extent is recycled once that copy is done.
        Why an arena and not the pool itself: on this ROCm 7.2 / dmabuf-IPC stack hipIpcOpenMemHandle
        never returns for an allocation whose size mod 4 GiB lies in [2 GiB, 4 GiB) (measured with
        scripts/ipc_probe.py: 0.5, 1, 1.5, 4, 4.5, 8, 12, 16 GiB map in ~2 ms; 2, 2.5, 3, 6 and a
        19.5 GiB serving pool hang), so the exported allocation is a fixed, IPC-safe size rather
        than whatever the pool happens to be; the extra on-GPU scatter costs ~30-60 us per
        4000-token prompt.
  shm   the decode worker also owns a HOST staging arena in /dev/shm (MXS_KV_SHM_BYTES, 2 GiB by
        default), page-locked with hipHostRegister.  A prefill worker that shares the host's
        /dev/shm (the P/D pair pod the operator renders, or the same node with hostIPC) but cannot
        map the GPU arena copies the request's blocks D2H into an extent of it; the decode worker
        copies them H2D into its pool.  Two DMA copies at host-link speed instead of a msgpack body
        over HTTP.
  host  staged through the control plane (no shared /dev/shm either): the prefill side ships the
        block bytes in the HTTP body, the decode side writes them.
The decode side reserves an extent in each arena it has; the prefill side uses the first that works
(xgmi, then shm, then host) and says which; the decode side lands from that one and recycles the
others.  Block layout is identical on both sides ([L, 2, Hkv, 16, D] per block).
"""
from __future__ import annotations

import base64
import logging
import math
import os
import threading
import time
from typing import Optional

import numpy as np
import torch

log = logging.getLogger(__name__)

STAGING_BYTES = int(os.environ.get("MXS_KV_STAGING_BYTES", str(4 << 30)))
SHM_BYTES = int(os.environ.get("MXS_KV_SHM_BYTES", str(2 << 30)))
_GIB = 1 << 30


class Extents:
    """First-fit allocator of contiguous block extents in a staging arena; an extent is recycled
    only once the copy that reads it has finished (an event, or None for immediately)."""

    def __init__(self, n: int):
        self.n = n
        self._free: list[list[int]] = [[0, n]] if n > 0 else []
        self._draining: list[tuple[int, int, object]] = []
        self._lock = threading.Lock()

    def acquire(self, k: int) -> Optional[int]:
        if k <= 0 or k > self.n:
            return None
        with self._lock:
            still = []
            for start, n, ev in self._draining:
                if ev is None or ev.query():
                    self._put(start, n)
                else:
                    still.append((start, n, ev))
            self._draining = still
            for ext in self._free:
                if ext[1] >= k:
                    start = ext[0]
                    ext[0] += k
                    ext[1] -= k
                    if ext[1] == 0:
                        self._free.remove(ext)
                    return start
            return None

    def release(self, start: int, n: int, after=None) -> None:
        with self._lock:
            self._draining.append((start, n, after))

    def _put(self, start: int, n: int) -> None:
        f = self._free
        f.append([start, n])
        f.sort()
        merged = [f[0]]
        for s0, n0 in f[1:]:
            if merged[-1][0] + merged[-1][1] == s0:
                merged[-1][1] += n0
            else:
                merged.append([s0, n0])
        self._free = merged

    def free_blocks(self) -> int:
        with self._lock:
            return sum(n for _, n in self._free) + sum(n for _, n, _ in self._draining)


def _unlink_quiet(path: str) -> None:
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass


class ShmArena:
    """KV blocks in /dev/shm shared by the workers of one pod / host (the `shm` backend)."""

    def __init__(self, name: str, nblocks: int, block_shape: tuple, dtype: torch.dtype, create: bool,
                 pin: bool):
        import mmap
        self.name, self.nblocks = name, nblocks
        esz = torch.empty(0, dtype=dtype).element_size()
        self.block_bytes = int(np.prod(block_shape)) * esz
        nbytes = nblocks * self.block_bytes
        path = "/dev/shm" + name
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(path, flags, 0o600)
        try:
            if create:
                os.ftruncate(fd, nbytes)
            self._mm = mmap.mmap(fd, nbytes, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self.owner = create
        if create:  # a worker that exits without close() still removes its name from /dev/shm
            import atexit
            atexit.register(_unlink_quiet, path)
        arr = np.frombuffer(self._mm, dtype=np.uint8)
        self.t = torch.from_numpy(arr).view(dtype).view(nblocks, *block_shape)
        self._pinned = False
        if pin:  # page-locked for DMA; a pin failure (RLIMIT_MEMLOCK, ...) leaves it pageable
            from .. import ops
            try:
                ops.ext().host_register(int(self.t.data_ptr()), nbytes)
                self._pinned = True
            except RuntimeError as e:
                log.warning("KV shm arena %s not page-locked (%r); copies go through pageable memory", name, e)

    def close(self) -> None:
        if self._pinned:
            from .. import ops
            ops.ext().host_unregister(int(self.t.data_ptr()))
            self._pinned = False
        self.t = None
        if self.owner:
            _unlink_quiet("/dev/shm" + self.name)


def ipc_safe_blocks(k: int, block_bytes: int) -> int:
    """Largest count <= k of block_bytes-sized blocks whose allocation -- rounded up to the caching
    allocator's 2 MiB granule -- keeps (size mod 4 GiB) below 2 GiB (see the module docstring)."""
    lim = 2 * _GIB - (2 << 20)
    r = (k * block_bytes) % (4 * _GIB)
    if r <= lim:
        return k
    base = k * block_bytes - r  # start of this 4 GiB window
    return max(1, (base + lim) // block_bytes)


class KVTransferAgent:
    def __init__(self, runner, backend: str = "xgmi", max_prompt_tokens: Optional[int] = None):
        self.runner = runner
        self.kv = runner.kv_cache
        self.block_bytes = runner.block_bytes
        self.is_gpu = self.kv.is_cuda
        self.backend = backend if (backend == "xgmi" and self.is_gpu) else "host"
        self._stream = torch.cuda.Stream(device=self.kv.device) if self.is_gpu else None
        self._lock = threading.Lock()
        self._opened: dict[str, int] = {}
        self.bytes_moved = 0
        self.transfers = 0
        # staging arena (decode side, allocated lazily by the first descriptor() call): at least one
        # max-length prompt, at most STAGING_BYTES
        bs = getattr(getattr(runner, "args", None), "block_size", 16)
        mtok = max_prompt_tokens or getattr(getattr(runner, "args", None), "max_model_len", 8192)
        bb = max(1, self.block_bytes)
        self.arena_blocks = max(math.ceil(mtok / bs), STAGING_BYTES // bb)
        self.arena_blocks = ipc_safe_blocks(self.arena_blocks, bb)
        self.staging: Optional[torch.Tensor] = None
        self._ext: Optional[Extents] = None
        self._desc: Optional[dict] = None
        # host staging arena in /dev/shm (decode side creates, prefill side attaches by name)
        self.shm: Optional[ShmArena] = None
        self._shm_ext: Optional[Extents] = None
        self._shm_peers: dict[str, ShmArena] = {}
        self.shm_blocks = max(math.ceil(mtok / bs), SHM_BYTES // bb) if SHM_BYTES > 0 else 0

    # -------------------------------------------------------------- decode side
    def _ensure_staging(self) -> None:
        if self.staging is not None or self.backend != "xgmi":
            return
        self.staging = torch.empty((self.arena_blocks,) + tuple(self.kv.shape[1:]), dtype=self.kv.dtype,
                                   device=self.kv.device)
        self._ext = Extents(self.arena_blocks)
        log.info("KV staging arena: %d blocks (%.2f GB)", self.arena_blocks,
                 self.arena_blocks * self.block_bytes / 1e9)

    def _ensure_shm(self) -> None:
        if self.shm is not None or self.shm_blocks <= 0:
            return
        name = f"/mxs-kv-{os.getpid()}-{int.from_bytes(os.urandom(4), 'little'):08x}"
        try:
            self.shm = ShmArena(name, self.shm_blocks, tuple(self.kv.shape[1:]), self.kv.dtype, create=True,
                                pin=self.is_gpu)
        except OSError as e:  # no (big enough) /dev/shm: the host backend remains
            log.warning("no /dev/shm KV staging arena (%r)", e)
            self.shm_blocks = 0
            return
        self._shm_ext = Extents(self.shm_blocks)
        log.info("KV shm staging arena %s: %d blocks (%.2f GB)", name, self.shm_blocks,
                 self.shm_blocks * self.block_bytes / 1e9)

    def descriptor(self, host_url: Optional[str] = None) -> dict:
        if self._desc is not None:
            return dict(self._desc, url=host_url)
        d = {"backend": self.backend, "block_bytes": self.block_bytes, "pid": os.getpid(),
             "num_blocks": int(self.kv.shape[0]), "url": host_url,
             "shape": list(self.kv.shape[1:]), "dtype": str(self.kv.dtype).replace("torch.", "")}
        if self.backend == "xgmi":
            from .. import ops
            self._ensure_staging()
            handle, off = ops.ext().ipc_export_pool(self.staging)
            d.update(handle=base64.b64encode(handle).decode(), offset=int(off), device=self.kv.device.index,
                     data_ptr=int(self.staging.data_ptr()), arena_blocks=self.arena_blocks)
        self._ensure_shm()
        if self.shm is not None:
            d.update(shm_name=self.shm.name, shm_blocks=self.shm_blocks)
        self._desc = d
        return dict(d)

    def acquire(self, n: int) -> Optional[int]:
        """Offset of a free extent of n GPU-arena blocks, or None (xgmi unavailable or full)."""
        if self.backend != "xgmi" or n <= 0:
            return None
        self._ensure_staging()
        return self._ext.acquire(n)

    def release(self, start: int, n: int, after=None) -> None:
        """Recycle a GPU-arena extent; `after` (a recorded event) delays it until the landing copy
        is done."""
        self._ext.release(start, n, after)

    def acquire_shm(self, n: int) -> Optional[int]:
        self._ensure_shm()
        return self._shm_ext.acquire(n) if self._shm_ext is not None else None

    def release_shm(self, start: int, n: int, after=None) -> None:
        self._shm_ext.release(start, n, after)

    def land_shm(self, start: int, dst_ids: list[int]) -> None:
        """Host arena extent -> pool blocks on the current stream (H2D DMA from page-locked shm)."""
        n = len(dst_ids)
        ev = None
        if n:
            src = self.shm.t[start:start + n]
            idx = torch.tensor(dst_ids, dtype=torch.long)
            if self.is_gpu:
                self.kv.index_copy_(0, idx.to(self.kv.device, non_blocking=True),
                                    src.to(self.kv.device, non_blocking=True))
                ev = torch.cuda.Event()
                ev.record()
            else:
                self.kv.index_copy_(0, idx, src)
        self.release_shm(start, n, ev)

    def land(self, start: int, dst_ids: list[int]) -> None:
        """Scatter a filled extent into the pool blocks on the CURRENT stream (call it on the engine's
        stream so the copy is ordered before the step that reads the blocks), then recycle it."""
        from .. import ops
        n = len(dst_ids)
        if n:
            s = torch.arange(start, start + n, dtype=torch.int32).pin_memory().to(self.kv.device, non_blocking=True)
            d = torch.tensor(dst_ids, dtype=torch.int32).pin_memory().to(self.kv.device, non_blocking=True)
            ops.ext().copy_blocks(int(self.kv.data_ptr()), self.staging, s, d, self.block_bytes)
        ev = torch.cuda.Event()
        ev.record()
        self.release(start, n, ev)

    def write_blocks(self, dst_ids: list[int], payload: bytes) -> None:
        """Host backend, decode side: place shipped blocks into the pool."""
        n = len(dst_ids)
        arr = np.frombuffer(payload, dtype=np.uint8).copy()
        src = torch.from_numpy(arr).view(self.kv.dtype).view(n, *self.kv.shape[1:])
        idx = torch.tensor(dst_ids, dtype=torch.long, device=self.kv.device)
        self.kv.index_copy_(0, idx, src.to(self.kv.device))
        if self.is_gpu:
            torch.cuda.synchronize(self.kv.device)

    def close(self) -> None:
        """Unmap every opened peer arena and drop the local ones (bench phases rebuild engines)."""
        if self._stream is not None:
            self._stream.synchronize()
        if self._opened:  # only this agent's mappings: the custom all-reduce's peer slots stay mapped
            from .. import ops
            for key in self._opened:
                ops.ext().ipc_close(base64.b64decode(key))
            self._opened.clear()
        for a in list(self._shm_peers.values()) + ([self.shm] if self.shm is not None else []):
            a.close()
        self._shm_peers.clear()
        self.shm = None
        self.staging = None
        self._desc = None

    def _shm_peer(self, target: dict) -> ShmArena:
        name = target["shm_name"]
        with self._lock:
            arena = self._shm_peers.get(name)
            if arena is None:
                arena = ShmArena(name, int(target["shm_blocks"]), tuple(self.kv.shape[1:]), self.kv.dtype,
                                 create=False, pin=self.is_gpu)
                self._shm_peers[name] = arena
        if arena.block_bytes != self.block_bytes:
            raise ValueError("KV block layout mismatch between prefill and decode workers")
        return arena

    def push_shm(self, src_ids: list[int], target: dict, start: int) -> float:
        """Prefill side: copy blocks into the decode worker's /dev/shm arena (same pod / host);
        blocking, returns seconds.  Raises OSError when that arena is not visible here."""
        t0 = time.perf_counter()
        ev = self.push_async([(src_ids, target, start, "shm")])
        if ev is not None:
            ev.synchronize()
        return time.perf_counter() - t0

    # -------------------------------------------------------------- prefill side
    def _remote_ptr(self, target: dict) -> int:
        if target.get("pid") == os.getpid():  # same process: plain device pointer
            return int(target["data_ptr"])
        key = target["handle"]
        with self._lock:
            ptr = self._opened.get(key)
            if ptr is None:
                from .. import ops
                ptr = ops.ipc_open(base64.b64decode(key), int(target["offset"]))  # deadline: TimeoutError
                self._opened[key] = ptr
            return ptr

    def connect(self, target: dict) -> None:
        """Map the target's staging slots ahead of the first transfer."""
        if target.get("backend") == "xgmi" and self.backend == "xgmi":
            self._remote_ptr(target)

    def read_blocks(self, src_ids: list[int]) -> bytes:
        idx = torch.tensor(src_ids, dtype=torch.long, device=self.kv.device)
        blk = self.kv.index_select(0, idx)
        return blk.cpu().contiguous().view(torch.uint8).numpy().tobytes()

    def push_xgmi(self, src_ids: list[int], target: dict, start: int) -> float:
        """Copy blocks into the target's staging arena at block offset `start` (IPC-mapped);
        blocking, returns seconds."""
        t0 = time.perf_counter()
        ev = self.push_async([(src_ids, target, start, "xgmi")])
        if ev is not None:
            ev.synchronize()
        return time.perf_counter() - t0

    def push_async(self, jobs: list, after=None):
        """Issue the KV pushes of `jobs` -- (src_ids, target, start, via) with via "xgmi" (the
        target's IPC-mapped GPU arena) or "shm" (its /dev/shm arena) -- without waiting for them.

        Ordering: the transfer stream waits on `after`, the event recorded right after the step that
        wrote these requests' last KV blocks (Request.kv_ready), not on everything queued on the
        compute stream: with async scheduling the next step is already queued when a step's outputs
        land, and waiting for it would hold every push one step back.  With
        `after` None the push orders after the whole current stream (callers without the event).
        Every xgmi job to one target goes out in ONE copy_blocks launch.  Returns an event recorded on
        the transfer stream after the copies (poll it; the source blocks must stay allocated until it
        fires), or None when the copies are already done (CPU)."""
        from .. import ops
        jobs = [j for j in jobs if j[0]]
        if not jobs:
            return None
        groups: dict = {}
        shm_jobs = []
        for src_ids, target, start, via in jobs:
            if via == "xgmi":
                if int(target["block_bytes"]) != self.block_bytes:
                    raise ValueError("KV block layout mismatch between prefill and decode workers")
                if start < 0 or start + len(src_ids) > int(target["arena_blocks"]):
                    raise ValueError(f"extent [{start}, +{len(src_ids)}) outside the staging arena")
                g = groups.setdefault(self._remote_ptr(target), ([], []))
                g[0].extend(src_ids)
                g[1].extend(range(start, start + len(src_ids)))
            elif via == "shm":
                if start < 0 or start + len(src_ids) > int(target["shm_blocks"]):
                    raise ValueError(f"extent [{start}, +{len(src_ids)}) outside the shm arena")
                shm_jobs.append((src_ids, self._shm_peer(target), start))
            else:
                raise ValueError(f"unknown KV push backend {via!r}")
        n = sum(len(j[0]) for j in jobs)
        self.bytes_moved += n * self.block_bytes
        self.transfers += len(jobs)
        if not self.is_gpu:
            for src_ids, arena, start in shm_jobs:
                idx = torch.tensor(src_ids, dtype=torch.long)
                arena.t[start:start + len(src_ids)].copy_(self.kv.index_select(0, idx))
            if groups:
                raise RuntimeError("xgmi push without a GPU")
            return None
        dev = self.kv.device
        if after is not None:
            self._stream.wait_event(after)
        else:
            self._stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self._stream):
            for ptr, (s_ids, d_ids) in groups.items():
                s_t = torch.tensor(s_ids, dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
                d_t = torch.tensor(d_ids, dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
                ops.ext().copy_blocks(ptr, self.kv, s_t, d_t, self.block_bytes)
            for src_ids, arena, start in shm_jobs:
                idx = torch.tensor(src_ids, dtype=torch.long).pin_memory().to(dev, non_blocking=True)
                arena.t[start:start + len(src_ids)].copy_(self.kv.index_select(0, idx), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        return ev
