"""KV transfer agent for disaggregated prefill -> decode (replaces NIXL).

Backends
  xgmi  the decode worker exports its block-major KV pool once (hipIpcGetMemHandle of the pool's
        allocation + offset); the prefill worker opens it (hipIpcOpenMemHandle, lazy peer access)
        and pushes a request's blocks with ONE copy kernel on a side stream: stores travel over
        xGMI straight into the decode GPU's HBM (or stay on-chip when both workers share a GPU).
  host  staged through host memory over the control plane (CPU backend, or GPUs without a shared
        IPC namespace): the prefill side ships the block bytes, the decode side writes them.
Block layout is identical on both sides ([L, 2, Hkv, 16, D] per block), so a transfer is a list of
(src_block, dst_block) pairs.
"""
from __future__ import annotations

import base64
import logging
import os
import threading
import time
from typing import Optional

import numpy as np
import torch

log = logging.getLogger(__name__)


class KVTransferAgent:
    def __init__(self, runner, backend: str = "xgmi"):
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

    # -------------------------------------------------------------- decode side
    def descriptor(self, host_url: Optional[str] = None) -> dict:
        d = {"backend": self.backend, "block_bytes": self.block_bytes, "pid": os.getpid(),
             "num_blocks": int(self.kv.shape[0]), "url": host_url,
             "shape": list(self.kv.shape[1:]), "dtype": str(self.kv.dtype).replace("torch.", "")}
        if self.backend == "xgmi":
            from .. import ops
            handle, off = ops.ext().ipc_export_pool(self.kv)
            d.update(handle=base64.b64encode(handle).decode(), offset=int(off),
                     device=self.kv.device.index, data_ptr=int(self.kv.data_ptr()))
        return d

    def write_blocks(self, dst_ids: list[int], payload: bytes) -> None:
        """Host backend, decode side: place shipped blocks into the pool."""
        n = len(dst_ids)
        arr = np.frombuffer(payload, dtype=np.uint8).copy()
        src = torch.from_numpy(arr).view(self.kv.dtype).view(n, *self.kv.shape[1:])
        idx = torch.tensor(dst_ids, dtype=torch.long, device=self.kv.device)
        self.kv.index_copy_(0, idx, src.to(self.kv.device))
        if self.is_gpu:
            torch.cuda.synchronize(self.kv.device)

    # -------------------------------------------------------------- prefill side
    def _remote_ptr(self, target: dict) -> int:
        if target.get("pid") == os.getpid():  # same process: plain device pointer
            return int(target["data_ptr"])
        key = target["handle"]
        with self._lock:
            ptr = self._opened.get(key)
            if ptr is None:
                from .. import ops
                ptr = int(ops.ext().ipc_open_pool(base64.b64decode(key), int(target["offset"])))
                self._opened[key] = ptr
            return ptr

    def read_blocks(self, src_ids: list[int]) -> bytes:
        idx = torch.tensor(src_ids, dtype=torch.long, device=self.kv.device)
        blk = self.kv.index_select(0, idx)
        return blk.cpu().contiguous().view(torch.uint8).numpy().tobytes()

    def push_xgmi(self, src_ids: list[int], dst_ids: list[int], target: dict) -> float:
        """Copy blocks into the (IPC-mapped) target pool; returns seconds spent (blocking)."""
        from .. import ops
        if not src_ids:
            return 0.0
        if int(target["block_bytes"]) != self.block_bytes:
            raise ValueError("KV block layout mismatch between prefill and decode workers")
        t0 = time.perf_counter()
        ptr = self._remote_ptr(target)
        with torch.cuda.stream(self._stream):
            s = torch.tensor(src_ids, dtype=torch.int32).pin_memory().to(self.kv.device, non_blocking=True)
            d = torch.tensor(dst_ids, dtype=torch.int32).pin_memory().to(self.kv.device, non_blocking=True)
            ops.ext().copy_blocks(ptr, self.kv, s, d, self.block_bytes)
        self._stream.synchronize()
        self.bytes_moved += len(src_ids) * self.block_bytes
        self.transfers += 1
        return time.perf_counter() - t0
