"""Persisted kernel choices (decode / prefill GEMM tables, MoE decode table).

The capture-time tuners (ops/decode_gemm.py, ops/moe.py) pick between the hand-written kernels and
hipBLASLt by timing.  Timed afresh on every start-up, near-ties flip between runs and the engine's
kernel mix (and its throughput) with them.  A TunedStore keeps the choice per (shape, batch bucket)
in a JSON file keyed by GPU architecture and CU count:

  * the package ships the tables measured on MI355X (mxserve/ops/tuned/<kind>_<arch>_<cus>cu.json);
    a shape found there is not re-timed, only re-checked for correctness, so every start-up on the
    same hardware runs the same kernels;
  * shapes not in the table are timed (median of repeated hipGraph timings, ops/decode_gemm.py) and
    added; MXS_TUNED_SAVE=1 writes the grown table back (to MXS_TUNED_DIR when set, else the package
    directory), MXS_RETUNE=1 ignores the stored choices (MXS_RETUNE=prefill_pf: only that table's).
"""
from __future__ import annotations

import json
import logging
import os
from typing import Optional

log = logging.getLogger(__name__)

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")


def device_tag(device=None) -> str:
    import torch
    p = torch.cuda.get_device_properties(device if device is not None else torch.cuda.current_device())
    arch = str(getattr(p, "gcnArchName", "") or p.name).split(":")[0].replace(" ", "_")
    return f"{arch}_{p.multi_processor_count}cu"


def _jsonable(v):
    if isinstance(v, tuple):
        return [_jsonable(x) for x in v]
    return v


def _tupled(v):
    if isinstance(v, list):
        return tuple(_tupled(x) for x in v)
    return v


class TunedStore:
    def __init__(self, kind: str, tag: str):
        self.kind = kind
        self.tag = tag
        rt = os.environ.get("MXS_RETUNE", "")
        self.retune = rt == "1" or kind in rt.split(",")  # "1": every table; "prefill_pf,...": those kinds
        self.save_enabled = os.environ.get("MXS_TUNED_SAVE") == "1"
        d = os.environ.get("MXS_TUNED_DIR")
        self.read_paths = ([os.path.join(d, self.filename)] if d else []) + [os.path.join(PKG_DIR, self.filename)]
        self.write_path = os.path.join(d or PKG_DIR, self.filename)
        self.entries: dict = {}
        self.hits = 0
        self.misses = 0
        self.dirty = False
        for p in reversed(self.read_paths):  # MXS_TUNED_DIR entries override the packaged ones
            self._load(p)

    @property
    def filename(self) -> str:
        return f"{self.kind}_{self.tag}.json"

    def _load(self, path: str) -> None:
        try:
            with open(path) as f:
                d = json.load(f)
        except FileNotFoundError:
            return
        except (OSError, ValueError) as e:
            log.warning("tuned table %s unreadable (%s); ignored", path, e)
            return
        for k, v in (d.get("entries") or {}).items():
            self.entries[k] = v

    def get(self, key: str) -> Optional[dict]:
        if self.retune:
            return None
        e = self.entries.get(key)
        if e is None:
            self.misses += 1
            return None
        self.hits += 1
        return dict(e, cfg=_tupled(e.get("cfg")))

    def put(self, key: str, entry: dict) -> None:
        self.entries[key] = {k: _jsonable(v) for k, v in entry.items()}
        self.dirty = True

    def save(self) -> Optional[str]:
        if not (self.save_enabled and self.dirty):
            return None
        os.makedirs(os.path.dirname(self.write_path), exist_ok=True)
        tmp = self.write_path + f".tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump({"kind": self.kind, "device": self.tag, "entries": dict(sorted(self.entries.items()))}, f,
                      indent=0, sort_keys=False)
            f.write("\n")
        os.replace(tmp, self.write_path)
        self.dirty = False
        log.info("tuned table written: %s (%d entries)", self.write_path, len(self.entries))
        return self.write_path


def median(xs: list) -> float:
    s = sorted(xs)
    n = len(s)
    return s[n // 2] if n % 2 else 0.5 * (s[n // 2 - 1] + s[n // 2])
