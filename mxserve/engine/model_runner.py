"""Model runner: turns a SchedulerOutput into device tensors, runs the forward + sampling, and
returns sampled token ids.

MI355X specifics:
  * the KV pool is ONE block-major tensor [num_blocks, L, 2, Hkv, 16, D] sized from free HBM
    (288 GB per GPU -> millions of tokens for 1B/8B models); a block holds every layer's K and V,
    so a P->D transfer of a request is ceil(ISL/16) contiguous copies.
  * decode-only steps replay a hipGraph captured per batch-size bucket (torch.cuda.CUDAGraph is
    hipGraph on ROCm): a 16-layer decode step is ~170 kernels, and the ~1.2 us per launch boundary
    would otherwise dominate (MI355X_MICROARCH.md "boundary" / "launches-baseline" rows).
  * host-side block tables are persistent numpy rows updated incrementally, so a step copies only
    the rows of the batch.
"""
from __future__ import annotations

import logging
import math
import time
from typing import Optional

import numpy as np
import torch

from .. import ops
from ..config import EngineArgs
from ..models.config import ModelConfig
from ..models.llama import AttnMetadata, build_model
from ..models.weights import load_weights
from ..parallel.comm import get_tp, tp_broadcast_object
from .scheduler import SchedulerOutput

log = logging.getLogger(__name__)

_DTYPES = {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float16": torch.float16,
           "float32": torch.float32, "fp32": torch.float32}


def _graph_buckets(max_bs: int) -> list[int]:
    b = [1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256, 320, 384, 448, 512]
    return [x for x in b if x <= max_bs] or [max_bs]


class ModelRunner:
    def __init__(self, args: EngineArgs, cfg: ModelConfig, device: Optional[str] = None):
        self.args = args
        self.cfg = cfg
        dev = device or args.resolved_device()
        if dev == "cuda":
            dev = f"cuda:{torch.cuda.current_device()}"
        self.device = torch.device(dev)
        self.is_gpu = self.device.type == "cuda"
        self.dtype = _DTYPES[args.dtype] if self.is_gpu else torch.float32
        self.bs = args.block_size
        t0 = time.time()
        self.model = build_model(cfg, self.device, self.dtype)
        self.weight_source = load_weights(self.model, args.load_format, args.seed)
        log.info("weights (%s) ready in %.1fs", self.weight_source, time.time() - t0)
        self.max_blocks_per_seq = math.ceil(args.max_model_len / self.bs)
        self.num_blocks = self._determine_num_blocks()
        m = self.model
        self.kv_cache = torch.zeros(self.num_blocks, cfg.num_layers, 2, m.nkv, self.bs, cfg.head_dim,
                                    dtype=self.dtype, device=self.device)
        self.block_bytes = self.kv_cache[0].numel() * self.kv_cache.element_size()
        # persistent host block-table rows, one per live request
        self._bt_rows = np.zeros((args.max_num_seqs + 8, self.max_blocks_per_seq), dtype=np.int32)
        self._row_of: dict[str, int] = {}
        self._row_state: dict[str, tuple] = {}
        self._free_rows = list(range(self._bt_rows.shape[0] - 1, -1, -1))
        self.graphs: dict[int, tuple] = {}
        self._graph_pool = None
        if self.is_gpu and not args.enforce_eager:
            self._capture_graphs()

    # ------------------------------------------------------------------ memory
    def _determine_num_blocks(self) -> int:
        a, c, m = self.args, self.cfg, self.model
        per_block = c.num_layers * 2 * m.nkv * self.bs * c.head_dim * (2 if self.dtype != torch.float32 else 4)
        if a.num_gpu_blocks:
            return int(a.num_gpu_blocks)
        if not self.is_gpu:
            return int(a.cpu_num_blocks)
        torch.cuda.synchronize()
        free, total = torch.cuda.mem_get_info(self.device)
        # activation workspace for the largest step + logits + graph pools
        act = a.max_num_batched_tokens * (c.hidden_size * 12 + 2 * c.intermediate_size // m.tp_size) * 2
        act += a.max_num_seqs * c.vocab_size * 4 * 3 + (2 << 30)
        budget = int(total * a.gpu_memory_utilization) - (total - free) - act
        n = max(64, budget // per_block)
        log.info("KV pool: %d blocks x %.1f KiB = %.1f GB (%d tokens)", n, per_block / 1024, n * per_block / 1e9,
                 n * self.bs)
        return int(n)

    # ------------------------------------------------------------------ block-table rows
    def _row_for(self, req) -> int:
        rid = req.request_id
        row = self._row_of.get(rid)
        if row is None:
            row = self._free_rows.pop()
            self._row_of[rid] = row
            self._row_state[rid] = (-1, 0)
        gen, synced = self._row_state[rid]
        ids = req.block_ids
        if gen != req.kv_gen or synced > len(ids):
            synced = 0
        if len(ids) > synced:
            self._bt_rows[row, synced:len(ids)] = ids[synced:]
        self._row_state[rid] = (req.kv_gen, len(ids))
        return row

    def release(self, request_id: str) -> None:
        row = self._row_of.pop(request_id, None)
        self._row_state.pop(request_id, None)
        if row is not None:
            self._free_rows.append(row)

    # ------------------------------------------------------------------ inputs
    def _prepare(self, so: SchedulerOutput):
        reqs = so.all()
        S = len(reqs)
        nd = len(so.decodes)
        toks, pos, slots, seq_lens, qsl, rows, sample_rows = [], [], [], [], [0], [], []
        temps, tps, tks, seeds, steps = [], [], [], [], []
        max_q = 0
        for i, s in enumerate(reqs):
            r = s.req
            start, n = r.num_computed_tokens, s.num_new_tokens
            if n == 1:
                toks.append(r.token_at(start))
                p = np.array([start], dtype=np.int64)
            else:
                at = r.all_token_ids()
                toks.extend(at[start:start + n])
                p = np.arange(start, start + n, dtype=np.int64)
            pos.append(p)
            bids = np.asarray(r.block_ids, dtype=np.int64)
            slots.append(bids[p // self.bs] * self.bs + p % self.bs)
            seq_lens.append(start + n)
            qsl.append(qsl[-1] + n)
            rows.append(self._row_for(r))
            if i >= nd:
                max_q = max(max_q, n)
            if s.sample:
                sample_rows.append(i)
                sp = r.sampling
                temps.append(sp.temperature)
                tps.append(sp.top_p)
                tks.append(sp.top_k)
                seeds.append(r.seed)
                steps.append(len(r.output_token_ids))
        mb = max(1, max(-(-sl // self.bs) for sl in seq_lens))
        host = dict(
            input_ids=np.asarray(toks, dtype=np.int64),
            positions=np.concatenate(pos),
            slot_mapping=np.concatenate(slots),
            seq_lens=np.asarray(seq_lens, dtype=np.int32),
            qsl=np.asarray(qsl, dtype=np.int32),
            block_tables=self._bt_rows[np.asarray(rows), :mb],
            logits_indices=np.asarray([qsl[i + 1] - 1 for i in sample_rows], dtype=np.int64),
            temperature=np.asarray(temps, dtype=np.float32), top_p=np.asarray(tps, dtype=np.float32),
            top_k=np.asarray(tks, dtype=np.int32), seeds=np.asarray(seeds, dtype=np.int64),
            steps=np.asarray(steps, dtype=np.int64),
        )
        meta = dict(S=S, nd=nd, max_q=max_q, max_seq=max(seq_lens), sample_rows=sample_rows)
        return host, meta

    def _to_dev(self, a: np.ndarray) -> torch.Tensor:
        t = torch.from_numpy(np.ascontiguousarray(a))
        if self.is_gpu:
            return t.pin_memory().to(self.device, non_blocking=True)
        return t

    # ------------------------------------------------------------------ execute
    def execute(self, so: SchedulerOutput) -> dict[str, int]:
        """Driver-rank entry: prepare host inputs, fan them out to TP followers, run."""
        if so.is_empty:
            return {}
        host, meta = self._prepare(so)
        meta["graph"] = bool(self.graphs) and not so.prefills and meta["S"] <= max(self.graphs)
        if get_tp().tp_size > 1:
            tp_broadcast_object(("step", host, meta))
        ids = self.execute_host(host, meta)
        if ids is None:
            return {}
        reqs = so.all()
        ids = ids.tolist()
        return {reqs[r].req.request_id: ids[k] for k, r in enumerate(meta["sample_rows"])}

    @torch.inference_mode()
    def execute_host(self, host: dict, meta: dict):
        if not meta["sample_rows"]:
            self._forward_eager(host, meta, sample=False)
            return None
        if meta.get("graph"):
            return self._run_graph(host, meta)
        return self._forward_eager(host, meta, sample=True)

    def follower_loop(self) -> None:
        """TP ranks > 0: mirror the driver's steps until it broadcasts shutdown."""
        while True:
            msg = tp_broadcast_object(None)
            if msg is None or msg[0] == "shutdown":
                return
            _, host, meta = msg
            self.execute_host(host, meta)

    def shutdown_followers(self) -> None:
        if get_tp().tp_size > 1 and get_tp().tp_rank == 0:
            tp_broadcast_object(("shutdown", None, None))

    def _metadata(self, d: dict, meta: dict, max_seq_len: Optional[int] = None) -> AttnMetadata:
        nd, S = meta["nd"], meta["S"]
        pq = None
        if S > nd and nd > 0:
            pq = d["qsl"][nd:] - d["qsl"][nd]
        elif S > nd:
            pq = d["qsl"]
        return AttnMetadata(
            positions=d["positions"], slot_mapping=d["slot_mapping"], block_tables=d["block_tables"],
            seq_lens=d["seq_lens"], query_start_loc=d["qsl"], logits_indices=d["logits_indices"],
            num_decodes=nd, num_prefills=S - nd, num_prefill_tokens=int(d["input_ids"].shape[0]) - nd,
            max_query_len=meta["max_q"], max_seq_len=max_seq_len or meta["max_seq"],
            prefill_query_start_loc=pq)

    def _forward_eager(self, host: dict, meta: dict, sample: bool):
        d = {k: self._to_dev(v) for k, v in host.items()}
        md = self._metadata(d, meta)
        hidden = self.model.forward(d["input_ids"], md, self.kv_cache)
        if not sample:
            return None
        logits = self.model.compute_logits(hidden)
        ids = ops.sample(logits, d["temperature"], d["top_p"], d["top_k"], d["seeds"], d["steps"])
        return ids.cpu()

    # ------------------------------------------------------------------ hipGraph decode
    def _alloc_static(self, maxb: int) -> dict:
        dev = self.device
        return dict(
            input_ids=torch.zeros(maxb, dtype=torch.int64, device=dev),
            positions=torch.zeros(maxb, dtype=torch.int64, device=dev),
            slot_mapping=torch.full((maxb,), -1, dtype=torch.int64, device=dev),
            seq_lens=torch.ones(maxb, dtype=torch.int32, device=dev),
            qsl=torch.arange(maxb + 1, dtype=torch.int32, device=dev),
            block_tables=torch.zeros(maxb, self.max_blocks_per_seq, dtype=torch.int32, device=dev),
            logits_indices=torch.arange(maxb, dtype=torch.int64, device=dev),
            temperature=torch.zeros(maxb, dtype=torch.float32, device=dev),
            top_p=torch.ones(maxb, dtype=torch.float32, device=dev),
            top_k=torch.zeros(maxb, dtype=torch.int32, device=dev),
            seeds=torch.zeros(maxb, dtype=torch.int64, device=dev),
            steps=torch.zeros(maxb, dtype=torch.int64, device=dev),
        )

    def _graph_body(self, st: dict, b: int) -> torch.Tensor:
        d = {k: (v[:b] if k != "qsl" else v[:b + 1]) for k, v in st.items()}
        md = AttnMetadata(
            positions=d["positions"], slot_mapping=d["slot_mapping"], block_tables=d["block_tables"],
            seq_lens=d["seq_lens"], query_start_loc=d["qsl"], logits_indices=d["logits_indices"],
            num_decodes=b, num_prefills=0, num_prefill_tokens=0, max_query_len=1,
            max_seq_len=self.args.max_model_len)
        hidden = self.model.forward(d["input_ids"], md, self.kv_cache)
        logits = self.model.compute_logits(hidden)
        return ops.sample(logits, d["temperature"], d["top_p"], d["top_k"], d["seeds"], d["steps"])

    def _capture_graphs(self) -> None:
        maxb = min(self.args.cuda_graph_max_bs, self.args.max_num_seqs)
        buckets = _graph_buckets(maxb)
        self._static = self._alloc_static(max(buckets))
        t0 = time.time()
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        with torch.inference_mode():
            for b in sorted(buckets, reverse=True):
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    for _ in range(2):  # warm-up (allocator, hipBLASLt heuristics)
                        self._graph_body(self._static, b)
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    out = self._graph_body(self._static, b)
                self.graphs[b] = (g, out)
        torch.cuda.synchronize()
        log.info("captured %d decode graphs (%s) in %.1fs", len(buckets), buckets, time.time() - t0)

    def _run_graph(self, host: dict, meta: dict) -> torch.Tensor:
        S = meta["S"]
        b = min(x for x in self.graphs if x >= S)
        st = self._static
        mb = host["block_tables"].shape[1]
        st["input_ids"][:S].copy_(self._to_dev(host["input_ids"]), non_blocking=True)
        st["positions"][:S].copy_(self._to_dev(host["positions"]), non_blocking=True)
        st["slot_mapping"][:S].copy_(self._to_dev(host["slot_mapping"]), non_blocking=True)
        st["seq_lens"][:S].copy_(self._to_dev(host["seq_lens"]), non_blocking=True)
        st["block_tables"][:S, :mb].copy_(self._to_dev(host["block_tables"]), non_blocking=True)
        for k in ("temperature", "top_p", "top_k", "seeds", "steps"):
            st[k][:S].copy_(self._to_dev(host[k]), non_blocking=True)
        if b > S:  # padding rows: no cache writes, 1-token context
            st["slot_mapping"][S:b].fill_(-1)
            st["seq_lens"][S:b].fill_(1)
        g, out = self.graphs[b]
        g.replay()
        return out[:S].cpu()

    # ------------------------------------------------------------------ misc
    def kv_stats(self) -> dict:
        return {"num_blocks": self.num_blocks, "block_bytes": self.block_bytes,
                "kv_bytes": self.num_blocks * self.block_bytes}

