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
import os
import time
from typing import Optional

import numpy as np
import torch

from .. import ops
from ..config import EngineArgs
from ..models.config import ModelConfig
from ..models.llama import AttnMetadata, build_model
from ..models.weights import load_weights
from ..parallel.comm import (collectives_capturable, collectives_local, get_tp, setup_meta_ring, tp_barrier,
                             tp_broadcast_object)
from ..parallel.custom_allreduce import CollectiveFault
from .scheduler import SchedulerOutput

log = logging.getLogger(__name__)

_DTYPES = {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float16": torch.float16,
           "float32": torch.float32, "fp32": torch.float32}


def _graph_buckets(max_bs: int) -> list[int]:
    b = [1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256, 320, 384, 448, 512]
    return [x for x in b if x <= max_bs] or [max_bs]


class InputBuffers:
    """All per-step inputs in ONE pinned host buffer with a fixed layout, mirrored by one device
    buffer: a step is one H2D copy, and the decode graphs read their inputs straight from the
    device views (stable addresses)."""

    _SEGS = (("input_ids", np.int64, "T"), ("positions", np.int64, "T"), ("slot_mapping", np.int64, "T"),
             ("logits_indices", np.int64, "S"), ("seeds", np.int64, "S"), ("steps", np.int64, "S"),
             ("srows", np.int64, "S"), ("trow", np.int64, "T"),
             ("bt_idx", np.int64, "U"), ("seq_lens", np.int32, "S"), ("qsl", np.int32, "S1"),
             ("rows", np.int32, "S"), ("sseq", np.int32, "S"), ("top_k", np.int32, "S"), ("bt_val", np.int32, "U"),
             ("hlen", np.int32, "S"), ("plen", np.int32, "S"),
             ("temperature", np.float32, "S"), ("top_p", np.float32, "S"),
             ("rep", np.float32, "S"), ("freq", np.float32, "S"), ("pres", np.float32, "S"))

    def __init__(self, T: int, S: int, U: int, device: torch.device, pin: bool):
        cap = {"T": T, "S": S, "S1": S + 1, "U": U}
        off = 0
        self.layout = {}
        for name, dt, c in self._SEGS:
            n = cap[c]
            self.layout[name] = (off, n, dt)
            off += -(-n * np.dtype(dt).itemsize // 64) * 64
        self.nbytes = off
        self.host = torch.zeros(off, dtype=torch.uint8, pin_memory=pin)
        self.dev = self.host.to(device) if device.type != "cpu" else self.host
        self.caps = {name: n for name, (_, n, _) in self.layout.items()}
        self._done = None
        tdt = {np.int64: torch.int64, np.int32: torch.int32, np.float32: torch.float32}
        self.hn, self.d = {}, {}
        for name, (o, n, dt) in self.layout.items():
            sz = n * np.dtype(dt).itemsize
            self.hn[name] = self.host[o:o + sz].numpy().view(dt)
            self.d[name] = self.dev[o:o + sz].view(tdt[dt])

    def upload(self) -> None:
        if self.dev is not self.host:
            self.dev.copy_(self.host, non_blocking=True)
            if self._done is None:
                self._done = torch.cuda.Event()
            self._done.record()

    def wait_free(self) -> None:
        """Block until the last upload has consumed the pinned buffer (a step that samples nothing
        never syncs the host, and the next step must not overwrite bytes still in flight)."""
        if self._done is not None:
            self._done.synchronize()

    def host_bytes(self) -> bytes:
        return self.host.numpy().tobytes()

    def load_host_bytes(self, b: bytes) -> None:
        self.host.numpy()[:] = np.frombuffer(b, dtype=np.uint8)


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
        self.model = build_model(cfg, self.device, self.dtype, args.moe_dispatch)
        self.weight_source = load_weights(self.model, args.load_format, args.seed)
        log.info("weights (%s) ready in %.1fs", self.weight_source, time.time() - t0)
        self.max_blocks_per_seq = math.ceil(args.max_model_len / self.bs)
        # fp8 KV cache: e4m3fn bytes held in a uint8 tensor (every torch indexing op supports it;
        # the kernels and the reference ops read it as e4m3fn)
        kvd = args.kv_cache_dtype.lower()
        if kvd not in ("auto", "bf16", "bfloat16", "fp8", "fp8_e4m3", "fp8_e4m3fn"):
            raise ValueError(f"kv_cache_dtype must be auto|fp8 (got {args.kv_cache_dtype!r})")
        self.kv_fp8 = kvd.startswith("fp8")
        self.kv_dtype = torch.uint8 if self.kv_fp8 else self.dtype
        if self.kv_fp8 and "MXS_KV_SCALE" not in os.environ:
            self.model.calibrate_kv_scales(self.bs)
        # norm-folded weights of the fused prefill chain: allocated before the KV pool is sized, and
        # only those the start-up tuner (not run under enforce_eager) may still choose
        self.model.prepare_fused_prefill(tuning=self.is_gpu and not args.enforce_eager,
                                         max_rows=args.max_num_batched_tokens + args.max_num_seqs)
        self.num_blocks = self._determine_num_blocks()
        m = self.model
        self.kv_cache = torch.zeros(self.num_blocks, cfg.num_layers, 2, m.nkv, self.bs, cfg.head_dim,
                                    dtype=self.kv_dtype, device=self.device)
        self.block_bytes = self.kv_cache[0].numel() * self.kv_cache.element_size()
        # block tables live on the device, one persistent row per live request, updated
        # incrementally (a decode step touches at most one new entry per request)
        n_rows = args.max_num_seqs + 8
        self.bt_dev = torch.zeros(n_rows, self.max_blocks_per_seq, dtype=torch.int32, device=self.device)
        # last sampled token per row: a decode whose input was sampled by a step still in flight
        # (async scheduling) reads it here on the device
        self.last_tok = torch.zeros(n_rows, dtype=torch.int64, device=self.device)
        self.pad_row = n_rows - 1  # graph padding rows point here; never given to a request
        self._row_of: dict[str, int] = {}
        self._row_state: dict[str, tuple] = {}
        self._free_rows = list(range(n_rows - 2, -1, -1))
        self._row_temp = np.zeros(n_rows, dtype=np.float32)
        self._row_topp = np.ones(n_rows, dtype=np.float32)
        self._row_topk = np.zeros(n_rows, dtype=np.int32)
        self._row_seed = np.zeros(n_rows, dtype=np.int64)
        self._row_lp = np.full(n_rows, -1, dtype=np.int32)  # top_logprobs per row; -1 = no logprobs
        # sampling penalties: per-row (repetition, frequency, presence) and prompt length, and the
        # token history every step writes on the device (input token of each position)
        self._row_pen = np.tile(np.array([1.0, 0.0, 0.0], dtype=np.float32), (n_rows, 1))
        self._row_plen = np.zeros(n_rows, dtype=np.int32)
        self._hist_init: list = []
        self.hist_len = args.max_model_len
        self.hist = torch.zeros(n_rows, self.hist_len, dtype=torch.int32, device=self.device)
        self._pen_counts = (torch.empty(n_rows, cfg.vocab_size, dtype=torch.int32, device=self.device)
                            if self.is_gpu else None)
        self._logits: Optional[torch.Tensor] = None  # last step's logits rows (logprobs read them)
        self.max_tokens_per_step = args.max_num_batched_tokens + args.max_num_seqs
        self.buf = InputBuffers(self.max_tokens_per_step, n_rows,
                                self.max_tokens_per_step // self.bs + 4 * self.max_blocks_per_seq + n_rows,
                                self.device, pin=self.is_gpu)
        # per-step inputs to the other TP ranks: the InputBuffers image + meta through a /dev/shm ring
        if get_tp().tp_size > 1:
            setup_meta_ring(self.buf.nbytes + (4 << 20))
        # sampled ids come back through two alternating pinned buffers (step N's result is read
        # while step N+1, launched just before, may already be writing the other one)
        self._out_slot = 0
        self._steps = 0
        if self.is_gpu:
            self._out_pinned = [torch.zeros(n_rows, dtype=torch.int64, pin_memory=True) for _ in range(2)]
            # timing-enabled: with the start events below they give each step's GPU time (engine/pacing.py
            # fits its step-time model on them; host clocks cannot see when a step's kernels started)
            self._out_events = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
            self._start_events = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            self._start_slot = 0
        # custom all-reduce health: every TP step's end polls each rank's error word into one of two
        # pinned arrays (engine.py discards and recomputes a step whose poll is non-zero)
        self.collective_faults = 0
        self._err_slot = 0
        if self.is_gpu and get_tp().tp_size > 1 and get_tp().custom_ar is not None:
            self._err_pinned = [torch.zeros(8, dtype=torch.int32, pin_memory=True) for _ in range(2)]
            self._err_events = [torch.cuda.Event(), torch.cuda.Event()]
        self.graphs: dict[int, tuple] = {}
        if get_tp().tp_size > 1:  # every rank's start-up work is done before the first collective
            tp_barrier()
        if self.is_gpu and not args.enforce_eager:
            self._capture_graphs()

    # ------------------------------------------------------------------ memory
    def _determine_num_blocks(self) -> int:
        n = self._local_num_blocks()
        tp = get_tp()
        if tp.tp_size > 1:  # every rank must manage the same block ids
            import torch.distributed as dist
            t = torch.tensor([n], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=tp.cpu_group or tp.group)
            n = int(t.item())
        return n

    def _local_num_blocks(self) -> int:
        a, c, m = self.args, self.cfg, self.model
        per_block = c.num_layers * 2 * m.nkv * self.bs * c.head_dim * torch.empty(0, dtype=self.kv_dtype).element_size()
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
    def _row_for(self, req, upd_idx: list, upd_val: list) -> int:
        rid = req.request_id
        row = self._row_of.get(rid)
        if row is None:
            row = self._free_rows.pop()
            self._row_of[rid] = row
            self._row_state[rid] = (-1, 0)
            sp = req.sampling
            self._row_temp[row] = sp.temperature
            self._row_topp[row] = sp.top_p
            self._row_topk[row] = sp.top_k
            self._row_seed[row] = req.seed
            self._row_lp[row] = -1 if sp.logprobs is None else int(sp.logprobs)
            self._row_pen[row] = (sp.repetition_penalty, sp.frequency_penalty, sp.presence_penalty)
            self._row_plen[row] = len(req.prompt_token_ids)
            if sp.has_penalties:  # history of tokens this row never computes (prefix-cache hits)
                self._hist_init.append((row, req.all_token_ids()[:self.hist_len]))
        gen, synced = self._row_state[rid]
        ids = req.block_ids
        n = len(ids)
        if gen != req.kv_gen or synced > n:
            synced = 0
        if n > synced:
            base = row * self.max_blocks_per_seq
            upd_idx.extend(range(base + synced, base + n))
            upd_val.extend(ids[synced:])
            self._row_state[rid] = (req.kv_gen, n)
        return row

    def release(self, request_id: str) -> None:
        row = self._row_of.pop(request_id, None)
        self._row_state.pop(request_id, None)
        if row is not None:
            self._free_rows.append(row)

    # ------------------------------------------------------------------ inputs
    def _prepare(self, so: SchedulerOutput, graph_bs: int = 0) -> dict:
        """Fill the pinned staging buffer for this step; returns the host-side meta."""
        bs = self.bs
        self.buf.wait_free()
        h = self.buf.hn
        dec, pre = so.decodes, so.prefills
        nd, S = len(dec), len(dec) + len(pre)
        upd_idx: list = []
        upd_val: list = []
        toks, pos, slots, lens, rows, steps = [], [], [], [], [], []
        for s in dec:
            r = s.req
            p = s.start
            npr = len(r.prompt_token_ids)
            if p < npr:
                toks.append(r.prompt_token_ids[p])
            elif p - npr < len(r.output_token_ids):
                toks.append(r.output_token_ids[p - npr])
            else:  # sampled by the step in flight: read from last_tok on the device
                toks.append(-1)
            pos.append(p)
            slots.append(r.block_ids[p // bs] * bs + p % bs)
            lens.append(p + 1)
            rows.append(self._row_for(r, upd_idx, upd_val))
            steps.append(s.out_idx)
        T = nd
        h["trow"][:nd] = rows
        h["input_ids"][:nd] = toks
        h["positions"][:nd] = pos
        h["slot_mapping"][:nd] = slots
        qsl = list(range(nd + 1))
        sample_rows = list(range(nd))
        max_q = 0
        for i, s in enumerate(pre):
            r = s.req
            start, n = s.start, s.num_new_tokens
            at = r.all_token_ids()
            h["input_ids"][T:T + n] = at[start:start + n]
            p = np.arange(start, start + n, dtype=np.int64)
            h["positions"][T:T + n] = p
            bids = np.asarray(r.block_ids, dtype=np.int64)
            h["slot_mapping"][T:T + n] = bids[p // bs] * bs + p % bs
            row = self._row_for(r, upd_idx, upd_val)
            h["trow"][T:T + n] = row
            T += n
            qsl.append(T)
            lens.append(start + n)
            rows.append(row)
            max_q = max(max_q, n)
            if s.sample:
                sample_rows.append(nd + i)
                steps.append(s.out_idx)
        rows_np = np.asarray(rows, dtype=np.int32)
        h["seq_lens"][:S] = lens
        h["qsl"][:S + 1] = qsl
        h["rows"][:S] = rows_np
        ns = len(sample_rows)
        srows = rows_np[sample_rows] if ns != S else rows_np
        h["logits_indices"][:ns] = np.asarray(qsl, dtype=np.int64)[np.asarray(sample_rows, dtype=np.int64) + 1] - 1
        h["temperature"][:ns] = self._row_temp[srows]
        h["top_p"][:ns] = self._row_topp[srows]
        h["top_k"][:ns] = self._row_topk[srows]
        h["seeds"][:ns] = self._row_seed[srows]
        h["steps"][:ns] = steps
        h["srows"][:ns] = srows
        h["sseq"][:ns] = sample_rows
        pen = self._row_pen[srows]
        h["rep"][:ns], h["freq"][:ns], h["pres"][:ns] = pen[:, 0], pen[:, 1], pen[:, 2]
        h["plen"][:ns] = self._row_plen[srows]
        h["hlen"][:ns] = np.asarray(lens, dtype=np.int32)[sample_rows] if ns else []
        use_pen = bool(ns) and bool((pen[:, 0] != 1.0).any() or (pen[:, 1:] != 0.0).any())
        if graph_bs > S:  # padding rows of a graph bucket: no cache write, 1-token context, greedy
            h["input_ids"][S:graph_bs] = 0
            h["positions"][S:graph_bs] = 0
            h["slot_mapping"][S:graph_bs] = -1
            h["seq_lens"][S:graph_bs] = 1
            h["rows"][S:graph_bs] = self.pad_row
            h["srows"][S:graph_bs] = self.pad_row
            h["trow"][S:graph_bs] = self.pad_row
            h["temperature"][S:graph_bs] = 0.0
            h["rep"][S:graph_bs], h["freq"][S:graph_bs], h["pres"][S:graph_bs] = 1.0, 0.0, 0.0
            h["hlen"][S:graph_bs] = 1
            h["plen"][S:graph_bs] = 1
        U = len(upd_idx)
        big_update = None
        if U > self.buf.caps["bt_idx"]:
            big_update = (np.asarray(upd_idx, dtype=np.int64), np.asarray(upd_val, dtype=np.int32))
            U = 0
        elif U:
            h["bt_idx"][:U] = upd_idx
            h["bt_val"][:U] = upd_val
        lp = None
        if ns:
            lpk = self._row_lp[srows]
            if (lpk >= 0).any():
                sel = np.nonzero(lpk >= 0)[0]
                lp = (sel.tolist(), int(lpk[sel].max()))
        hist_init, self._hist_init = self._hist_init, []
        return dict(S=S, T=T, nd=nd, max_q=max_q, max_seq=max(lens), sample_rows=sample_rows, U=U,
                    big_update=big_update, graph_bs=graph_bs, lp=lp, pen=use_pen, hist_init=hist_init)

    def _upload(self, meta: dict) -> None:
        self.buf.upload()
        for row, toks in meta.get("hist_init") or ():
            t = torch.tensor(toks, dtype=torch.int32)
            self.hist[row, :len(toks)].copy_(t.to(self.device) if self.is_gpu else t)
        bt = self.bt_dev.view(-1)
        if meta["U"]:
            U = meta["U"]
            bt.index_copy_(0, self.buf.d["bt_idx"][:U], self.buf.d["bt_val"][:U])
        if meta["big_update"] is not None:
            idx, val = meta["big_update"]
            if self.is_gpu:
                bt.index_copy_(0, torch.from_numpy(idx).to(self.device), torch.from_numpy(val).to(self.device))
            else:
                bt.index_copy_(0, torch.from_numpy(idx), torch.from_numpy(val))

    # ------------------------------------------------------------------ execute
    def launch(self, so: SchedulerOutput) -> Optional[dict]:
        """Driver-rank entry: prepare inputs, fan them out to TP followers, enqueue the step and
        the copy of its sampled ids to the host.  Does not wait for the GPU."""
        if so.is_empty:
            return None
        S = len(so.decodes) + len(so.prefills)
        gbs = 0
        if self.graphs and not so.prefills and S <= max(self.graphs):
            gbs = min(x for x in self.graphs if x >= S)
        meta = self._prepare(so, gbs)
        t0ev = None
        if self.is_gpu:
            self._start_slot = (self._start_slot + 1) % len(self._start_events)
            t0ev = self._start_events[self._start_slot]
            t0ev.record()
        tp = get_tp()
        car = tp.custom_ar if tp.tp_size > 1 and self.is_gpu else None
        if car is not None and car.disabled:
            car = None
        if tp.tp_size > 1:
            self._steps += 1
            tp_broadcast_object(("step", self.buf.host_bytes(), meta))
            _fault_injection(self._steps, tp.tp_rank)
        ids = self.execute_host(meta)
        handle = {"so": so, "rows": meta["sample_rows"]}
        if car is not None:
            # every TP step, sampling or not: a fault is caught at the step that contains it
            self._err_slot ^= 1
            handle["err"] = self._err_pinned[self._err_slot]
            car.poll_into(handle["err"])
            if ids is None:
                ev = self._err_events[self._err_slot]
                ev.record()
                handle["ev"] = ev
        if ids is None:
            return handle
        lp = None
        if meta.get("lp") is not None:
            sel, k = meta["lp"]
            rows = torch.tensor(sel, dtype=torch.int64).to(self.device, non_blocking=True)
            with torch.inference_mode():
                lp = ops.logprobs(self._logits, rows, ids.index_select(0, rows), k)
            if self.is_gpu:
                lp = tuple(t.to("cpu", non_blocking=True) for t in lp)  # pageable: lands by the event below
            handle["lp_sel"] = sel
        if self.is_gpu:
            self._out_slot ^= 1
            pinned = self._out_pinned[self._out_slot][:ids.shape[0]]
            pinned.copy_(ids, non_blocking=True)
            ev = self._out_events[self._out_slot]
            ev.record()
            handle.update(pinned=pinned, ev=ev, ev0=t0ev)
        else:
            handle["ids"] = ids
        if lp is not None:
            handle["lp"] = lp
        return handle

    def collect(self, handle: Optional[dict]) -> dict[str, int]:
        """Wait for a launched step's sampled ids; {request_id: token}.  Log-probs, when any row
        asked for them, are left in handle["logprobs"] = {request_id: (logprob, [(id, logprob)])}."""
        if handle is None:
            return {}
        if "ev" in handle:
            handle["ev"].synchronize()
            err = handle.get("err")
            if err is not None and any(err.tolist()):
                raise CollectiveFault([int(v) for v in err.tolist()])
            if "pinned" not in handle:
                return {}
            if handle.get("ev0") is not None:
                handle["gpu_s"] = handle["ev0"].elapsed_time(handle["ev"]) * 1e-3
            ids = handle["pinned"].tolist()
        elif "ids" in handle:
            ids = handle["ids"].tolist()
        else:
            return {}
        reqs = handle["so"].all()
        rows = handle["rows"]
        if "lp" in handle:
            tok_lp, top_ids, top_lp = (t.tolist() for t in handle["lp"])
            handle["logprobs"] = {reqs[rows[k]].req.request_id: (tok_lp[j], list(zip(top_ids[j], top_lp[j])))
                                  for j, k in enumerate(handle["lp_sel"])}
        return {reqs[r].req.request_id: ids[k] for k, r in enumerate(rows)}

    def execute(self, so: SchedulerOutput) -> dict[str, int]:
        return self.collect(self.launch(so))

    def drain(self, handle: Optional[dict]) -> None:
        """Wait for a launched step without reading its results (it is being discarded)."""
        if handle is not None and "ev" in handle:
            handle["ev"].synchronize()

    @torch.inference_mode()
    def execute_host(self, meta: dict):
        """Run one step on this rank; returns the device tensor of sampled ids (or None)."""
        self._upload(meta)
        if meta["graph_bs"]:
            g, out, logits = self.graphs[meta["graph_bs"]]
            g.replay()
            self._logits = logits
            return out[:meta["S"]]
        return self._forward_eager(meta, sample=bool(meta["sample_rows"]))

    def follower_loop(self) -> None:
        """TP ranks > 0: mirror the driver's steps until it broadcasts shutdown."""
        while True:
            msg = tp_broadcast_object(None)
            if msg is None or msg[0] == "shutdown":
                return
            kind, host_bytes, meta = msg
            if kind == "car_reset":
                self._reset_collectives(meta)
                continue
            self._steps += 1
            _fault_injection(self._steps, get_tp().tp_rank)
            # the previous step's non_blocking H2D copy may still be reading the pinned buffer
            self.buf.wait_free()
            self.buf.load_host_bytes(host_bytes)
            self.execute_host(meta)

    def recover_collectives(self, fault: CollectiveFault) -> None:
        """Driver rank, after a custom all-reduce fault (its steps already discarded by the engine):
        log the diagnosis, then re-arm the path on every rank -- or, after MXS_CAR_MAX_FAULTS faults,
        turn it off and re-capture the decode graphs over RCCL."""
        tp = get_tp()
        car = tp.custom_ar
        diag = car.diagnose() if car is not None else []
        self.collective_faults += 1
        self.last_collective_fault = {"error_words": fault.words, "ranks": diag}
        limit = int(os.environ.get("MXS_CAR_MAX_FAULTS", "3"))
        meta = {"disable": self.collective_faults >= limit}
        log.error("custom all-reduce fault %d (%s): %s", self.collective_faults,
                  "turning it off" if meta["disable"] else "re-arming", self.last_collective_fault)
        tp_broadcast_object(("car_reset", None, meta))
        self._reset_collectives(meta)

    def _reset_collectives(self, meta: dict) -> None:
        """Every rank, in step order: quiesce, barrier, clear this rank's signal page, barrier.  With
        meta["disable"]: all-reduces go to RCCL from now on and the decode graphs (which hold the custom
        kernels) are re-captured over it when the group's backend can be captured (RCCL), else decode
        runs eagerly (gloo functional runs)."""
        tp = get_tp()
        car = tp.custom_ar
        if self.is_gpu:
            torch.cuda.synchronize()
        tp_barrier()
        if car is not None:
            car.faults += 1
            if meta.get("disable"):
                car.disabled = True
            else:
                car.reset()
        tp_barrier()
        if meta.get("disable"):
            self.graphs.clear()
            if self.is_gpu and not self.args.enforce_eager:
                self._capture_graphs(tune=False)

    def shutdown_followers(self) -> None:
        if get_tp().tp_size > 1 and get_tp().tp_rank == 0:
            tp_broadcast_object(("shutdown", None, None))

    def _views(self, S: int, T: int, ns: int) -> dict:
        d = self.buf.d
        return dict(input_ids=d["input_ids"][:T], positions=d["positions"][:T], slot_mapping=d["slot_mapping"][:T],
                    seq_lens=d["seq_lens"][:S], qsl=d["qsl"][:S + 1], rows=d["rows"][:S],
                    logits_indices=d["logits_indices"][:ns], temperature=d["temperature"][:ns],
                    top_p=d["top_p"][:ns], top_k=d["top_k"][:ns], seeds=d["seeds"][:ns], steps=d["steps"][:ns],
                    srows=d["srows"][:ns], sseq=d["sseq"][:ns], trow=d["trow"][:T], hlen=d["hlen"][:ns],
                    plen=d["plen"][:ns], rep=d["rep"][:ns], freq=d["freq"][:ns], pres=d["pres"][:ns])

    def _write_hist(self, v: dict, inp: torch.Tensor) -> None:
        """Token history for the penalties: every input token at (its row, its position)."""
        idx = v["trow"] * self.hist_len + v["positions"]
        self.hist.view(-1).index_copy_(0, idx, inp.to(torch.int32))

    def _penalize(self, v: dict, logits: torch.Tensor) -> None:
        ops.apply_penalties(logits, self.hist, v["srows"], v["hlen"], v["plen"], v["rep"], v["freq"], v["pres"],
                            self._pen_counts)

    def _forward_eager(self, meta: dict, sample: bool):
        S, T, nd = meta["S"], meta["T"], meta["nd"]
        v = self._views(S, T, len(meta["sample_rows"]))
        bt = self.bt_dev.index_select(0, v["rows"].long())
        pq = None
        if S > nd:
            pq = v["qsl"][nd:] - nd if nd > 0 else v["qsl"]
        md = AttnMetadata(positions=v["positions"], slot_mapping=v["slot_mapping"], block_tables=bt,
                          seq_lens=v["seq_lens"], query_start_loc=v["qsl"], logits_indices=v["logits_indices"],
                          num_decodes=nd, num_prefills=S - nd, num_prefill_tokens=T - nd,
                          max_query_len=meta["max_q"], max_seq_len=meta["max_seq"], prefill_query_start_loc=pq,
                          sample_seq=v["sseq"])
        inp = v["input_ids"]
        if nd:
            d_in = inp[:nd]
            d_in.copy_(torch.where(d_in < 0, self.last_tok.index_select(0, v["rows"][:nd].long()), d_in))
        self._write_hist(v, inp)
        hidden = self.model.forward(inp, md, self.kv_cache)
        if not sample:
            return None
        logits = self.model.compute_logits(hidden)
        if meta.get("pen"):
            self._penalize(v, logits)
        self._logits = logits
        ids = ops.sample(logits, v["temperature"], v["top_p"], v["top_k"], v["seeds"], v["steps"])
        self.last_tok.index_copy_(0, v["srows"], ids)
        return ids

    # ------------------------------------------------------------------ hipGraph decode
    def _graph_body(self, b: int) -> tuple:
        v = self._views(b, b, b)
        rows = v["rows"].long()
        bt = self.bt_dev.index_select(0, rows)
        inp = v["input_ids"]
        inp = torch.where(inp < 0, self.last_tok.index_select(0, rows), inp)
        self._write_hist(v, inp)
        md = AttnMetadata(
            positions=v["positions"], slot_mapping=v["slot_mapping"], block_tables=bt,
            seq_lens=v["seq_lens"], query_start_loc=v["qsl"], logits_indices=self._arange[:b],
            num_decodes=b, num_prefills=0, num_prefill_tokens=0, max_query_len=1,
            max_seq_len=self.args.max_model_len)
        hidden = self.model.forward(inp, md, self.kv_cache)
        logits = self.model.compute_logits(hidden)
        self._penalize(v, logits)  # rows with neutral penalties exit at once
        ids = ops.sample(logits, v["temperature"], v["top_p"], v["top_k"], v["seeds"], v["steps"])
        self.last_tok.index_copy_(0, v["srows"], ids)
        return ids, logits

    def _capture_graphs(self, tune: bool = True) -> None:
        maxb = min(self.args.cuda_graph_max_bs or min(self.args.max_num_seqs, 512), self.args.max_num_seqs)
        m = self.model
        # largest collective message of a decode step at batch b: the all-reduces of [b, H] and the
        # logits all-gather ([b, vocab/tp] per rank)
        msg = lambda b: b * max(self.cfg.hidden_size, m.vocab_local) * 2  # noqa: E731
        buckets = [b for b in _graph_buckets(maxb) if collectives_capturable(msg(b))]
        if not buckets:
            log.warning("no decode bucket has graph-capturable collectives; decode runs eagerly")
            return
        if tune:
            self._tune_gemms(buckets)
        self._capture(buckets)

    def _tune_gemms(self, buckets: list) -> None:
        m = self.model
        # decode projection GEMMs: hand-written MFMA kernel vs hipBLASLt, measured per bucket
        from ..ops import decode_gemm
        w = m.w
        # qkv feeds the rope / cache-write kernel (fusable at any TP); o / down feed the residual add +
        # next RMSNorm (llama.py _forward_fused: at TP = 1 the split-K slabs go into the norm kernel, at
        # TP > 1 into the fused all-reduce + add + norm kernel): the tuner times each with its epilogue
        from ..parallel.comm import get_tp
        fuse = getattr(m, "fuse_residual", False) and (m.tp_size == 1 or get_tp().custom_ar is not None)
        norm = ("add_norm",) if fuse else None
        shapes = {"qkv": (w["l0.qkv"], 0, ("rope", m.nh, m.nkv, m.hd) if self.cfg.head_dim in (64, 128) else None),
                  "o": (w["l0.o"], 0, norm), "lm_head": (m.lm_head_weight(), 0)}
        if not self.cfg.is_moe:
            shapes.update(gate_up=(w["l0.gate_up"], 1), down=(w["l0.down"], 0, norm))
        with torch.inference_mode():
            t0 = time.time()
            self.decode_gemm_report = decode_gemm.tune(shapes, buckets, self.device, self.dtype)
            self.decode_gemm_tune_s = time.time() - t0
            self.prefill_gemm_report = decode_gemm.tune_prefill(
                {k: v[0] for k, v in shapes.items() if v[1] == 0 and k != "lm_head"}, self.device, self.dtype)
            # prefill / mixed-step GEMMs: row-count plans around hipBLASLt's kernel-choice cliffs
            from ..ops import mplan
            self.mplan_report = mplan.tune({k: v[0] for k, v in shapes.items() if k != "lm_head"},
                                           self.args.max_num_batched_tokens + self.args.max_num_seqs, self.device)
            # prefill projections left on hipBLASLt: its fastest solution per row bucket (the gemm_pf
            # tuner below then compares against this path)
            from ..ops import prefill_hblt
            self.prefill_hblt_report = prefill_hblt.tune(
                {k: v[0] for k, v in shapes.items() if k != "lm_head"},
                {"o", "down"} if getattr(m, "pf_chain", False) else set(),
                self.args.max_num_batched_tokens + self.args.max_num_seqs, self.device, self.dtype)
            # prefill projections: the stream-K MFMA kernel (SwiGLU fused for gate_up) vs that path
            from ..ops import prefill_pf
            pf_w = {k: (v[0], v[1]) for k, v in shapes.items() if k != "lm_head"}
            self.prefill_pf_report = prefill_pf.tune(pf_w, self.args.max_num_batched_tokens + self.args.max_num_seqs,
                                                     self.device, self.dtype)
            if getattr(m, "pf_chain", False):  # the fused prefill chain (llama.py _forward_pf): fused vs unfused
                fw = {"o": (w["l0.o"], None, prefill_pf.CODE_RESID), "down": (w["l0.down"], None, prefill_pf.CODE_RESID)}
                for p, code in (("qkv", prefill_pf.CODE_RS), ("gate_up", prefill_pf.CODE_RS_SWIGLU)):
                    if "l0." + p in m.wf:  # folded only where the stored table does not reject it
                        fw[p] = (w["l0." + p], m.wf["l0." + p], code)
                rep = prefill_pf.tune_fused(fw, self.args.max_num_batched_tokens + self.args.max_num_seqs,
                                            self.device, self.dtype, self.cfg.rms_norm_eps)
                self.prefill_pf_report = self.prefill_pf_report + rep
                m.drop_folded([p for p in ("qkv", "gate_up")
                               if not any(r["proj"] == p and r["chosen"].startswith("gemm_pf") for r in rep)])
                torch.cuda.empty_cache()
            if self.cfg.is_moe and "l0.w13" in w:  # expert GEMMs at decode batches (local experts)
                from ..ops import moe as moe_ops
                self.moe_gemm_report = moe_ops.tune(w["l0.w13"], w["l0.w2"], buckets, self.cfg.num_experts_per_tok,
                                                    self.cfg.num_experts, m.e_offset, self.device)

    def _capture(self, buckets: list) -> None:
        self._arange = torch.arange(max(buckets), dtype=torch.int64, device=self.device)
        # benign contents for capture: every row is a 1-token sequence that writes nowhere
        h = self.buf.hn
        h["slot_mapping"][:] = -1
        h["seq_lens"][:] = 1
        h["rows"][:] = self.pad_row
        h["srows"][:] = self.pad_row
        h["qsl"][:] = np.arange(len(h["qsl"]))
        h["temperature"][:] = 0
        h["top_p"][:] = 1
        h["trow"][:] = self.pad_row
        h["rep"][:] = 1
        h["freq"][:] = 0
        h["pres"][:] = 0
        h["hlen"][:] = 1
        self.buf.upload()
        t0 = time.time()
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        tp_rank = get_tp().tp_rank
        with torch.inference_mode():
            for b in sorted(buckets, reverse=True):
                # the warm-up runs collectives: every rank starts it together.  Host work per rank
                # differs in length (the previous bucket's capture + hipGraph instantiation, first-call
                # library loads), and at TP on one shared GPU it spread ranks by over the all-reduce
                # wait budget (profiles/r5/car_timeout/README.md)
                tb = time.time()
                if get_tp().tp_size > 1 and not self.cfg.is_moe:
                    with collectives_local():  # first-call loads at this rank's own pace (comm.py)
                        self._graph_body(b)
                torch.cuda.synchronize()
                tp_barrier()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    for _ in range(2):  # warm-up (allocator, hipBLASLt heuristics)
                        self._graph_body(b)
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                tc = time.time()
                with torch.cuda.graph(g, pool=pool):
                    out, logits = self._graph_body(b)
                self.graphs[b] = (g, out, logits)
                log.info("rank %d bucket %d: barrier+warm-up %.2fs, capture %.2fs", tp_rank, b, tc - tb,
                          time.time() - tc)
        torch.cuda.synchronize()
        log.info("captured %d decode graphs (%s) in %.1fs", len(buckets), buckets, time.time() - t0)

    # ------------------------------------------------------------------ misc
    def close(self) -> None:
        if self.is_gpu:
            torch.cuda.synchronize(self.device)
        self.graphs.clear()
        self._logits = None
        for name in ("kv_cache", "model", "bt_dev", "last_tok", "hist", "_pen_counts", "buf"):
            setattr(self, name, None)

    def kv_stats(self) -> dict:
        return {"num_blocks": self.num_blocks, "block_bytes": self.block_bytes,
                "kv_bytes": self.num_blocks * self.block_bytes}



def _fault_injection(step: int, rank: int) -> None:
    """MXS_FAULT="car_delay:rank=R:step=K:ms=T" (tests): TP rank R sleeps T ms before launching its
    K-th step, so its peers' custom all-reduce waits run out (with MXS_CAR_TIMEOUT_MS < T)."""
    from ..utils.tracing import FAULTS
    kv = FAULTS.args.get("car_delay")
    if kv is None:
        return
    if int(kv.get("rank", 1)) == rank and int(kv.get("step", 5)) == step:
        log.warning("MXS_FAULT: rank %d sleeping %s ms before step %d", rank, kv.get("ms", "1000"), step)
        time.sleep(float(kv.get("ms", "1000")) / 1e3)
