"""Decode projection GEMMs on the hand-written MFMA kernel (csrc/kernels/gemm_decode.hip), chosen per
(batch bucket, projection) by measurement.

When the decode graphs are captured, ModelRunner calls `tune()` with the model's projection shapes
(qkv, o, gate_up with SiLU*mul fused, down, lm_head) and the graph batch buckets.  For every pair it
times hipBLASLt (+ the separate SiLU*mul kernel for gate_up) and a set of kernel configurations
(wave tile MF x NF fragments, wave layout, split-K), each as 20 calls replayed from one hipGraph
(no launch gaps, the way the decode graphs run them), checks the winner against hipBLASLt's output
and records it.  `linear()` / `gate_up_silu()` then use the table; anything not tuned, or where
hipBLASLt won, stays on hipBLASLt.  MXS_DECODE_GEMM=off disables the kernel, =force uses a default
configuration without timing (tests).
"""
from __future__ import annotations

import bisect
import json
import logging
import os
import time
from typing import Optional

import torch

log = logging.getLogger(__name__)

# largest decode batch the table serves (MXS_DECODE_GEMM_MAX_M; the graph buckets run to 384)
MAX_M = int(os.environ.get("MXS_DECODE_GEMM_MAX_M", "448"))  # the bench's 448-sequence cap
# buckets the capture-time tuner measures (the whole decode-graph range): up to OLD_FORMS_MAX_M the
# register / LDS forms compete, above it only the medium-M (mt) kernel, since the register-staged forms
# measured 1.3-2.5x behind hipBLASLt there (profiles/r2_decode_gemm_probe_vs_hipblaslt.jsonl)
MAX_TUNE_M = int(os.environ.get("MXS_DECODE_GEMM_TUNE_MAX_M", str(MAX_M)))
OLD_FORMS_MAX_M = 64
MODE = os.environ.get("MXS_DECODE_GEMM", "auto")  # auto | off | force


def _mf(M: int) -> int:
    return 1 if M <= 16 else (2 if M <= 32 else 4)


def unroll(mf: int, nf: int) -> int:
    """k-steps per load group (csrc/kernels/gemm_decode.hip decode_gemm_unroll)."""
    return 8 if mf + nf <= 3 else (4 if mf + nf <= 6 else 2)


def candidates(M: int, N: int, K: int, epi: int, all_mf: bool = False, lds: bool = True,
               mt: bool = True) -> list[tuple]:
    """(mf, nf, wm, splitk, lu) configurations that tile the shape (wave row tile MF x 16 sized to M
    unless all_mf: then every MF, i.e. more row tiles re-reading the weights from L2).  lu = 0: the
    register kernel (wm waves over M); lu = 2 / 4: the LDS form (X tile shared by the workgroup's 4
    waves through LDS, lu k-steps per group).  With mt (dense weights; the grouped MoE form passes
    mt=False), from M = MT_MIN_M on, also the medium-M kernel's ("mt", wm, wn, wnf, splitk)
    configurations, plus the persistent prefill kernel ("pf", 0) on the widest projections and the
    skinny split-K form ("sk", kr, groups) at M <= 64."""
    out = []
    for mf in ((1, 2, 4) if all_mf else (_mf(M),)):
        out += _candidates_mf(M, N, K, epi, mf)
        if lds and mf > 1:  # one 16-row tile: the X fragment is as small as one W fragment
            out += _candidates_lds(N, K, epi, mf)
    # dense only (the grouped MoE form has no mt kernel); below MT_MIN_M only for large matrices,
    # where its coalesced LDS-staged weight stream reaches 5.3-5.6 TB/s (Llama-3-70B gate_up / down at
    # M = 8-32, profiles/r2_mt_gemm_probe_70b_cold_weights.jsonl) -- TP-8 shards of those included
    if mt and (M >= MT_MIN_M or N * K * 2 >= MT_SMALL_M_MIN_BYTES):
        out += mt_candidates(M, N, K, epi)
    # the persistent 256 x 256-tile prefill kernel (gemm_pf.hip, data-parallel tiles) on the widest
    # projections only -- lm_head: 501 column tiles keep every CU busy at any batch; 154 vs 183 us at
    # M = 256 (profiles/r4/gemm_pf_at_decode_batches.jsonl), while narrow ones leave it a dozen tiles
    if not mt:  # the grouped (MoE) form: register / LDS configurations only
        return out
    if M >= PF_MIN_M and N % 256 == 0 and K % 64 == 0 and N >= PF_MIN_N:
        out.append(("pf", 0))
    # M <= 4: whole weight rows streamed once, 1 KiB per load instruction (gemv_stream_kernel; SwiGLU
    # in the epilogue or the split-K reduce): ("gv", rows per wave, waves splitting K[, k-groups])
    if M <= GV_MAX_M:
        out += gv_candidates(M, N, K, epi)
    # small batches: 16-column weight slices streamed with every load in flight (skinny_gemm_kernel;
    # SwiGLU: slabs + the SiLU*mul reduce)
    if M <= 64 and N % (32 if epi else 16) == 0:
        krs = (128, 256) if M <= 16 else (64, 128)  # 2 / 4 token fragments above 16 rows
        out += [("sk", kr, K // (4 * kr)) for kr in krs if K % (4 * kr) == 0]
    return out


PF_MIN_M = 128
PF_MIN_N = 32768
# the kernel takes M <= 16, but from 8 rows on its dot2 VALU work outgrows the weight stream: at M = 8 /
# 16 the skinny form and hipBLASLt win every shape measured (profiles/r5/gemv/gv_probe_8_16.jsonl)
GV_MAX_M = 4


def gv_candidates(M: int, N: int, K: int, epi: int) -> list[tuple]:
    """Row-stream GEMV configurations (gemm_decode.hip launch_gemv_stream) that tile the shape:
    ("gv", rows per wave, waves splitting a workgroup's K, workgroups splitting K over the grid)."""
    mr = 1 if M <= 1 else (2 if M <= 2 else (4 if M <= 4 else (8 if M <= 8 else 16)))
    ocols = N // 2 if epi else N
    out = []
    for kg in ((1, 2) if M <= 4 else (1, 2, 4, 8)):
        if mr * (K // kg) * 2 > 64 * 1024 or (kg > 1 and ocols % 4):
            continue
        for nr in (2, 4):
            for kw in (1, 2, 4):
                per_wg = (4 // kw) * (nr // 2 if epi else nr)
                if K % (512 * kw * kg) == 0 and ocols % per_wg == 0:
                    out.append(("gv", nr, kw) if kg == 1 else ("gv", nr, kw, kg))
    return out


MT_MIN_M = 64
SPLITS = (1, 2, 4, 8, 16, 32)  # split-K factors the tuner tries (16 / 32: narrow shards over a long K)
MT_SMALL_M_MIN_BYTES = int(os.environ.get("MXS_MT_SMALL_M_MIN_BYTES", str(48 << 20)))
MT_COUNTERS = 1 << 16  # tile counters of the in-launch split-K reduction (every launch leaves them zero)
# in-launch split-K reduction (last arriver sums the slabs): measured slower than the separate reduce
# kernel at every decode shape (agent-scope release per workgroup + a serial slab read), so opt-in
MT_FUSED_REDUCE = os.environ.get("MXS_MT_FUSED_REDUCE", "0") == "1"
# (WM, WN, MR, WNF) of the medium-M kernel (gemm_decode.hip mt_gemm_kernel): WM x WN waves, each 32 MR
# rows x 32 WNF weight rows
MT_LAYOUTS = ((4, 1, 2, 2), (4, 2, 2, 2), (4, 1, 2, 4), (2, 2, 2, 2), (2, 2, 2, 4), (2, 4, 2, 2), (1, 4, 2, 2),
              (1, 2, 2, 2), (2, 1, 2, 2), (8, 1, 1, 4), (4, 2, 1, 2), (2, 4, 1, 2))


def mt_candidates(M: int, N: int, K: int, epi: int, max_blocks: int = 1024) -> list[tuple]:
    out = []
    for wm, wn, mr, wnf in MT_LAYOUTS:
        bm = 32 * mr * wm
        if bm > 64 and bm >= 2 * M:  # half the tile's rows empty: a smaller WM covers it
            continue
        if epi and wnf % 2:
            continue
        outb = 32 * (wnf // 2 if epi else wnf) * wn
        outN = N // 2 if epi else N
        if outN % outb:
            continue
        ntm = -(-M // bm)
        tiles = ntm * (outN // outb)
        for sk in SPLITS[:5]:
            if K % (64 * sk) or K // sk < 128 or tiles * sk > max_blocks:
                continue
            out.append(("mt", wm, wn, mr, wnf, sk))
            if ntm > 1:  # row tiles fastest: the tiles sharing a weight slice run together on one XCD
                out.append(("mt", wm, wn, mr, wnf, sk, 1))
    return out


def _candidates_lds(N: int, K: int, epi: int, mf: int) -> list[tuple]:
    out = []
    for nf in (2, 4):
        nh = nf // 2 if epi else nf
        if (N // 2 if epi else N) % (4 * nh * 16):
            continue
        for lu in (2, 4):
            for sk in (1, 2, 4, 8):
                if K % (32 * lu * sk) == 0:
                    out.append((mf, nf, 1, sk, lu))
    return out


def _candidates_mf(M: int, N: int, K: int, epi: int, mf: int) -> list[tuple]:
    out = []
    for wm in (1, 2, 4):
        if wm > 1 and (wm // 2) * mf * 16 >= M:  # waves with no rows at all
            continue
        wn = 4 // wm
        for nf in (2, 4):
            nh = nf // 2 if epi else nf
            outN = N // 2 if epi else N
            if outN % (wn * nh * 16):
                continue
            ntiles = outN // (wn * nh * 16)
            for sk in SPLITS:
                if K % (32 * unroll(mf, nf) * sk):
                    continue
                # deep splits only where the column tiles alone leave the chip idle (TP-sharded
                # projections: Llama-3-70B qkv at TP 8 is 1280 columns over K = 8192)
                if sk > 8 and (ntiles * sk > 1024 or K // sk < 256):
                    continue
                out.append((mf, nf, wm, sk, 0))
    return out


class DecodeGemmTable:
    def __init__(self):
        self.entries: dict[tuple, list] = {}  # (N, K, epi) -> sorted [(M bucket, cfg or None)]
        self.part: Optional[torch.Tensor] = None  # fp32 split-K workspace (stable for graphs)
        self.cnt: Optional[torch.Tensor] = None  # mt kernel tile counters (in-launch split-K reduce)
        self.report: list = []
        self.store_stats: dict = {}

    def lookup(self, M: int, N: int, K: int, epi: int) -> Optional[tuple]:
        if MODE == "off" or M > MAX_M:
            return None
        if MODE == "force":
            c = [x for x in candidates(M, N, K, epi) if x[0] not in ("mt", "pf", "sk", "gv")]
            return next((x for x in c if x[3] == 1), c[0] if c else None)
        ent = self.entries.get((N, K, epi))
        if not ent:
            return None
        i = bisect.bisect_left(ent, (M,))
        if i == len(ent):
            return None
        return ent[i][1]

    @staticmethod
    def splitk(cfg: tuple) -> int:
        if cfg[0] == "pf":
            return 1
        if cfg[0] == "gv":  # ("gv", nr, kw[, kg])
            return int(cfg[3]) if len(cfg) > 3 else 1
        if cfg[0] == "sk":  # ("sk", kr, k-groups of 4 x kr)
            return cfg[2]
        return cfg[5] if cfg[0] == "mt" else cfg[3]

    def run(self, out: torch.Tensor, x: torch.Tensor, w: torch.Tensor, cfg: tuple, epi: int,
            reduce: bool = True) -> bool:
        """reduce=False (split-K configurations only): leave the fp32 slabs [sk][M][N] in self.part for
        the caller's epilogue kernel (ops.linear_add_rms_norm)."""
        from . import ext
        if cfg[0] == "pf":
            from . import gemm_pf
            return gemm_pf(x, w, epi, out, int(cfg[1])) is not None
        if cfg[0] == "gv":
            kg = int(cfg[3]) if len(cfg) > 3 else 1
            if epi and kg > 1 and not reduce:
                return False  # SwiGLU applies in the reduce
            part = None
            if kg > 1:
                need = kg * x.shape[0] * w.shape[0]
                if self.part is None or self.part.numel() < need:
                    if torch.cuda.is_current_stream_capturing():
                        return False
                    self.part = torch.empty(need, dtype=torch.float32, device=x.device)
                part = self.part
            return bool(ext().gemv_stream(out, x, w, part, int(cfg[1]), int(cfg[2]), int(epi), kg, reduce))
        if cfg[0] == "sk":
            groups = w.shape[1] // (4 * int(cfg[1]))
            if groups != cfg[2] or (epi and not reduce):
                return False
            part = None
            if groups > 1 or epi:
                need = groups * x.shape[0] * w.shape[0]
                if self.part is None or self.part.numel() < need:
                    if torch.cuda.is_current_stream_capturing():
                        return False
                    self.part = torch.empty(need, dtype=torch.float32, device=x.device)
                part = self.part
            return bool(ext().skinny_gemm(out, x, w, part, int(cfg[1]), reduce, int(epi)))
        mt = cfg[0] == "mt"
        if mt:
            wm, wn, mr, wnf, sk = cfg[1:6]
            order = cfg[6] if len(cfg) > 6 else 0
        else:
            mf, nf, wm, sk = cfg[:4]
            lu = cfg[4] if len(cfg) > 4 else 0
        part = None
        if sk > 1:
            need = sk * x.shape[0] * w.shape[0]
            if self.part is None or self.part.numel() < need:
                if torch.cuda.is_current_stream_capturing():
                    return False  # never allocate inside a capture (tune() sizes it beforehand)
                self.part = torch.empty(need, dtype=torch.float32, device=x.device)
            part = self.part
        if mt:
            if sk > 1 and (self.cnt is None or self.cnt.device != x.device):
                if torch.cuda.is_current_stream_capturing():
                    return False
                self.cnt = torch.zeros(MT_COUNTERS, dtype=torch.int32, device=x.device)
            return bool(ext().mt_gemm(out, x, w, part, wm, wn, mr, wnf, sk, epi,
                                      self.cnt if MT_FUSED_REDUCE and reduce else None, order, reduce))
        return bool(ext().decode_gemm(out, x, w, part, mf, nf, wm, sk, epi, lu, reduce))


TABLE = DecodeGemmTable()


COLD_BYTES = 512 << 20  # > the 256 MiB Infinity Cache: timed weights come from HBM, as in a decode step


def weight_copies(w: torch.Tensor, cold_bytes: int = COLD_BYTES, cap: int = 20) -> list:
    """[w] plus enough copies that cycling through them streams more bytes than the Infinity Cache
    holds: a decode step reads every layer's weights once (GBs), so a timing that replays one
    8-70 MB matrix from the cache ranks kernels on the wrong memory level."""
    n = max(1, min(cap, -(-cold_bytes // (w.numel() * w.element_size()))))
    return [w] + [w.clone() for _ in range(n - 1)]


def _graph_time(fn, iters: int = 20) -> float:
    """Microseconds per call of `fn`, from `iters` calls captured in one hipGraph.  `fn` may take the
    call index (to cycle through weight copies)."""
    import inspect
    if not inspect.signature(fn).parameters:
        f0 = fn
        fn = lambda i: f0()  # noqa: E731
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    del g
    return e0.elapsed_time(e1) * 1e3 / iters


FINALISTS = 3  # candidates re-timed after the screening pass
ROUNDS = 3  # interleaved timing rounds of the finalists and hipBLASLt; the median decides
WIN_MARGIN = 0.97  # a kernel replaces hipBLASLt only when its median is 3 % lower


def pick(lib_fn, cand_fns: dict) -> tuple:
    """Robust choice between hipBLASLt (`lib_fn`) and candidate kernels ({cfg: fn}): one screening
    timing per candidate, then FINALISTS candidates and the library re-timed in ROUNDS interleaved
    rounds; returns (cfg or None, median us of the choice, median us of hipBLASLt)."""
    from .tuned import median
    screen = sorted(((_graph_time(fn), cfg) for cfg, fn in cand_fns.items()), key=lambda t: t[0])
    finals = [cfg for _, cfg in screen[:FINALISTS]]
    times: dict = {None: []}
    for cfg in finals:
        times[cfg] = []
    for _ in range(ROUNDS):
        times[None].append(_graph_time(lib_fn))
        for cfg in finals:
            times[cfg].append(_graph_time(cand_fns[cfg]))
    med = {cfg: median(v) for cfg, v in times.items()}
    t_lib = med[None]
    best, best_t = None, t_lib
    for cfg in finals:
        if med[cfg] < t_lib * WIN_MARGIN and (best is None or med[cfg] < best_t):
            best, best_t = cfg, med[cfg]
    return best, best_t, t_lib


def _epilogues(spec, M: int, N: int, device, dtype):
    """(plain, slab) epilogue callables of a projection for timing: plain(y) runs the separate
    epilogue kernel on the bf16 projection output, slab(sk) the fused one on sk unreduced slabs.
    spec: ("add_norm",) -- residual add + RMSNorm (o / down at TP = 1); ("rope", Hq, Hkv, D) -- rope +
    cache write (qkv; unmapped slots, so the timing leaves no cache bytes behind)."""
    from . import ext
    if spec is None:
        return None, None
    if spec[0] == "add_norm":
        res = torch.randn(M, N, device=device).to(dtype)
        nw = torch.ones(N, device=device, dtype=dtype)
        h = torch.empty(M, N, device=device, dtype=dtype)
        return (lambda y: ext().fused_add_rms_norm(h, y, res, nw, 1e-5),
                lambda sk: ext().splitk_add_rms_norm(h, res, TABLE.part, sk, nw, 1e-5))
    _, hq, hkv, hd = spec
    pos = torch.zeros(M, dtype=torch.int64, device=device)
    slot = torch.full((M,), -1, dtype=torch.int64, device=device)
    cs = torch.zeros(8, hd, dtype=torch.float32, device=device)
    kv = torch.zeros(1, 2, hkv, 16, hd, dtype=dtype, device=device)
    q = torch.empty(M, hq, hd, dtype=dtype, device=device)
    return (lambda y: ext().rope_and_cache(q, y, pos, cs, kv, slot, None, None, hq, hkv, hd, 1e-6, 1.0, 1.0),
            lambda sk: ext().splitk_rope_and_cache(q, TABLE.part, sk, M, pos, cs, kv, slot, None, None, hq, hkv, hd,
                                                   1e-6, 1.0, 1.0))


def tune(shapes: dict, buckets: list, device, dtype=torch.bfloat16) -> list:
    """shapes: {name: (weight tensor [N, K], epi[, epilogue spec])}.  Fills TABLE; returns the report
    rows.  Choices come from the persisted table (ops/tuned.py) when it has the (shape, bucket);
    otherwise they are measured (pick()) and added to it.  With an epilogue spec (_epilogues) every
    alternative is timed together with what follows it in the layer: hipBLASLt and unsplit kernels
    plus the separate epilogue kernel, split-K kernels with their slabs summed by the fused epilogue
    (ops.linear_add_rms_norm / ops.linear_rope_and_cache), so the choice prices the fusion."""
    if MODE != "auto":
        return []
    from . import silu_mul
    from .tuned import TunedStore, device_tag
    t0 = time.time()
    bks = sorted(b for b in buckets if b <= min(MAX_M, MAX_TUNE_M))
    if not bks:
        return []
    store = TunedStore("decode_gemm", device_tag(device))
    # workspace for the largest split-K any candidate may pick
    need = max(max(SPLITS) * max(bks) * v[0].shape[0] for v in shapes.values())
    TABLE.part = torch.empty(need, dtype=torch.float32, device=device)
    TABLE.cnt = torch.zeros(MT_COUNTERS, dtype=torch.int32, device=device)
    rows = []
    for name, val in shapes.items():
        w, epi = val[0], val[1]
        spec = val[2] if len(val) > 2 else None
        tag = {None: "", "add_norm": "+norm", "rope": "+rope"}[spec[0] if spec else None]
        N, K = w.shape
        ent = []
        ws = None
        for M in bks:
            x = (torch.randn(M, K, device=device) * 0.5).to(dtype)
            outN = N // 2 if epi else N
            ref_out = silu_mul(torch.nn.functional.linear(x, w)) if epi else torch.nn.functional.linear(x, w)
            out = torch.empty(M, outN, dtype=dtype, device=device)
            key = f"{N}x{K}x{epi}{tag}@{M}"
            st = store.get(key)
            source = "table"
            if st is not None:
                best, best_t, t_lib = st.get("cfg"), st.get("us"), st.get("hipblaslt_us")
                if best is not None and not TABLE.run(out, x, w, best, epi):
                    best = None  # no longer tiles this shape: hipBLASLt
            else:
                source = "measured"
                if ws is None:
                    ws = weight_copies(w)  # timed from HBM, as the decode step reads them
                plain, slab = _epilogues(spec, M, N, device, dtype)
                if epi:
                    lib_fn = lambda i: silu_mul(torch.nn.functional.linear(x, ws[i % len(ws)]))  # noqa: E731
                elif plain is not None:
                    lib_fn = lambda i: plain(torch.nn.functional.linear(x, ws[i % len(ws)]))  # noqa: E731
                else:
                    lib_fn = lambda i: torch.nn.functional.linear(x, ws[i % len(ws)])  # noqa: E731
                fns = {}
                for cfg in candidates(M, N, K, epi):
                    if cfg[0] not in ("mt", "pf", "sk", "gv") and M > OLD_FORMS_MAX_M:
                        continue
                    if not TABLE.run(out, x, w, cfg, epi):
                        continue
                    if plain is None:
                        fns[cfg] = (lambda c: (lambda i: TABLE.run(out, x, ws[i % len(ws)], c, epi)))(cfg)
                    elif TABLE.splitk(cfg) > 1:
                        fns[cfg] = (lambda c: (lambda i: (TABLE.run(out, x, ws[i % len(ws)], c, epi, reduce=False),
                                                          slab(TABLE.splitk(c)))))(cfg)
                    else:
                        fns[cfg] = (lambda c: (lambda i: (TABLE.run(out, x, ws[i % len(ws)], c, epi),
                                                          plain(out))))(cfg)
                best, best_t, t_lib = pick(lib_fn, fns) if fns else (None, None, _graph_time(lib_fn))
            if best is not None:  # correctness gate: the winner must match hipBLASLt's result
                TABLE.run(out, x, w, best, epi)
                err = (out.float() - ref_out.float()).abs().max().item()
                tol = 0.02 * max(1.0, ref_out.float().abs().max().item())
                if not err <= tol:
                    log.warning("decode GEMM %s M=%d cfg %s mismatches hipBLASLt (%.3g); not used", name, M, best, err)
                    best, best_t = None, t_lib
            if source == "measured":
                store.put(key, {"cfg": best, "us": round(best_t, 2) if best_t else None,
                                "hipblaslt_us": round(t_lib, 2) if t_lib else None})
            ent.append((M, best))
            rows.append({"proj": name, "M": M, "N": N, "K": K, "epi": epi, "hipblaslt_us": t_lib and round(t_lib, 2),
                         "chosen": "hipblaslt" if best is None else "mfma", "cfg": best,
                         "us": best_t and round(best_t, 2), "source": source, "epilogue": tag or None})
        TABLE.entries[(N, K, epi)] = ent
        del ws
    TABLE.report = rows
    TABLE.store_stats = {"table_hits": store.hits, "measured": store.misses, "device": store.tag}
    store.save()
    won = sum(r["chosen"] == "mfma" for r in rows)
    log.info("decode GEMM tuning: MFMA kernel chosen for %d of %d (bucket, projection) pairs in %.1fs "
             "(%d from the persisted table)", won, len(rows), time.time() - t0, store.hits)
    path = os.environ.get("MXS_DECODE_GEMM_REPORT")
    if path:
        with open(path, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return rows


class PrefillGemmTable:
    """Prefill-sized GEMMs (256 < M <= PREFILL_MAX_M) on the tile kernel of gemm_prefill.hip where
    the startup measurement found it faster than hipBLASLt: (N, K) -> sorted [(M bucket, cfg|None)].
    Above PREFILL_MAX_M the library's 256 x 256 tiles fill the chip and win
    (profiles/r2_prefill_gemm_probe_v1.jsonl)."""

    def __init__(self):
        self.entries: dict = {}
        self.report: list = []

    def lookup(self, M: int, N: int, K: int):
        if MODE == "off" or M > PREFILL_MAX_M:
            return None
        ent = self.entries.get((N, K))
        if not ent:
            return None
        i = bisect.bisect_left(ent, (M,))
        return ent[i][1] if i < len(ent) else None


PREFILL_MAX_M = int(os.environ.get("MXS_PREFILL_GEMM_MAX_M", "768"))
PREFILL_TABLE = PrefillGemmTable()


def _event_time(fn, iters: int = 10) -> float:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def tune_prefill(weights: dict, device, dtype=torch.bfloat16, buckets=(384, 512, 768)) -> list:
    """weights: {name: [N, K] tensor}.  Per M bucket: every tile / split-K configuration of the
    prefill kernel vs hipBLASLt (eager launches, as prefill runs), correctness-gated; the choice is
    persisted like the decode table's (median of ROUNDS timings of the finalists)."""
    if MODE != "auto":
        return []
    from .. import ops
    from .tuned import TunedStore, device_tag, median
    store = TunedStore("prefill_gemm", device_tag(device))
    rows = []
    for name, w in weights.items():
        N, K = w.shape
        ent = []
        for M in sorted(b for b in buckets if 256 < b <= PREFILL_MAX_M):
            x = (torch.randn(M, K, device=device) * 0.5).to(dtype)
            ref = torch.nn.functional.linear(x, w)
            out = torch.empty(M, N, dtype=dtype, device=device)
            key = f"{N}x{K}@{M}"
            st = store.get(key)
            if st is not None:
                best, best_t, t_lib = st.get("cfg"), st.get("us"), st.get("hipblaslt_us")
                if best is not None and not ops.prefill_gemm(out, x, w, best):
                    best = None
                source = "table"
            else:
                source = "measured"
                cands = [cfg for cfg in ops.prefill_gemm_configs(M, N, K) if ops.prefill_gemm(out, x, w, cfg)]
                screen = sorted((_event_time(lambda: ops.prefill_gemm(out, x, w, c)), c) for c in cands)
                finals = [c for _, c in screen[:FINALISTS]]
                tl, tc = [], {c: [] for c in finals}
                for _ in range(ROUNDS):
                    tl.append(_event_time(lambda: torch.nn.functional.linear(x, w)))
                    for c in finals:
                        tc[c].append(_event_time(lambda: ops.prefill_gemm(out, x, w, c)))
                t_lib = median(tl)
                best, best_t = None, t_lib
                for c in finals:
                    t = median(tc[c])
                    if t < t_lib * WIN_MARGIN and (best is None or t < best_t):
                        best, best_t = c, t
            if best is not None:
                ops.prefill_gemm(out, x, w, best)
                err = (out.float() - ref.float()).abs().max().item()
                if not err <= 0.02 * max(1.0, ref.float().abs().max().item()):
                    best, best_t = None, t_lib
            if source == "measured":
                store.put(key, {"cfg": best, "us": round(best_t, 2), "hipblaslt_us": round(t_lib, 2)})
            ent.append((M, best))
            rows.append({"proj": name, "M": M, "N": N, "K": K, "hipblaslt_us": t_lib and round(t_lib, 2),
                         "chosen": "hipblaslt" if best is None else "mfma", "cfg": best,
                         "us": best_t and round(best_t, 2), "source": source})
        PREFILL_TABLE.entries[(N, K)] = ent
    PREFILL_TABLE.report = rows
    store.save()
    return rows
