"""Multi-GPU probe: tensor / expert parallelism, collectives and xGMI peer copies measured on the
node a multi-GPU bench runs on.

bench.py (N >= 2 ranks) starts one probe process per rank BEFORE anything touches the GPU; each
blocks on stdin until its rank has finished the serving phases and released its engine.  The probes
then form their own process group -- RCCL when every rank has its own GPU, else gloo with the custom
IPC all-reduce carrying the model's collectives (ranks sharing one GPU) -- and measure:

  disagg_headline  (when bench.py hands over its arguments in MXS_PROBE_DISAGG_ARGV) bench.py's own
               disaggregated phase, run first and outside the section budget; the per-rank stat rows
               go back to bench.py, which reports them as the line's `disagg`
  collectives  all-reduce of bf16 buffers 64 KiB - 256 MiB through the process group (RCCL over xGMI
               on a real node): time, algorithm and bus bandwidth (2 (n-1) / n x bytes / t); the
               custom IPC all-reduce (one-shot / two-shot) 16 KiB - 8 MiB
  tp           Llama-3-70B layer shapes (2 layers, random weights) sharded TP=N against the
               unsharded model on rank 0: logit error, argmax agreement, and the forward time of a
               64-token batch at TP=N vs TP=1
  ep           Mixtral-8x7B layer shapes (2 layers), experts sharded EP=N with the device-side IPC
               token dispatch, against the unsharded model
  tp_engine    the full Llama-3-70B (80 layers, random weights; BASELINE config 4) as a TP=N serving
               engine -- rank 0 schedules, ranks 1..N-1 mirror its steps (ModelRunner.follower_loop),
               decode in hipGraphs with the custom all-reduce captured -- 64 requests of 512 prompt
               tokens, 64 output tokens each: median decode step (the ITL at batch 64) and prefill rate
  ep_engine    the full Mixtral-8x7B the same way with its experts sharded EP=N (tokens dispatched to
               the expert owners by the device-side IPC all-to-all; BASELINE config 5's EP)
  disagg_8b    Llama-3-8B disaggregated 1P+1D (BASELINE config 3): ranks [0, N/2) prefill, [N/2, N)
               decode, the KV of each prompt pushed over xGMI into the decode GPU's arena -- bench.py's
               disagg phase (Poisson arrivals, ISL 4000 / OSL 500, steady-state warmup) at 4 req/s per
               pair: TTFT (KV transfer included) and ITL
  p2p          rank 0: peer copy bandwidth to every other GPU it sees, one link at a time and all
               links at once (hipMemcpyPeer over xGMI)

bench.py's own disagg phase runs here first (disagg_headline).  Its first trial faulted the next
section: the KV agent's teardown unmapped the custom all-reduce's peer slots (an ipc_close_all;
fixed: agents close only their own mappings; profiles/r2_s5_hosted_disagg_fault.txt).

A crash or hang in a probe costs only the probe (its rank reports {"status": "failed"}); the
serving numbers of the bench stand.  Rank 0 prints one line `PROBE {json}` on its original stdout.
The CPU plumbing run (bench.py --device cpu) uses the tiny configs over gloo.
"""
from __future__ import annotations

import json
import os
import sys
import time
import traceback

MODEL_TP = "meta-llama/Meta-Llama-3-70B-Instruct@layers=2"
MODEL_EP = "mistralai/Mixtral-8x7B-Instruct-v0.1@layers=2"
MODEL_TP_ENGINE = "meta-llama/Meta-Llama-3-70B-Instruct"
MODEL_EP_ENGINE = "mistralai/Mixtral-8x7B-Instruct-v0.1"
MODEL_DISAGG = "meta-llama/Meta-Llama-3-8B-Instruct"


def _md(n, dev):
    import torch
    from ..models.llama import AttnMetadata
    nb = (n + 15) // 16
    pos = torch.arange(n, device=dev)
    qsl = torch.tensor([0, n], dtype=torch.int32, device=dev)
    return AttnMetadata(positions=pos, slot_mapping=pos.clone(), block_tables=torch.arange(
        nb, dtype=torch.int32, device=dev).unsqueeze(0), seq_lens=torch.tensor([n], dtype=torch.int32, device=dev),
        query_start_loc=qsl, logits_indices=torch.arange(n, device=dev), num_decodes=0, num_prefills=1,
        num_prefill_tokens=n, max_query_len=n, max_seq_len=n, prefill_query_start_loc=qsl)


class Probe:
    def __init__(self):
        import torch
        self.torch = torch
        self.rank = int(os.environ["RANK"])
        self.world = int(os.environ["WORLD_SIZE"])
        self.local = int(os.environ.get("LOCAL_RANK", self.rank))
        self.on_gpu = os.environ.get("MXS_PROBE_DEVICE", "auto") != "cpu" and torch.cuda.is_available()
        self.ndev = torch.cuda.device_count() if self.on_gpu else 0
        self.shared = self.on_gpu and self.ndev < self.world
        self.dev = torch.device("cuda", self.local % self.ndev) if self.on_gpu else torch.device("cpu")
        self.dtype = torch.bfloat16 if self.on_gpu else torch.float32
        self.backend = "nccl" if self.on_gpu and not self.shared else "gloo"
        self.res: dict = {"status": "starting"}  # filled section by section (the deadline dumps it)
        self.current = "init"

    # ------------------------------------------------------------------ helpers
    def sync(self):
        if self.on_gpu:
            self.torch.cuda.synchronize()

    def timeit(self, fn, iters: int, warmup: int = 3) -> float:
        """Median seconds per call (device-synchronised around each call)."""
        for _ in range(warmup):
            fn()
        self.sync()
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            self.sync()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2]

    def barrier(self):
        import torch.distributed as dist
        from ..parallel.comm import get_tp
        dist.barrier(group=get_tp().cpu_group)

    # ------------------------------------------------------------------ sections
    def collectives(self) -> dict:
        import torch.distributed as dist
        from ..parallel.comm import get_tp
        torch, n = self.torch, self.world
        st = get_tp()
        out = {"backend": self.backend, "all_reduce": [], "custom_all_reduce": []}
        # RCCL up to 256 MiB (prefill-sized all-reduces); gloo (CPU run, ranks sharing a GPU) small only
        sizes = [64 << 10, 1 << 20, 16 << 20, 256 << 20] if self.backend == "nccl" else [64 << 10, 1 << 20]
        for nbytes in sizes:
            x = torch.ones(nbytes // 2 if self.on_gpu else nbytes // 4, dtype=self.dtype, device=self.dev)
            t = self.timeit(lambda: dist.all_reduce(x, group=st.group), iters=10 if nbytes >= 16 << 20 else 30)
            out["all_reduce"].append({"bytes": nbytes, "us": round(t * 1e6, 1), "algbw_GBps": round(nbytes / t / 1e9, 2),
                                      "busbw_GBps": round(2 * (n - 1) / n * nbytes / t / 1e9, 2)})
            del x
        car = st.custom_ar
        if car is not None:
            for nbytes in (16 << 10, 256 << 10, 1 << 20, 8 << 20):
                x = torch.ones(nbytes // 2, dtype=torch.bfloat16, device=self.dev)
                if not car.should_use(x):
                    continue
                y = torch.empty_like(x)
                t = self.timeit(lambda: car.all_reduce(x, out=y), iters=50)
                ok = bool(car.check()) and bool((y == float(n)).all().item())
                out["custom_all_reduce"].append({"bytes": nbytes, "us": round(t * 1e6, 1),
                                                 "busbw_GBps": round(2 * (n - 1) / n * nbytes / t / 1e9, 2),
                                                 "correct": ok})
        return out

    def graph_collectives(self) -> dict:
        """The decode graphs' collectives, captured in a hipGraph and replayed with fresh inputs: the
        lm_head logits all-gather at a bucket above the IPC slot (RCCL inside the graph on a real
        node), a 1 MiB one (IPC all-to-all), and a 16 MiB RCCL all-reduce.  Each replay's result is
        checked against the rank-dependent fill."""
        from ..parallel.comm import collectives_capturable, get_tp, tp_all_gather
        import torch.distributed as dist
        torch, n = self.torch, self.world
        if not self.on_gpu:
            return {"skipped": "no GPU"}
        st = get_tp()
        out = {"backend": self.backend, "cases": []}
        cols = 16032  # Llama-3-70B vocab shard at TP 8
        for op, nbytes in (("all_gather", 1 << 20), ("all_gather", 16 << 20), ("all_reduce", 16 << 20)):
            case = {"op": op, "bytes": nbytes}
            if not collectives_capturable(nbytes):
                case["skipped"] = "not capturable on this group (gloo beyond the IPC slot)"
                out["cases"].append(case)
                continue
            rows = max(1, nbytes // 2 // (cols if op == "all_gather" else 4096))
            x = torch.zeros(rows, cols if op == "all_gather" else 4096, dtype=torch.bfloat16, device=self.dev)

            def body():
                if op == "all_gather":
                    return tp_all_gather(x, dim=-1)
                dist.all_reduce(x, group=st.group)
                return x

            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):  # warm-up outside the capture (communicator set-up)
                body()
            torch.cuda.current_stream().wait_stream(s)
            self.sync()
            self.barrier()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                y = body()
            ok = True
            for it in (1, 2, 3):
                x.fill_(float((self.rank + 1) * it))
                g.replay()
                self.sync()
                if op == "all_gather":
                    got = y.view(rows, n, cols)[0, :, :8].float().cpu()
                    want = torch.tensor([[(r + 1) * it] * 8 for r in range(n)], dtype=torch.float32)
                else:
                    got = y[0, :8].float().cpu()
                    want = torch.full((8,), float(it * n * (n + 1) // 2))
                ok = ok and bool(torch.equal(got, want))
            t = self.timeit(g.replay, iters=10)
            car = st.custom_ar
            # tp_all_gather pushes each peer one x-sized segment through the IPC all-to-all when it fits
            ipc = op == "all_gather" and car is not None and not car.disabled and x.numel() * 2 <= car.max_bytes
            case.update(correct=ok, replay_us=round(t * 1e6, 1),
                        path="ipc" if ipc else ("rccl" if self.backend == "nccl" else "gloo"))
            out["cases"].append(case)
            del g, x
        return out

    def _logits_and_time(self, model: str, full: dict, moe_dispatch: str, n_tok: int = 64):
        from ..models.config import get_model_config
        from ..models.llama import build_model
        torch = self.torch
        cfg = get_model_config(model)
        m = build_model(cfg, self.dev, self.dtype, moe_dispatch)
        m.load_full_state(full)
        ids = torch.randint(3, cfg.vocab_size, (n_tok,), generator=torch.Generator().manual_seed(2)).to(self.dev)
        kv = torch.zeros((n_tok + 15) // 16, cfg.num_layers, 2, m.nkv, 16, cfg.head_dim, dtype=self.dtype,
                         device=self.dev)
        md = _md(n_tok, self.dev)
        with torch.inference_mode():
            logits = m.compute_logits(m.forward(ids, md, kv)).float().cpu()
            t = self.timeit(lambda: m.forward(ids, md, kv), iters=10 if self.on_gpu else 3)
        del m, kv
        return logits, t

    def sharded_vs_full(self, model: str, moe_dispatch: str) -> dict:
        from ..models.config import get_model_config
        from ..models.weights import random_full_state
        from ..parallel import comm
        torch = self.torch
        cfg = get_model_config(model)
        full = random_full_state(cfg, seed=4, std=0.02, dtype=self.dtype, device=self.dev)
        got, t_n = self._logits_and_time(model, full, moe_dispatch)
        st = comm.get_tp()
        car_ok = st.custom_ar.check() if st.custom_ar is not None else None
        res = {"model": model, "ranks": self.world, "ms_64_tokens": round(t_n * 1e3, 3),
               "custom_all_reduce": st.custom_ar is not None, "custom_all_reduce_healthy": car_ok}
        ref = None
        if self.rank == 0:  # the same weights unsharded, in this process
            comm.set_tp(comm.ParallelState())
            try:
                ref, t_1 = self._logits_and_time(model, full, "allreduce")
            finally:
                comm.set_tp(st)
            res["ms_64_tokens_unsharded"] = round(t_1 * 1e3, 3)
            res["speedup_vs_unsharded"] = round(t_1 / t_n, 3)
        del full
        if self.on_gpu:
            torch.cuda.empty_cache()
        # every rank's logits to rank 0 (host tensors over the CPU group)
        import torch.distributed as dist
        parts = [None] * self.world
        dist.all_gather_object(parts, got.numpy(), group=st.cpu_group)
        if self.rank == 0:
            r = ref
            scale = float(r.abs().max())
            errs, agree = [], []
            for p in parts:
                g = torch.from_numpy(p)
                errs.append(float((g - r).abs().max()) / scale)
                agree.append(float((g.argmax(-1) == r.argmax(-1)).float().mean()))
            res["max_rel_err"] = round(max(errs), 5)
            res["argmax_agreement_min"] = round(min(agree), 4)
            res["ranks_consistent"] = all(bool((torch.from_numpy(p) == torch.from_numpy(parts[0])).all()) for p in parts)
        return res

    def tp_engine(self, model: str, moe_dispatch: str = "allreduce", batch: int = 64, isl: int = 512,
                  osl: int = 64) -> dict:
        from ..config import EngineArgs
        from ..engine.model_runner import ModelRunner
        from ..models.config import get_model_config
        torch = self.torch
        if not self.on_gpu:
            batch, isl, osl = 8, 48, 8
        blocks = batch * (-(-(isl + osl) // 16)) + 256
        args = EngineArgs(model=model, device="cuda" if self.on_gpu else "cpu", tensor_parallel_size=self.world,
                          max_num_seqs=batch, cuda_graph_max_bs=batch, max_model_len=isl + osl + 64,
                          num_gpu_blocks=blocks, cpu_num_blocks=blocks, load_format="random", seed=7,
                          moe_dispatch=moe_dispatch)
        if self.rank != 0:  # mirror rank 0's steps until it shuts the group down
            runner = ModelRunner(args, get_model_config(model))
            runner.follower_loop()
            runner.close()
            del runner
            if self.on_gpu:
                torch.cuda.empty_cache()
            return {}
        from ..engine.engine import LLMEngine
        from ..engine.request import SamplingParams
        t0 = time.perf_counter()
        eng = LLMEngine(args)
        t_build = time.perf_counter() - t0
        g = torch.Generator().manual_seed(3)
        vocab = eng.model_config.vocab_size
        sp = SamplingParams(max_tokens=osl, temperature=0.0, ignore_eos=True)
        for i in range(batch):
            eng.add_request(torch.randint(100, vocab - 100, (isl,), generator=g).tolist(), sp, request_id=f"tp{i}")
        steps = []  # (wall seconds since the previous step returned, outputs returned)
        t_prev = t_start = time.perf_counter()
        first_all = None
        seen = set()
        while eng.has_unfinished():
            outs = eng.step()
            now = time.perf_counter()
            steps.append((now - t_prev, len(outs)))
            t_prev = now
            seen.update(o.request_id for o in outs)
            if first_all is None and len(seen) == batch:
                first_all = now - t_start
        total = time.perf_counter() - t_start
        dec = sorted(dt for dt, n in steps if n == batch)
        res = {"model": model, "tp": self.world, "moe_dispatch": moe_dispatch, "batch": batch, "isl": isl, "osl": osl,
               "engine_build_s": round(t_build, 1), "graphs": sorted(eng.runner.graphs),
               "decode_steps": len(dec),
               "decode_step_ms_p50": round(1e3 * dec[len(dec) // 2], 3) if dec else None,
               "decode_tok_per_s": round(batch / dec[len(dec) // 2], 1) if dec else None,
               "prefill_tok_per_s": round(batch * isl / first_all, 1) if first_all else None,
               "total_s": round(total, 2)}
        st = eng.runner
        from ..parallel.comm import get_tp
        car = get_tp().custom_ar
        res["custom_all_reduce"] = car is not None and not car.disabled
        eng.close()
        del eng, st
        if self.on_gpu:
            torch.cuda.empty_cache()
        return res

    def disagg(self, model: str, qps_per_gpu: float, argv: list | None = None, raw: bool = False) -> dict:
        """bench.py's disaggregated phase on this probe group (each engine TP = 1).  `argv`: run it
        with exactly these bench.py arguments (the bench's own headline disagg phase, hosted here so
        that a fault on the cross-GPU KV path cannot take the bench's aggregated result with it);
        `raw`: return the per-rank stat rows for bench.py to summarize."""
        import torch.distributed as dist
        from ..parallel import comm
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        if root not in sys.path:
            sys.path.insert(0, root)
        import bench
        st = comm.get_tp()
        n = self.world
        if argv is None:
            if n % 2:
                return {"skipped": "needs an even number of ranks"}
            argv = ["--model", model, "--disagg-qps", str(qps_per_gpu), "--disagg-prefill-ranks", str(n // 2), "--steps", "60", "--warmup", "10", "--iters-per-step", "10",
                    "--max-warmup-s", "45", "--steady-window-s", "2.5", "--min-ttft-samples", "25",
                    "--device", "auto" if self.on_gpu else "cpu", "--disagg-max-num-seqs", "64",
                    "--num-gpu-blocks", "40000"]
            if not self.on_gpu:
                argv += ["--steps", "12", "--warmup", "8", "--iters-per-step", "1", "--max-warmup-s", "8", "--steady-window-s", "1",
                         "--min-ttft-samples", "5", "--disagg-qps", "4"]
        a = bench.parse(argv)
        p = bench.disagg_plan(a, n)[0]
        probe = self
        pg_decode = dist.new_group(list(range(p, n)), backend="gloo")

        class Ctx(bench.Ctx):  # the probe's process group instead of a new one; control over gloo
            def __init__(self):
                self.torch, self.dist = probe.torch, dist
                self.world, self.rank, self.local = n, probe.rank, probe.local
                self.on_gpu, self.ndev, self.shared_gpu = probe.on_gpu, probe.ndev, probe.shared
                self.pg_decode = pg_decode
                self.sync = probe.sync

            def barrier(self):
                dist.barrier(group=st.cpu_group)
                self.sync()

            def gather(self, vals):
                import numpy as np
                t = probe.torch.tensor(vals, dtype=probe.torch.float64)
                parts = [probe.torch.zeros_like(t) for _ in range(n)]
                dist.all_gather(parts, t, group=st.cpu_group)
                return np.stack([p.numpy() for p in parts])

        comm.set_tp(comm.ParallelState())  # every engine here is TP = 1
        try:
            col, info = bench.phase_disagg(a, Ctx())
        finally:
            comm.set_tp(st)
        if raw:
            return {"col": col.tolist(), "info": info}
        res = bench.summarize(col, a.steps, list(range(p, n)))
        res.update(info, model=model, parallelism=f"disagg {p}P+{n - p}D")
        return res

    def tp_layer(self) -> dict:
        """Llama-3-70B decode layer of one TP shard at this world size (mxserve/tools/tp_layer_bench.py):
        tuned shard GEMMs + the fused all-reduce / residual-add / RMSNorm epilogues, the chain captured
        in a hipGraph on every rank against the weight-streaming floor.  A real node only: ranks that
        share a GPU are time-sliced by the command processor, so their collectives measure nothing."""
        if not self.on_gpu:
            return {"skipped": "no GPU"}
        if self.shared:
            return {"skipped": "ranks share a GPU (time-sliced collectives); see profiles/r4/tp"}
        from . import tp_layer_bench
        return tp_layer_bench.run((1, 8, 64), shared=False, barrier=self.barrier, log=lambda s: None) or {}

    def p2p(self) -> dict:
        torch = self.torch
        if not self.on_gpu or self.ndev < 2 or self.rank != 0:
            return {"skipped": "needs >= 2 visible GPUs (rank 0 only)"}
        nbytes = 256 << 20
        src = torch.empty(nbytes, dtype=torch.uint8, device=self.dev)
        peers = [d for d in range(min(self.ndev, 8)) if d != self.dev.index]
        dsts = {d: torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{d}") for d in peers}
        out = {"bytes": nbytes, "per_peer_GBps": {}}
        for d in peers:
            t = self.timeit(lambda: dsts[d].copy_(src, non_blocking=True), iters=5, warmup=2)
            out["per_peer_GBps"][str(d)] = round(nbytes / t / 1e9, 1)
        streams = {d: torch.cuda.Stream(device=self.dev) for d in peers}

        def all_at_once():
            for d in peers:
                with torch.cuda.stream(streams[d]):
                    dsts[d].copy_(src, non_blocking=True)
            for d in peers:
                streams[d].synchronize()
        t = self.timeit(all_at_once, iters=5, warmup=2)
        out["all_peers_GBps"] = round(len(peers) * nbytes / t / 1e9, 1)
        del dsts, src
        torch.cuda.empty_cache()
        return out

    # ------------------------------------------------------------------ main
    # Wall seconds a section needs to finish on an MI355X node (the r2 2-rank run took 0.2-41 s per
    # section; engines of the 70B / Mixtral shapes dominate): a section starts only if the deadline
    # leaves it this much.  CPU plumbing runs use the small number.
    SECTION_COST_S = {"collectives": 20, "graph_collectives": 15, "tp": 40, "ep": 40, "p2p": 15, "tp_engine": 120, "ep_engine": 120,
                      "disagg_8b": 90}

    def section_fits(self, name: str, t_sections: float, deadline: float, cap: float) -> str:
        """'' if the section may start, else why not.  Rank 0's clock decides for every rank (the
        sections run collectives, so all ranks must agree on which ones start)."""
        import torch.distributed as dist
        from ..parallel.comm import get_tp
        why = ""
        need = self.SECTION_COST_S.get(name, 30) if self.on_gpu else 5
        if deadline and time.time() + need > deadline:
            why = f"run deadline: {deadline - time.time():.0f}s left, the section needs ~{need}s"
        elif cap > 0 and time.perf_counter() - t_sections > 0.6 * cap:
            why = f"probe wall budget of {cap:.0f}s spent"
        box = [why]
        dist.broadcast_object_list(box, src=0, group=get_tp().cpu_group)
        return box[0]

    def run(self) -> dict:
        from ..parallel.comm import init_distributed
        if self.on_gpu:
            self.torch.cuda.set_device(self.dev)
        # a collective some rank never joins (a section failed on one rank only) raises instead of
        # waiting gloo's default 30 min
        init_distributed(self.world, backend=self.backend, device=self.dev if self.on_gpu else None,
                         timeout_s=float(os.environ.get("MXS_PROBE_PG_TIMEOUT_S", "180")))
        res = self.res
        res.update(status="ok", ranks=self.world, backend=self.backend, shared_gpu=self.shared)
        tp_model = MODEL_TP if self.on_gpu else "tiny-llama"
        ep_model = MODEL_EP if self.on_gpu else "tiny-mixtral"
        # cheapest and most informative first: a run short of time still measures the collectives
        # and the sharded-vs-unsharded parity before the engine-sized sections
        sections = [("collectives", self.collectives),
                    ("graph_collectives", self.graph_collectives),
                    ("tp", lambda: self.sharded_vs_full(tp_model, "allreduce")),
                    ("ep", lambda: self.sharded_vs_full(ep_model, "a2a")),
                    ("p2p", self.p2p),
                    ("tp_layer", self.tp_layer),
                    ("tp_engine", lambda: self.tp_engine(MODEL_TP_ENGINE if self.on_gpu else "tiny-llama")),
                    ("ep_engine", lambda: self.tp_engine(MODEL_EP_ENGINE if self.on_gpu else "tiny-mixtral", "a2a")),
                    ("disagg_8b", lambda: self.disagg(MODEL_DISAGG if self.on_gpu else "tiny-llama", 2.0))]
        from ..models.config import get_model_config
        only = [x for x in os.environ.get("MXS_PROBE_SECTIONS", "").split(",") if x]
        if only:  # a subset (GPU tests)
            sections = [(nm, fn) for nm, fn in sections if nm in only]
        headline = os.environ.get("MXS_PROBE_DISAGG_ARGV")
        if headline:  # bench.py's own disagg phase first, outside the optional sections' cap
            argv = json.loads(headline)
            sections.insert(0, ("disagg_headline", lambda: self.disagg("", 0.0, argv=argv, raw=True)))
        deadline = float(os.environ.get("MXS_PROBE_DEADLINE", "0"))  # absolute (time.time()); 0: none
        cap = float(os.environ.get("MXS_PROBE_TIMEOUT_S", os.environ.get("MXS_PROBE_BUDGET_S", "0")))
        if os.environ.get("MXS_PROBE_BUDGET_S"):  # a direct cap on the optional sections (tests)
            cap = float(os.environ["MXS_PROBE_BUDGET_S"]) / 0.6
        t_start = time.perf_counter()
        for name, fn in sections:
            self.current = name
            why = "" if name == "disagg_headline" else self.section_fits(name, t_start, deadline, cap)
            if why:
                res[name] = {"skipped": why}
                continue
            if name in ("ep", "ep_engine") and get_model_config(ep_model).num_experts % self.world:
                res[name] = {"skipped": f"{self.world} ranks do not divide the experts"}
                continue
            if name in ("tp", "tp_engine") and get_model_config(tp_model).num_heads % self.world:
                res[name] = {"skipped": f"{self.world} ranks do not divide the attention heads"}
                continue
            t0 = time.perf_counter()
            if os.environ.get("MXS_PROBE_FAULT") == f"hang:{name}":  # tests: a section that never returns
                while True:
                    time.sleep(1.0)
            try:
                res[name] = fn()
            except Exception as e:  # noqa: BLE001 - report, keep the other sections
                traceback.print_exc()
                tb = traceback.extract_tb(e.__traceback__)
                res[name] = {"status": "failed", "error": repr(e)[:300], "rank": self.rank,
                             "where": [f"{os.path.basename(f.filename)}:{f.lineno} {f.name}" for f in tb[-4:]]}
            if isinstance(res[name], dict):
                res[name]["wall_s"] = round(time.perf_counter() - t0, 1)
            try:
                self.barrier()
            except Exception as e:  # noqa: BLE001 - a rank lost in that section: keep what was measured
                traceback.print_exc()
                res["aborted_after"] = {"section": name, "error": repr(e)[:200]}
                break
            if name == "disagg_headline":  # the optional sections' cap starts after it
                t_start = time.perf_counter()
        self.current = "done"
        return res


_EMIT_LOCK = None
_EMITTED = []
_DETACHED = False


def _emit(result_out, res: dict) -> None:
    """Write the one `PROBE {json}` line (the deadline watchdog and the main thread race for it)."""
    with _EMIT_LOCK:
        if _EMITTED:
            return
        _EMITTED.append(True)
        try:
            result_out.write("PROBE " + json.dumps(res, default=str) + "\n")
            result_out.flush()
        except (OSError, ValueError):
            pass


def _watch(result_out, probe_box: list, t0: float) -> None:
    """The probe's own deadline (bench.py hands it MXS_PROBE_DEADLINE) and parent watch: at the
    deadline rank 0 reports the sections finished so far and names the one that did not; every rank
    exits.  If the bench rank that started this probe dies, the probe exits at once."""
    import threading
    global _EMIT_LOCK
    _EMIT_LOCK = threading.Lock()
    deadline = float(os.environ.get("MXS_PROBE_DEADLINE", "0"))
    ppid = os.getppid()

    def loop():
        while True:
            time.sleep(0.5)
            if os.getppid() != ppid and not _DETACHED:  # a detached probe outlives its bench rank
                os._exit(1)
            if deadline and time.time() > deadline:
                break
        p = probe_box[0] if probe_box else None
        rank = int(os.environ.get("RANK", "0"))
        print(f"mgpu_probe rank {rank}: deadline reached in section {getattr(p, 'current', 'init')!r}",
              file=sys.stderr, flush=True)
        if rank == 0:
            res = dict(p.res) if p is not None else {}
            res.update(status="partial", timed_out_section=getattr(p, "current", "init"),
                       wall_s=round(time.perf_counter() - t0, 1))
            _emit(result_out, res)
        sys.stderr.flush()
        os._exit(0)
    threading.Thread(target=loop, daemon=True, name="probe-deadline").start()


def main() -> int:
    # keep this process's stdout for the result line only: library chatter goes to stderr
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    sys.stdout = sys.stderr
    box: list = []
    t0 = time.perf_counter()
    _watch(result_out, box, t0)
    line = sys.stdin.readline().split()
    if not line or line[0] != "go":  # the bench rank ended (or failed) before its serving phases finished
        return 0
    if len(line) > 1:  # the rendezvous port rank 0's bench process picked
        os.environ["MASTER_PORT"] = line[1]
    if "detach" in line[2:]:  # bench ranks > 0 leave once they have released their probe
        global _DETACHED
        _DETACHED = True
    t0 = time.perf_counter()
    try:
        p = Probe()
        box.append(p)
        res = p.run()
        res["wall_s"] = round(time.perf_counter() - t0, 1)
        if p.rank == 0:
            _emit(result_out, res)
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        traceback.print_exc()
        _emit(result_out, {"status": "failed", "error": repr(e)[:300]})
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
