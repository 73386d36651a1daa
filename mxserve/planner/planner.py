"""SLA planner: scales a running graph's prefill / decode (or aggregated) worker replicas from live
load (the Dynamo planner the reference's DGDR flow can deploy as a
`componentType: planner` service).

Every `interval` seconds it scrapes the frontend's Prometheus endpoint, turns counter deltas into
the window's request rate, mean ISL / OSL, mean TTFT and ITL, and decides replica counts:

  predictive  replicas = ceil(rate / per-replica capacity / target utilisation), with per-replica
              capacities from the MI355X roofline of mxserve.profiler.sla at the observed ISL/OSL
              (prefill: 1 / TTFT requests/s; decode: the largest batch meeting the ITL target, so
              batch / (OSL x ITL) requests/s; aggregated: both on one replica);
  reactive    a window whose mean TTFT (ITL) breaks the SLA adds a prefill (decode) replica even if
              the prediction says otherwise -- the roofline is an estimate;
  limits      at least 1 replica per role, total GPUs within the node, scale-down only after
              `cooldown` seconds without a scale-up (no flapping).

The decision is applied as a merge patch of spec.services.<name>.replicas on the DGD; the operator
reconciles the Deployments.  `--dry-run` only logs.
"""
from __future__ import annotations

import argparse
import os
import logging
import math
import re
import time
from dataclasses import dataclass
from typing import Callable, Optional

from ..models.config import get_model_config
from ..profiler import sla

log = logging.getLogger(__name__)

DGD_KIND = "DynamoGraphDeployment"
_SAMPLE = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{[^}]*\})?\s+([-+0-9.eEinfINFaN]+)$')


def parse_prometheus(text: str) -> dict[str, float]:
    """Sum every sample of a metric over its label sets: {name: total}."""
    out: dict[str, float] = {}
    for line in text.splitlines():
        if not line or line[0] == "#":
            continue
        m = _SAMPLE.match(line.strip())
        if m:
            out[m.group(1)] = out.get(m.group(1), 0.0) + float(m.group(3))
    return out


@dataclass
class Window:
    seconds: float
    rps: float
    isl: float
    osl: float
    ttft_ms: Optional[float]
    itl_ms: Optional[float]


@dataclass
class PlannerConfig:
    namespace: str
    dgd: str
    model: str
    ttft_ms: float = 600.0
    itl_ms: float = 25.0
    interval_s: float = 30.0
    cooldown_s: float = 180.0
    target_util: float = 0.7
    max_gpus: int = 8
    system: str = "mi355x"
    default_isl: int = 4000
    default_osl: int = 500
    dry_run: bool = False


@dataclass
class Role:
    key: str  # DGD service name
    kind: str  # "prefill" | "decode" | "agg"
    replicas: int
    gpus: int  # per replica (TP degree)


class Planner:
    def __init__(self, cfg: PlannerConfig, kube, scrape: Callable[[], dict[str, float]],
                 clock: Callable[[], float] = time.monotonic):
        self.cfg = cfg
        self.kube = kube
        self.scrape = scrape
        self.clock = clock
        self.model = get_model_config(cfg.model)
        self.sys = sla.SYSTEMS.get(cfg.system, sla.SYSTEMS["mi355x"])
        self._prev: Optional[tuple[float, dict]] = None
        self._last_up = -1e18
        self.history: list = []

    # ------------------------------------------------------------------ observe
    def observe(self) -> Optional[Window]:
        now, cur = self.clock(), self.scrape()
        prev, self._prev = self._prev, (now, cur)
        if prev is None:
            return None
        dt = max(1e-6, now - prev[0])

        def d(name):
            return cur.get(name, 0.0) - prev[1].get(name, 0.0)

        n = d("dynamo_frontend_requests_total")
        nin = d("dynamo_frontend_input_sequence_tokens_count")
        nout = d("dynamo_frontend_output_sequence_tokens_count")
        nt = d("dynamo_frontend_time_to_first_token_seconds_count")
        ni = d("dynamo_frontend_inter_token_latency_seconds_count")
        return Window(
            seconds=dt, rps=max(0.0, n) / dt,
            isl=d("dynamo_frontend_input_sequence_tokens_sum") / nin if nin > 0 else self.cfg.default_isl,
            osl=d("dynamo_frontend_output_sequence_tokens_sum") / nout if nout > 0 else self.cfg.default_osl,
            ttft_ms=1e3 * d("dynamo_frontend_time_to_first_token_seconds_sum") / nt if nt > 0 else None,
            itl_ms=1e3 * d("dynamo_frontend_inter_token_latency_seconds_sum") / ni if ni > 0 else None)

    # ------------------------------------------------------------------ decide
    def roles(self) -> list[Role]:
        dgd = self.kube.get(DGD_KIND, self.cfg.dgd, self.cfg.namespace)
        if dgd is None:
            raise LookupError(f"DGD {self.cfg.namespace}/{self.cfg.dgd} not found")
        out = []
        for key, s in (dgd.get("spec", {}).get("services") or {}).items():
            if s.get("componentType") != "worker":
                continue
            gpus = int(((s.get("resources") or {}).get("limits") or {}).get("gpu", 1) or 1)
            out.append(Role(key, s.get("subComponentType") or "agg", int(s.get("replicas", 1)), gpus))
        return out

    def capacity(self, kind: str, tp: int, isl: float, osl: float) -> float:
        """Requests/s one replica sustains at the SLA: the per-GPU role capacities the DGDR profiler
        and bench.py plan with (profiler/capacity.py: measured MI355X table, else roofline), scaled
        to the replica's TP degree by the roofline's own ratio."""
        from ..profiler import capacity as capm
        c, s = self.model, self.sys
        isl, osl = max(1, int(isl)), max(1, int(osl))
        cap = capm.capacity(c.name, isl, osl, self.cfg.itl_ms, s.name)
        ctx = isl + osl // 2

        def dec_model(t):
            b = sla.max_decode_batch(c, s, ctx, t, self.cfg.itl_ms / 1e3)
            return b / (osl * sla.decode_itl(c, s, max(1, b), ctx, t)) if b else 0.0
        pre = cap["prefill_rps"] * sla.prefill_latency(c, s, isl, 1) / sla.prefill_latency(c, s, isl, tp)
        d1 = dec_model(1)
        dec = cap["decode_rps"] * dec_model(tp) / d1 if d1 > 0 else dec_model(tp)
        if kind == "prefill":
            return pre
        if kind == "decode":
            return dec
        # agg: one replica does both halves of every request
        return 1.0 / (1.0 / dec + 1.0 / pre) if dec > 0 else pre / 10

    def decide(self, w: Window, roles: list[Role]) -> dict[str, int]:
        cfg = self.cfg
        want = {}
        for r in roles:
            cap = max(1e-9, self.capacity(r.kind, r.gpus, w.isl, w.osl))
            n = math.ceil(w.rps / (cap * cfg.target_util)) if w.rps > 0 else 1
            late_ttft = w.ttft_ms is not None and w.ttft_ms > cfg.ttft_ms
            late_itl = w.itl_ms is not None and w.itl_ms > cfg.itl_ms
            if (r.kind in ("prefill", "agg") and late_ttft) or (r.kind in ("decode", "agg") and late_itl):
                n = max(n, r.replicas + 1)
            want[r.key] = max(1, n)
        # node budget: trim the role with the most headroom first
        by_key = {r.key: r for r in roles}
        while sum(want[k] * by_key[k].gpus for k in want) > cfg.max_gpus:
            k = max((k for k in want if want[k] > 1), key=lambda k: want[k] * by_key[k].gpus, default=None)
            if k is None:
                break
            want[k] -= 1
        # scale-down hysteresis
        now = self.clock()
        if any(want[r.key] > r.replicas for r in roles):
            self._last_up = now
        if now - self._last_up < cfg.cooldown_s:
            for r in roles:
                want[r.key] = max(want[r.key], r.replicas)
        return want

    # ------------------------------------------------------------------ act
    def step(self) -> Optional[dict]:
        w = self.observe()
        if w is None:
            return None
        roles = self.roles()
        want = self.decide(w, roles)
        changes = {r.key: want[r.key] for r in roles if want[r.key] != r.replicas}
        rec = {"window": w.__dict__, "replicas": {r.key: r.replicas for r in roles}, "changes": changes}
        self.history.append(rec)
        if changes:
            log.info("planner: %s (rps %.2f, ttft %s ms, itl %s ms)", changes, w.rps, w.ttft_ms, w.itl_ms)
            if not self.cfg.dry_run:
                patch = {"spec": {"services": {k: {"replicas": v} for k, v in changes.items()}}}
                self.kube.merge_patch(DGD_KIND, self.cfg.dgd, self.cfg.namespace, patch)
        return rec

    def run(self, stop: Callable[[], bool] = lambda: False) -> None:
        while not stop():
            try:
                self.step()
            except Exception:  # noqa: BLE001 - keep planning through transient API errors
                log.exception("planner step failed")
            time.sleep(self.cfg.interval_s)


def http_scraper(url: str) -> Callable[[], dict[str, float]]:
    import httpx

    def scrape():
        return parse_prometheus(httpx.get(url.rstrip("/") + "/metrics", timeout=10).text)
    return scrape


PLANNER_METRICS = ("dynamo_frontend_requests_total", "dynamo_frontend_input_sequence_tokens_count",
                   "dynamo_frontend_input_sequence_tokens_sum", "dynamo_frontend_output_sequence_tokens_count",
                   "dynamo_frontend_output_sequence_tokens_sum", "dynamo_frontend_time_to_first_token_seconds_count",
                   "dynamo_frontend_time_to_first_token_seconds_sum",
                   "dynamo_frontend_inter_token_latency_seconds_count",
                   "dynamo_frontend_inter_token_latency_seconds_sum")


def prometheus_scraper(endpoint: str, namespace: str) -> Callable[[], dict[str, float]]:
    """Counters of the frontend(s) of `namespace` through the Prometheus HTTP API -- the endpoint
    the platform installer hands over (PROMETHEUS_ENDPOINT; install-dynamo-1node.sh in the
    reference passes it to the platform chart as prometheusEndpoint, :214-218).  Same {name: total}
    shape as http_scraper, summed over every frontend replica Prometheus scrapes."""
    import httpx
    names = "|".join(PLANNER_METRICS)
    query = f'sum by (__name__) ({{__name__=~"{names}", namespace="{namespace}"}})'

    def scrape():
        r = httpx.get(endpoint.rstrip("/") + "/api/v1/query", params={"query": query}, timeout=10)
        r.raise_for_status()
        d = r.json()
        if d.get("status") != "success":
            raise RuntimeError(f"prometheus query failed: {d}")
        return {res["metric"]["__name__"]: float(res["value"][1]) for res in d["data"]["result"]}
    return scrape


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="mxserve SLA planner")
    ap.add_argument("--namespace", required=True)
    ap.add_argument("--dgd", required=True)
    ap.add_argument("--model", required=True)
    ap.add_argument("--frontend-url", default=None, help="scrape this frontend's /metrics directly")
    ap.add_argument("--prometheus-endpoint", default=os.environ.get("PROMETHEUS_ENDPOINT"),
                    help="query Prometheus instead (every frontend replica of the namespace)")
    ap.add_argument("--ttft", type=float, default=600.0, help="ms")
    ap.add_argument("--itl", type=float, default=25.0, help="ms")
    ap.add_argument("--interval", type=float, default=30.0)
    ap.add_argument("--cooldown", type=float, default=180.0)
    ap.add_argument("--max-gpus", type=int, default=8)
    ap.add_argument("--server", default=None)
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    from ..utils.logs import setup_logging
    setup_logging()
    from ..k8s.client import KubeClient
    cfg = PlannerConfig(namespace=a.namespace, dgd=a.dgd, model=a.model, ttft_ms=a.ttft, itl_ms=a.itl,
                        interval_s=a.interval, cooldown_s=a.cooldown, max_gpus=a.max_gpus, dry_run=a.dry_run)
    if a.frontend_url:
        scrape = http_scraper(a.frontend_url)
    elif a.prometheus_endpoint:
        scrape = prometheus_scraper(a.prometheus_endpoint, a.namespace)
    else:
        ap.error("one of --frontend-url / --prometheus-endpoint (or PROMETHEUS_ENDPOINT) is required")
    Planner(cfg, KubeClient(a.server), scrape).run()
