"""Prometheus metrics with the exact names/labels the reference's Grafana dashboard queries
(examples/dgdr/trtllm/grafana-dynamo-dashboard-configmap.yaml:121-512):
  dynamo_frontend_requests_total{model,request_type,status}
  dynamo_frontend_{time_to_first_token,inter_token_latency,request_duration}_seconds{model}
  dynamo_frontend_{input,output}_sequence_tokens{model}
plus inflight / queued gauges and worker-side dynamo_component_* KV stats."""
from __future__ import annotations

import os

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

_LAT = (0.001, 0.0025, 0.005, 0.0075, 0.01, 0.015, 0.02, 0.025, 0.035, 0.05, 0.075, 0.1, 0.15, 0.25, 0.35, 0.5,
        0.75, 1.0, 1.5, 2.0, 3.0, 5.0, 10.0, 30.0)
_DUR = (0.05, 0.1, 0.25, 0.5, 1.0, 2.0, 4.0, 8.0, 15.0, 30.0, 60.0, 120.0, 300.0)
_TOK = (1, 8, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 131072)


def _multiproc() -> bool:
    """prometheus_client multiprocess mode (a multi-process frontend, frontend/multiproc.py)."""
    return bool(os.environ.get("PROMETHEUS_MULTIPROC_DIR"))


class FrontendMetrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        mp = _multiproc()
        sum_kw = {"multiprocess_mode": "livesum"} if mp else {}
        max_kw = {"multiprocess_mode": "livemax"} if mp else {}
        self.requests = Counter("dynamo_frontend_requests", "Frontend requests",
                                ["model", "endpoint", "request_type", "status"], registry=r)
        self.inflight = Gauge("dynamo_frontend_inflight_requests", "In-flight requests", ["model"], registry=r,
                              **sum_kw)
        self.queued = Gauge("dynamo_frontend_queued_requests", "Requests waiting for first token", ["model"],
                            registry=r, **sum_kw)
        self.ttft = Histogram("dynamo_frontend_time_to_first_token_seconds", "TTFT", ["model"], buckets=_LAT,
                              registry=r)
        self.itl = Histogram("dynamo_frontend_inter_token_latency_seconds", "ITL", ["model"], buckets=_LAT,
                             registry=r)
        self.duration = Histogram("dynamo_frontend_request_duration_seconds", "Request duration", ["model"],
                                  buckets=_DUR, registry=r)
        self.isl = Histogram("dynamo_frontend_input_sequence_tokens", "ISL", ["model"], buckets=_TOK, registry=r)
        self.osl = Histogram("dynamo_frontend_output_sequence_tokens", "OSL", ["model"], buckets=_TOK, registry=r)
        # every process sees every worker: the max over processes, not the sum
        self.workers = Gauge("dynamo_frontend_workers", "Registered workers", ["model", "role"], registry=r, **max_kw)
        self.kv_hit = Counter("dynamo_frontend_kv_router_overlap_blocks", "Prefix blocks matched by the KV router",
                              ["model"], registry=r)
        self.migrations = Counter("dynamo_frontend_request_migrations", "Streams moved to another worker mid-request",
                                  ["model"], registry=r)
        # why each streamed response ended: ok | client_gone | api_error_<status> | error_<exception type>
        self.stream_close = Counter("dynamo_frontend_stream_close", "Streamed responses by close reason",
                                    ["model", "reason"], registry=r)

    def render(self) -> bytes:
        if _multiproc():
            from prometheus_client import multiprocess
            reg = CollectorRegistry()
            multiprocess.MultiProcessCollector(reg)
            return generate_latest(reg)
        return generate_latest(self.registry)


class WorkerMetrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.kv_active = Gauge("dynamo_component_kv_active_blocks", "KV blocks in use", ["model"], registry=r)
        self.kv_total = Gauge("dynamo_component_kv_total_blocks", "KV blocks in the pool", ["model"], registry=r)
        self.kv_usage = Gauge("dynamo_component_gpu_cache_usage_percent", "KV cache usage %", ["model"], registry=r)
        self.hit_rate = Gauge("dynamo_component_gpu_prefix_cache_hit_rate", "Prefix cache hit rate", ["model"],
                              registry=r)
        self.running = Gauge("dynamo_component_num_requests_running", "Running requests", ["model"], registry=r)
        self.waiting = Gauge("dynamo_component_num_requests_waiting", "Waiting requests", ["model"], registry=r)
        self.gen_tokens = Counter("dynamo_component_generation_tokens", "Generated tokens", ["model"], registry=r)
        self.kv_xfer_bytes = Counter("dynamo_component_kv_transfer_bytes", "KV bytes moved P->D", ["model", "backend"],
                                     registry=r)
        self.kv_xfer_lat = Histogram("dynamo_component_kv_transfer_seconds", "KV transfer latency", ["model"],
                                     buckets=_LAT, registry=r)
        # TP steps discarded and recomputed because a custom all-reduce wait ran out (engine.py
        # _recover_collective_fault); any increase is worth an alert
        self.car_timeouts = Counter("dynamo_component_custom_ar_timeouts", "Custom all-reduce faults recovered",
                                    ["model"], registry=r)
        self._car_seen: dict = {}

    def update(self, model: str, stats: dict) -> None:
        tot = stats.get("kv_total_blocks", 0)
        free = stats.get("kv_free_blocks", 0)
        self.kv_total.labels(model).set(tot)
        self.kv_active.labels(model).set(tot - free)
        self.kv_usage.labels(model).set(100.0 * stats.get("kv_usage", 0.0))
        self.hit_rate.labels(model).set(stats.get("prefix_hit_rate", 0.0))
        self.running.labels(model).set(stats.get("num_running", 0))
        self.waiting.labels(model).set(stats.get("num_waiting", 0))
        n = int(stats.get("custom_ar_timeouts", 0))
        self.car_timeouts.labels(model).inc(max(0, n - self._car_seen.get(model, 0)))
        self._car_seen[model] = max(n, self._car_seen.get(model, 0))

    def render(self) -> bytes:
        return generate_latest(self.registry)
