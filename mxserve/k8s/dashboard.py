"""Grafana dashboard for an mxserve deployment, emitted as the sidecar-discovered ConfigMap
(R17, reference examples/dgdr/trtllm/grafana-dynamo-dashboard-configmap.yaml:1-20: ConfigMap in
`monitoring`, label grafana_dashboard: "1").

Same panel set as the reference dashboard -- frontend RPS / TTFT / ITL / request duration / ISL-OSL,
GPU utilisation + power, node CPU + load, container CPU, pod memory -- with the GPU panels reading
the AMD device-metrics-exporter series (deployed by the AMD GPU Operator) instead of DCGM, plus the
worker-side series this stack exports (KV-cache usage, running / waiting requests, prefix-cache hit
rate, P->D KV transfer latency).

  python -m mxserve.k8s.dashboard > examples/dgdr/trtllm/grafana-dynamo-dashboard-configmap.yaml
"""
from __future__ import annotations

import json
import sys

import yaml

NS = 'namespace=~"$namespace"'
# the reference ConfigMap's contract (grafana-dynamo-dashboard-configmap.yaml:12,1006): anything
# provisioned or bookmarked against the reference dashboard keeps working
UID = "dynamo-dashboard"
DATA_KEY = "dynamo-dashboard.json"
# reference DCGM series -> the AMD device-metrics-exporter gauge plotted in their place
DCGM_TO_AMD = {"DCGM_FI_DEV_GPU_UTIL": "gpu_gfx_activity", "DCGM_FI_DEV_POWER_USAGE": "gpu_power_usage"}


def _ratio(metric: str, scale: str = "1000*") -> str:
    return f"{scale}(rate({metric}_sum{{{NS}}}[1m]) / rate({metric}_count{{{NS}}}[1m]))"


# (title, unit, [(expr, legend)])
PANELS = [
    # the reference's split: one series per (request_type = stream | unary, status), every label kept
    ("Frontend Requests / Sec", "reqps",
     [(f"rate(dynamo_frontend_requests_total{{{NS}}}[1m])", "{{request_type}}, {{status}},")]),
    ("Frontend Avg Time to First Token", "ms",
     [(_ratio("dynamo_frontend_time_to_first_token_seconds"), "{{model}}")]),
    ("Frontend Avg Inter-Token Latency", "ms",
     [(_ratio("dynamo_frontend_inter_token_latency_seconds"), "{{model}}")]),
    ("Frontend Avg Request Duration", "ms",
     [(_ratio("dynamo_frontend_request_duration_seconds"), "{{model}}")]),
    ("Frontend Avg Input/Output Sequence Length", "short",
     [(_ratio("dynamo_frontend_input_sequence_tokens", ""), "ISL {{model}}"),
      (_ratio("dynamo_frontend_output_sequence_tokens", ""), "OSL {{model}}")]),
    ("Frontend Inflight / Queued Requests", "short",
     [(f"sum by (model) (dynamo_frontend_inflight_requests{{{NS}}})", "inflight {{model}}"),
      (f"sum by (model) (dynamo_frontend_queued_requests{{{NS}}})", "queued {{model}}")]),
    ("Worker KV-Cache Usage", "percent",
     [(f"dynamo_component_gpu_cache_usage_percent{{{NS}}}", "{{pod}}")]),
    ("Worker Running / Waiting Requests", "short",
     [(f"dynamo_component_num_requests_running{{{NS}}}", "running {{pod}}"),
      (f"dynamo_component_num_requests_waiting{{{NS}}}", "waiting {{pod}}")]),
    ("Worker Output Tokens / Sec", "short",
     [(f"sum by (pod) (rate(dynamo_component_generation_tokens_total{{{NS}}}[1m]))", "{{pod}}")]),
    ("Prefix-Cache Hit Rate / KV-Router Overlap", "short",
     [(f"dynamo_component_gpu_prefix_cache_hit_rate{{{NS}}}", "hit rate {{pod}}"),
      (f"rate(dynamo_frontend_kv_router_overlap_blocks_total{{{NS}}}[1m])", "overlap blocks/s {{model}}")]),
    ("Disaggregated KV Transfer (P->D)", "ms",
     [(_ratio("dynamo_component_kv_transfer_seconds"), "avg latency {{pod}}"),
      (f"rate(dynamo_component_kv_transfer_bytes_total{{{NS}}}[1m]) / 1e9", "GB/s {{pod}}")]),
    ("AMD GPU Utilization & Power", "short",
     [("gpu_gfx_activity", "util % gpu{{gpu_id}}"), ("gpu_power_usage", "power W gpu{{gpu_id}}")]),
    ("AMD GPU Memory (HBM3E)", "decbytes",
     [("gpu_used_vram", "used gpu{{gpu_id}}"), ("gpu_total_vram", "total gpu{{gpu_id}}")]),
    ("Node CPU Utilization & Load", "short",
     [('100 - (avg by (instance) (rate(node_cpu_seconds_total{mode="idle"}[5m])) * 100)', "cpu % {{instance}}"),
      ("node_load1", "load1 {{instance}}"), ("node_load5", "load5 {{instance}}")]),
    ("Container CPU Usage", "short",
     [(f'sum by (pod) (rate(container_cpu_usage_seconds_total{{{NS}, container!=""}}[5m]))', "{{pod}}")]),
    ("Memory Usage per Pod", "bytes",
     [(f'sum by (pod) (container_memory_working_set_bytes{{{NS}, container!=""}})', "{{pod}}")]),
]


def dashboard() -> dict:
    panels = []
    for i, (title, unit, targets) in enumerate(PANELS):
        panels.append({
            "id": i + 1, "type": "timeseries", "title": title,
            "datasource": {"type": "prometheus", "uid": "${datasource}"},
            "gridPos": {"h": 8, "w": 12, "x": 12 * (i % 2), "y": 8 * (i // 2)},
            "fieldConfig": {"defaults": {"unit": unit, "custom": {"lineWidth": 1, "fillOpacity": 10}},
                            "overrides": []},
            "options": {"legend": {"displayMode": "list", "placement": "bottom"},
                        "tooltip": {"mode": "multi"}},
            "targets": [{"refId": chr(65 + j), "expr": e, "legendFormat": lg, "range": True}
                        for j, (e, lg) in enumerate(targets)],
        })
    return {
        "title": "Dynamo Dashboard (MI355X)", "uid": UID, "schemaVersion": 39, "version": 1,
        "editable": True, "refresh": "10s", "time": {"from": "now-30m", "to": "now"}, "tags": ["mxserve", "dynamo"],
        "templating": {"list": [
            {"name": "datasource", "type": "datasource", "query": "prometheus", "current": {}},
            {"name": "namespace", "type": "query", "datasource": {"type": "prometheus", "uid": "${datasource}"},
             "query": "label_values(dynamo_frontend_requests_total, namespace)", "includeAll": True,
             "multi": True, "current": {"text": "All", "value": "$__all"}, "refresh": 2},
        ]},
        "panels": panels,
    }


def configmap(namespace: str = "monitoring") -> dict:
    return {"apiVersion": "v1", "kind": "ConfigMap",
            "metadata": {"name": "grafana-dynamo-dashboard", "namespace": namespace,
                         "labels": {"grafana_dashboard": "1"}},
            "data": {DATA_KEY: json.dumps(dashboard(), indent=2)}}


class _BlockDumper(yaml.SafeDumper):
    pass


def _str(dumper, s):
    return dumper.represent_scalar("tag:yaml.org,2002:str", s, style="|" if "\n" in s else None)


_BlockDumper.add_representer(str, _str)


def main() -> None:
    sys.stdout.write("# Generated by `python -m mxserve.k8s.dashboard` -- edit PANELS there, not here.\n")
    yaml.dump(configmap(), sys.stdout, Dumper=_BlockDumper, sort_keys=False, width=200)


if __name__ == "__main__":
    main()
