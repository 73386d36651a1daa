#!/usr/bin/env bash
# End-to-end served benchmark on one GPU (the reference's run-benchmarks.sh path, :61-71): OpenAI
# frontend process + worker process (started as the manifests start them) + the open-loop load
# generator over HTTP/SSE.  Compare with the in-process bench.py at the same QPS / ISL / OSL.
#   scripts/served_bench.sh [QPS] [NUM_REQUESTS] [OUT_DIR]
set -euo pipefail
cd "$(dirname "$0")/.."
QPS="${1:-42}"
N="${2:-1800}"
OUT="${3:-gpurun_out/served}"
MODEL="${MODEL:-meta-llama/Llama-3.2-1B-Instruct}"
FE_PORT="${FE_PORT:-18000}"
W_PORT="${W_PORT:-18081}"
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH="$PWD" MXS_CUDA_GRAPH_MAX_BS=384
python3 -m dynamo.frontend --http-port "$FE_PORT" --num-procs "${FE_PROCS:-4}" > "$OUT/frontend.log" 2>&1 &
FE=$!
python3 -m dynamo.vllm --model "$MODEL" --frontend-url "http://127.0.0.1:$FE_PORT" --host 127.0.0.1 \
  --port "$W_PORT" --max-num-seqs 384 --max-num-batched-tokens 8192 > "$OUT/worker.log" 2>&1 &
W=$!
cleanup() { kill "$W" "$FE" 2>/dev/null || true; wait "$W" "$FE" 2>/dev/null || true; }
trap cleanup EXIT
for i in $(seq 1 240); do
  if curl -sf "http://127.0.0.1:$FE_PORT/v1/models" | grep -q '"id"'; then break; fi
  kill -0 "$W" 2>/dev/null || { echo "worker died"; tail -50 "$OUT/worker.log"; exit 1; }
  sleep 1
done
curl -sf "http://127.0.0.1:$FE_PORT/v1/models" | grep -q '"id"' || { echo "no worker registered"; exit 1; }
echo "[served] worker registered; running QPS $QPS x $N requests"
python3 -m benchmarks.utils.benchmark --benchmark-name served --endpoint-url "http://127.0.0.1:$FE_PORT" \
  --model "$MODEL" --output-dir "$OUT" --concurrency "" --request-rate "$QPS" --num-requests "$N" \
  --isl 4000 --osl 500 --token-ids --vocab 128256 --warmup-s 15 &
B=$!
# CPU of each process over the run (frontend parent / frontend processes summed / worker / load
# generator): which one is the limit
( while kill -0 "$B" 2>/dev/null; do
    echo "$(date +%s) $(ps -o pcpu= -p "$FE") $(ps -o pcpu= --ppid "$FE" | awk '{s+=$1} END {print s+0}') $(ps -o pcpu= -p "$W") $(ps -o pcpu= -p "$B")"; sleep 5
  done ) > "$OUT/cpu_fe_worker_client.txt" &
wait "$B"
curl -sf "http://127.0.0.1:$FE_PORT/metrics" > "$OUT/frontend_metrics.txt" || true
curl -sf "http://127.0.0.1:$W_PORT/stats" > "$OUT/worker_stats.json" || true
# request traces (per frontend process: a few fetches land on different processes)
for i in 1 2 3 4 5 6 7 8; do curl -sf "http://127.0.0.1:$FE_PORT/debug/traces?n=300" > "$OUT/traces_$i.json" || true; done
python3 - "$OUT" <<'PY'
import glob, json, statistics, sys
seen, rows = set(), []
for f in glob.glob(sys.argv[1] + "/traces_*.json"):
    try:
        for t in json.load(open(f))["traces"]:
            if t["request_id"] not in seen and "first_token" in t.get("spans_ms", {}):
                seen.add(t["request_id"])
                rows.append(t)
    except (OSError, ValueError, KeyError):
        pass
if rows:
    med = lambda xs: round(statistics.median(xs), 2) if xs else None
    sp = [r["spans_ms"] for r in rows]
    wk = [r.get("worker_ms") or {} for r in rows]
    out = {"traces": len(rows), "routed_ms_p50": med([s.get("routed", 0) for s in sp]),
           "first_token_ms_p50": med([s["first_token"] for s in sp]),
           "worker_queue_ms_p50": med([w["queue_ms"] for w in wk if "queue_ms" in w]),
           "worker_prefill_ms_p50": med([w["prefill_ms"] for w in wk if "prefill_ms" in w]),
           "worker_inbox_ms_p50": med([w["inbox_ms"] for w in wk if "inbox_ms" in w]),
           "delivery_ms_p50": med([w["delivery_ms"] for w in wk if "delivery_ms" in w])}
    print("[served] TTFT breakdown (median over %d traces): %s" % (len(rows), json.dumps(out)))
    json.dump(out, open(sys.argv[1] + "/ttft_breakdown.json", "w"))
PY
python3 - "$OUT/frontend_metrics.txt" <<'PY'
import sys
from mxserve.planner.planner import parse_prometheus
m = parse_prometheus(open(sys.argv[1]).read())
n = m.get("dynamo_frontend_time_to_first_token_seconds_count", 0)
if n:
    print("[served] frontend-side mean TTFT %.1f ms over %d requests (request received -> first token out)"
          % (1e3 * m["dynamo_frontend_time_to_first_token_seconds_sum"] / n, n))
PY
