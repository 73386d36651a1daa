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
python3 - "$OUT/frontend_metrics.txt" <<'PY'
import sys
from mxserve.planner.planner import parse_prometheus
m = parse_prometheus(open(sys.argv[1]).read())
n = m.get("dynamo_frontend_time_to_first_token_seconds_count", 0)
if n:
    print("[served] frontend-side mean TTFT %.1f ms over %d requests (request received -> first token out)"
          % (1e3 * m["dynamo_frontend_time_to_first_token_seconds_sum"] / n, n))
PY
