#!/usr/bin/env bash
# Benchmark an OpenAI endpoint (concurrency sweep + fixed-QPS points) and optionally plot.
#   ./run-benchmarks.sh -u <endpoint-url> -m <model> -o <output-dir> -b <benchmark-name> [-p]
# Relative output dirs are resolved against the current directory.
set -euo pipefail
usage() { sed -n '2,4p' "$0" >&2; }
API_URL="" MODEL="" OUTPUT_DIR="" BENCHMARK_NAME="" PLOT=false
while getopts ":u:m:o:b:ph" opt; do
  case "$opt" in
    u) API_URL="$OPTARG" ;; m) MODEL="$OPTARG" ;; o) OUTPUT_DIR="$OPTARG" ;; b) BENCHMARK_NAME="$OPTARG" ;;
    p) PLOT=true ;; h) usage; exit 0 ;;
    \?) echo "Unknown option: -$OPTARG" >&2; usage; exit 1 ;;
    :) echo "Missing value for -$OPTARG" >&2; usage; exit 1 ;;
  esac
done
[[ -n "$API_URL" && -n "$MODEL" && -n "$OUTPUT_DIR" && -n "$BENCHMARK_NAME" ]] || { echo "Missing required options." >&2; usage; exit 1; }
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
[[ -f "$HERE/.venv/bin/activate" ]] && source "$HERE/.venv/bin/activate"  # shellcheck disable=SC1091
mkdir -p "$OUTPUT_DIR"
OUT="$(cd "$OUTPUT_DIR" && pwd)"
export PYTHONPATH="${HERE}${PYTHONPATH:+:$PYTHONPATH}"
python3 -m benchmarks.utils.benchmark --benchmark-name "$BENCHMARK_NAME" --endpoint-url "$API_URL" \
  --model "$MODEL" --output-dir "$OUT" ${BENCH_EXTRA_ARGS:-}
if [[ "$PLOT" == "true" ]]; then
  python3 -m benchmarks.utils.plot --data-dir "$OUT"
fi
