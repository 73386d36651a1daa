#!/usr/bin/env bash
export MXS_BENCH_ITERS_PER_STEP=${MXS_BENCH_ITERS_PER_STEP:-1}  # the --steps / --warmup counts below are engine iterations
# Interleaved A/B of late admission (engine/pacing.py) on the headline bench, in one box session:
# off / on / off / on ... with N timed steps each; one JSON line per run in $OUT/ab.jsonl.
#   scripts/ab_late_admission.sh [ROUNDS] [STEPS] [OUT]
set -euo pipefail
cd "$(dirname "$0")/.."
ROUNDS="${1:-2}"
STEPS="${2:-1000}"
OUT="${3:-gpurun_out/ab_late}"
mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
for i in $(seq 1 "$ROUNDS"); do
  for mode in 0 1; do
    MXS_LATE_ADMISSION=$mode timeout -k 10 240 python -u bench.py --steps "$STEPS" --warmup 20 > "$OUT/run.json" 2>/dev/null
    python3 - "$OUT/run.json" "$mode" "$i" >> "$OUT/ab.jsonl" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keep = {k: d[k] for k in ("value", "ttft_p50_ms", "ttft_p90_ms", "itl_p50_ms", "itl_p90_ms", "ms_per_step",
                          "running_mean", "requests_with_first_token")}
print(json.dumps(dict(keep, late_admission=int(sys.argv[2]), round=int(sys.argv[3]),
                      pacing=d["engine"].get("late_admission"))))
PY
    tail -1 "$OUT/ab.jsonl"
  done
done
