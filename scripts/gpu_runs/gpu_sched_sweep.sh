#!/usr/bin/env bash
export MXS_BENCH_ITERS_PER_STEP=${MXS_BENCH_ITERS_PER_STEP:-1}  # the --steps / --warmup counts below are engine iterations
# Scheduler knobs at the headline config: prefill token budget x max running seqs x QPS.
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MXS_STEP_TIMING=1
mkdir -p gpurun_out
out=gpurun_out/sched_sweep.jsonl; : > $out
for cfg in "40 8192 256" "40 16384 256" "44 16384 384" "44 8192 384" "48 16384 384"; do
  set -- $cfg
  echo "== qps $1 mbt $2 seqs $3"
  timeout -k 10 300 python bench.py --qps $1 --max-num-batched-tokens $2 --max-num-seqs $3 \
    --steps 1500 --warmup 1500 > gpurun_out/sched.log 2>&1 || { tail -30 gpurun_out/sched.log; exit 1; }
  tail -2 gpurun_out/sched.log | tee -a $out | cut -c1-200
done
