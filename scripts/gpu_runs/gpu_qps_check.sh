#!/usr/bin/env bash
export MXS_BENCH_ITERS_PER_STEP=${MXS_BENCH_ITERS_PER_STEP:-1}  # the --steps / --warmup counts below are engine iterations
# Longer timed window at the candidate default operating points (steady-state check).
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MXS_STEP_TIMING=1
mkdir -p gpurun_out
out=gpurun_out/qps_check.jsonl; : > $out
for cfg in ${QPS_CFGS:-"44 384 3000" "42 384 3000"}; do
  set -- $(echo $cfg | tr ',' ' ')
  echo "== qps $1 seqs $2 steps $3"
  timeout -k 10 400 python bench.py --qps $1 --max-num-seqs $2 --steps $3 --warmup 1500 ${BENCH_ARGS:-} \
    > gpurun_out/qc.log 2>&1 || { tail -30 gpurun_out/qc.log; exit 1; }
  tail -2 gpurun_out/qc.log | tee -a $out | cut -c1-120
done
