#!/usr/bin/env bash
export MXS_BENCH_ITERS_PER_STEP=${MXS_BENCH_ITERS_PER_STEP:-1}  # the --steps / --warmup counts below are engine iterations
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/microbench.py ${MICRO_ARGS:-} > gpurun_out/micro.log 2>&1 || { tail -30 gpurun_out/micro.log; exit 1; }
cat gpurun_out/micro.log | grep '^{'
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --qps 32 --steps 300 --warmup 900 > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  tail -1 gpurun_out/prof.log
  find gpurun_out/prof -name "*trace*" -delete
  head -40 $(find gpurun_out/prof -name "*kernel_stats.csv")
fi
