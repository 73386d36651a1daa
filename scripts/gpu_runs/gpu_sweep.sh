#!/usr/bin/env bash
export MXS_BENCH_ITERS_PER_STEP=${MXS_BENCH_ITERS_PER_STEP:-1}  # the --steps / --warmup counts below are engine iterations
# QPS sweep of bench.py + one rocprofv3 kernel-stats run.
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out/sweep
for q in ${QPS_LIST:-16 32 48}; do
  echo "== qps $q"
  timeout -k 10 300 python bench.py --qps $q --steps ${STEPS:-1500} --warmup ${WARMUP:-1500} > gpurun_out/sweep/q$q.log 2>&1 || { tail -30 gpurun_out/sweep/q$q.log; exit 1; }
  tail -1 gpurun_out/sweep/q$q.log
done
if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --qps ${PROF_QPS:-32} --steps 400 --warmup 800 > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  tail -1 gpurun_out/prof.log
  find gpurun_out/prof -name "*trace*" -delete
  find gpurun_out/prof -name "*stats*" | head
fi
