#!/usr/bin/env bash
export MXS_BENCH_ITERS_PER_STEP=${MXS_BENCH_ITERS_PER_STEP:-1}  # the --steps / --warmup counts below are engine iterations
# rocprofv3 kernel-trace stats of a bench run (summaries only; traces deleted to stay under 64 MiB).
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
rm -rf gpurun_out/prof && mkdir -p gpurun_out/prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --qps ${PROF_QPS:-36} --steps ${PROF_STEPS:-600} --warmup ${PROF_WARMUP:-900} ${BENCH_ARGS:-} \
  > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
tail -1 gpurun_out/prof.log
find gpurun_out/prof -name "*trace*" -delete
find gpurun_out/prof -name "*stats*"
