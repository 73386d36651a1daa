#!/usr/bin/env bash
export MXS_BENCH_ITERS_PER_STEP=${MXS_BENCH_ITERS_PER_STEP:-1}  # the --steps / --warmup counts below are engine iterations
# One gpurun call: every GPU test, smoke, short bench (extensions are built in-tree beforehand).
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/test_gpu.log 2>&1 || { tail -60 gpurun_out/test_gpu.log; exit 1; }
tail -3 gpurun_out/test_gpu.log
echo "== smoke"
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -50 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo "== bench"
timeout -k 10 400 python bench.py --steps ${BENCH_STEPS:-1500} --warmup ${BENCH_WARMUP:-1500} ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -50 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
