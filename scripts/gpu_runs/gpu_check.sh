#!/usr/bin/env bash
export MXS_BENCH_ITERS_PER_STEP=${MXS_BENCH_ITERS_PER_STEP:-1}  # the --steps / --warmup counts below are engine iterations
# One gpurun call: kernel numerics, smoke, short bench, rocprofv3 kernel stats.
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
echo "== build"; python setup_ext.py > gpurun_out/build.log 2>&1
echo "== kernel tests"
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/test_kernels.log 2>&1 || { tail -50 gpurun_out/test_kernels.log; exit 1; }
tail -3 gpurun_out/test_kernels.log
echo "== smoke"
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -50 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
echo "== bench"
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-300} --warmup ${BENCH_WARMUP:-300} ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -50 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
