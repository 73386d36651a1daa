#!/usr/bin/env bash
# quick iteration: selected kernel tests + microbench (no profiler)
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "${TESTK:-decode}" > gpurun_out/quick_tests.log 2>&1 || { tail -40 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
timeout -k 10 300 python scripts/microbench.py ${MICRO_ARGS:-} > gpurun_out/micro.log 2>&1 || { tail -30 gpurun_out/micro.log; exit 1; }
grep '^{' gpurun_out/micro.log
