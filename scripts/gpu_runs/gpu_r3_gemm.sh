set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_big" > gpurun_out/gemm_big_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gemm_big_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/gemm_big_probe.py 8192 4096 2048 > gpurun_out/gemm_big_probe.log 2>&1; rc=$?; cat gpurun_out/gemm_big_probe.log | grep '^{'; exit $rc
