set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big" -m gpu 2>&1 | tail -5
GB_VARIANTS=6,7 timeout -k 10 300 python -u scripts/gemm_big_probe.py 8192 4240 4096 2048
