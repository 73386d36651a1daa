set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2u
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "skinny or decode_gemm_all" > gpurun_out/s2u/kt.log 2>&1 || true
grep -cE "PASSED" gpurun_out/s2u/kt.log || true
grep -E "FAILED" gpurun_out/s2u/kt.log | head || true
timeout -k 10 400 python -u scripts/tp_shard_gemm_probe.py > gpurun_out/s2u/shard.jsonl 2> gpurun_out/s2u/shard.err
