# session 3 of round 3: restored tree on MI355X -- GPU suite, smoke, 1-GPU bench line, gemm_big vs hipBLASLt probe
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3_suite.log 2>&1 && echo SUITE_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s3_bench1.json 2> gpurun_out/s3_bench1.err && echo BENCH1_OK && \
timeout -k 10 240 python scripts/gemm_big_probe.py > gpurun_out/s3_gemm_big.log 2>&1 && echo GEMMBIG_OK
rc=$?
tail -2 gpurun_out/s3_suite.log; tail -1 gpurun_out/s3_smoke.log; cut -c1-700 gpurun_out/s3_bench1.json; cat gpurun_out/gemm_big_probe.jsonl 2>/dev/null
exit $rc
