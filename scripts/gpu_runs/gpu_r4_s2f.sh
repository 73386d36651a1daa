set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2f
timeout -k 10 240 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "fused_prefill_chain" > gpurun_out/s2f/et.log 2>&1 || true
grep -E "PASSED|FAILED|Error|assert" gpurun_out/s2f/et.log | tail -10
for cfg in "50 3072 0" "49 4096 0" "50 6144 17" "50 5120 0"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --qps $1 --max-num-batched-tokens $2 --itl-target-ms $3 > gpurun_out/s2f/q$1_c$2_t$3.json 2> gpurun_out/s2f/q$1_c$2_t$3.err
done
