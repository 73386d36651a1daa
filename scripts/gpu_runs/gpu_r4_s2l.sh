set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2l
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_engine_gpu.py > gpurun_out/s2l/et.log 2>&1 || true
grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/s2l/et.log | tail -40
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2l/bench.json 2> gpurun_out/s2l/bench.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --qps 50 --max-num-seqs 512 > gpurun_out/s2l/bench_q50_s512.json 2> gpurun_out/s2l/bench_q50_s512.err
