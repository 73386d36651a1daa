set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2k
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "rope" > gpurun_out/s2k/kt.log 2>&1 || true
grep -E "PASSED|FAILED|Error" gpurun_out/s2k/kt.log | tail -40
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/s2kprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/s2k/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/s2k/bench_prof.err
cd $GRAFT_REPO_ROOT
find /tmp/s2kprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/s2k/ \;
