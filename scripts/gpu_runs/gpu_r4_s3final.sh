set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3final
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s3final/gpu_suite.log 2>&1 || true
tail -n 4 gpurun_out/s3final/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3final/smoke.log 2>&1
tail -n 2 gpurun_out/s3final/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s3final/bench.json 2> gpurun_out/s3final/bench.err
tail -c 400 gpurun_out/s3final/bench.json
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/s3prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/s3final/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/s3final/bench_prof.err
cd $GRAFT_REPO_ROOT
find /tmp/s3prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/s3final/ \;
