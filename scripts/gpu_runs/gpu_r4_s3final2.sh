set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3final2
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s3final2/gpu_suite.log 2>&1 || true
tail -n 4 gpurun_out/s3final2/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3final2/smoke.log 2>&1
tail -n 2 gpurun_out/s3final2/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s3final2/bench.json 2> gpurun_out/s3final2/bench.err
tail -c 400 gpurun_out/s3final2/bench.json
