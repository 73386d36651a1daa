set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/suite3
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/suite3/gpu_suite.log 2>&1 || true
tail -n 6 gpurun_out/suite3/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite3/smoke.log 2>&1
tail -n 2 gpurun_out/suite3/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/suite3/bench.json 2> gpurun_out/suite3/bench.err
tail -c 700 gpurun_out/suite3/bench.json
