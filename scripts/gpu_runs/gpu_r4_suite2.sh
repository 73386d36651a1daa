set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/suite2
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/suite2/gpu_suite.log 2>&1 || true
tail -n 15 gpurun_out/suite2/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite2/smoke.log 2>&1
tail -n 3 gpurun_out/suite2/smoke.log
