set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/suite
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite/gpu_suite.log 2>&1
tail -n 5 gpurun_out/suite/gpu_suite.log
