set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6tserv
timeout -k 10 500 python -u -m pytest tests/test_a_serving_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6tserv/tests.log 2>&1
tail -4 gpurun_out/r6tserv/tests.log
