set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5suite
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5suite/suite.log 2>&1
tail -3 gpurun_out/r5suite/suite.log
