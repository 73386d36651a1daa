set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6suite
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6suite/suite.log 2>&1
tail -3 gpurun_out/r6suite/suite.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6suite/smoke.log 2>&1
tail -2 gpurun_out/r6suite/smoke.log
