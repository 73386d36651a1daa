set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6thblt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "hblt" > gpurun_out/r6thblt/tests.log 2>&1
tail -6 gpurun_out/r6thblt/tests.log
