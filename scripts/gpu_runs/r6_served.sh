# Served path after the stats-sync fix: the async fault-word test, then the default bench (served
# phase on) twice: 2 client processes (default) and 4.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6served}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "fault_word or test_gemm_pf" > $D/tests.log 2>&1
tail -1 $D/tests.log
MXS_BENCH_LOG_DIR=$D/logs2 timeout -k 10 600 python -u bench.py > $D/bench_c2.json 2> $D/bench_c2.err
tail -c 700 $D/bench_c2.json
MXS_SERVED_CLIENT_PROCS=4 MXS_BENCH_LOG_DIR=$D/logs4 timeout -k 10 600 python -u bench.py > $D/bench_c4.json 2> $D/bench_c4.err
tail -c 700 $D/bench_c4.json
