# hipBLASLt solution tables: GPU tests, retune (prefill_hblt new; prefill_pf re-measured against it),
# then the bench on the new tables.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6hbltune}
mkdir -p $D/tuned
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "hblt or fault_word" > $D/tests.log 2>&1
tail -1 $D/tests.log
MXS_HBLT=tune MXS_RETUNE=prefill_hblt,prefill_pf MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 \
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $D/bench_retune.json 2> $D/bench_retune.err
ls $D/tuned
MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 timeout -k 10 400 python -u bench.py --steps 40 --warmup 10 > $D/bench_after.json 2> $D/bench_after.err
MXS_HBLT=off MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 timeout -k 10 400 python -u bench.py --steps 40 --warmup 10 > $D/bench_hblt_off.json 2> $D/bench_hblt_off.err
MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 timeout -k 10 400 python -u bench.py --steps 40 --warmup 10 --qps 50 > $D/bench_after_q50.json 2> $D/bench_after_q50.err
tail -c 300 $D/bench_after.json
