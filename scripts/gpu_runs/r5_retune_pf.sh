set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5tune}
mkdir -p $D/tuned
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
MXS_RETUNE=prefill_pf MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 \
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $D/bench_retune.json 2> $D/bench_retune.err
ls $D/tuned
MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $D/bench_after.json 2> $D/bench_after.err
tail -c 1200 $D/bench_after.json
