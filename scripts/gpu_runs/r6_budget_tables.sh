# Tables for the 7168-token step budget (row buckets up to 7168 + 448): measure the buckets the
# packaged tables lack (hipBLASLt solutions, gemm_pf, M plans), then the default bench from them.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6budget}
mkdir -p $D/tuned
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
MXS_HBLT=tune MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 \
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $D/bench_tune.json 2> $D/bench_tune.err
ls -la $D/tuned
MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned timeout -k 10 600 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err
tail -c 400 $D/bench_default.json
