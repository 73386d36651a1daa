set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5d}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
MXS_BENCH_VERBOSE=1 MXS_BENCH_LOG_DIR=$D timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $D/bench.json 2> $D/bench.err
tail -c 2500 $D/bench.json
