# Default bench (served phase on) for the served TTFT breakdown.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6servedbd}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
MXS_BENCH_LOG_DIR=$D/logs timeout -k 10 600 python -u bench.py > $D/bench.json 2> $D/bench.err
tail -c 1500 $D/bench.json
