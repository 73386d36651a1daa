set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5dt}
mkdir -p $D/tuned
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned timeout -k 10 400 python3 scripts/retune_decode_buckets.py --buckets 1,2,4 > $D/retune_1_4.jsonl 2> $D/retune.err
cat $D/retune_1_4.jsonl
MXS_BENCH_SERVED=0 timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --qps 4 > $D/bench_q4_before.json 2> $D/bench_q4_before.err
MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --qps 4 > $D/bench_q4_after.json 2> $D/bench_q4_after.err
tail -c 300 $D/bench_q4_after.json
