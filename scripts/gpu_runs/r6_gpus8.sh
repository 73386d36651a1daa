# the driver's 8-GPU SCALE command rehearsed with the 8 ranks sharing ONE GPU
# (3P+5D disagg plan, 8-rank custom all-reduce, TP-8 / EP-8 probe sections, routed arrivals).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6g8}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
T0=$(date +%s)
MXS_BENCH_VERBOSE=1 timeout -k 10 620 python bench.py --gpus 8 --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS:-} > $D/bench8.json 2> $D/bench8.err
echo "wall_s $(( $(date +%s) - T0 ))" | tee $D/wall.txt
tail -c 2500 $D/bench8.json
