# VERDICT r5 next #4, on one GPU within its 16-process guard: (a) the driver's --gpus 8 command with
# the disagg phase hosted by the 8 bench ranks (no probe processes: 8 ranks + 8 probes + the arrival
# hub exceed 16 processes on one GPU; on an 8-GPU node each GPU has 2), then (b) the 8-rank multi-GPU
# probe on its own (every section, its own wall budget).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6g8b}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
T0=$(date +%s)
MXS_BENCH_VERBOSE=1 timeout -k 10 620 python bench.py --gpus 8 --steps ${STEPS:-20} --warmup ${WARMUP:-5} --probe-timeout-s 0 ${BENCH_ARGS:-} > $D/bench8.json 2> $D/bench8.err
echo "bench wall_s $(( $(date +%s) - T0 ))" | tee $D/wall.txt
tail -c 2500 $D/bench8.json
T1=$(date +%s)
timeout -k 10 560 python scripts/probes/run_probe_ranks.py 8 540 > $D/probe8.json 2> $D/probe8.err
echo "probe wall_s $(( $(date +%s) - T1 ))" | tee -a $D/wall.txt
tail -c 3000 $D/probe8.json
