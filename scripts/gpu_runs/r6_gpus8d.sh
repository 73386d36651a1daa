# The driver's 8-GPU command shape on ONE GPU with the process census running: agg in the 8 ranks,
# disagg + probe sections in the probe processes (ranks > 0 detach and exit at the hand-over).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6g8d}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
T0=$(date +%s)
MXS_BENCH_SHARED_BLOCKS=16000 MXS_BENCH_VERBOSE=1 timeout -k 10 640 python scripts/probes/gpu_open_census.py 5 $D/census8.jsonl -- python bench.py --gpus 8 --steps 20 --warmup 5 ${BENCH_ARGS:---qps 5} > $D/bench8.json 2> $D/bench8.err
echo "bench8 wall_s $(( $(date +%s) - T0 ))" | tee $D/wall.txt
python -c "
import json
rows=[json.loads(l) for l in open('$D/census8.jsonl')]
print('census max GPU-open processes:', max(r['n'] for r in rows))
"
tail -c 3000 $D/bench8.json
