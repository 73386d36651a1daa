# (A) which processes hold the GPU during a full-structure 2-rank bench (ranks + probe processes);
# (B) the 8-rank bench on one GPU at a rate one GPU can carry, disagg in the ranks, smaller pools;
# (C) the 8-rank probe without the full-70B TP engine section (minutes per step when 8 ranks share a GPU)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6g8c}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 500 python scripts/probes/gpu_open_census.py 5 $D/census2.jsonl -- python bench.py --gpus 2 --steps 8 --warmup 3 --qps 20 > $D/bench2.json 2> $D/bench2.err
python -c "
import json
rows=[json.loads(l) for l in open('$D/census2.jsonl')]
print('census max GPU-open processes (2 ranks):', max(r['n'] for r in rows))
best=max(rows, key=lambda r: r['n'])
for p in best['procs']: print('  ', p['pid'], p['ppid'], p['cmd'][:120])
"
T0=$(date +%s)
MXS_BENCH_SHARED_BLOCKS=16000 MXS_BENCH_VERBOSE=1 timeout -k 10 620 python bench.py --gpus 8 --steps 20 --warmup 5 --qps 5 --probe-timeout-s 0 > $D/bench8.json 2> $D/bench8.err
echo "bench8 wall_s $(( $(date +%s) - T0 ))" | tee $D/wall.txt
tail -c 1500 $D/bench8.json
T1=$(date +%s)
MXS_PROBE_SECTIONS=collectives,graph_collectives,tp,ep,p2p,tp_layer,ep_engine,disagg_8b timeout -k 10 460 python scripts/probes/run_probe_ranks.py 8 440 > $D/probe8.json 2> $D/probe8.err
echo "probe8 wall_s $(( $(date +%s) - T1 ))" | tee -a $D/wall.txt
tail -c 2500 $D/probe8.json
