# running-sequence cap vs saturation: bench at QPS list with MAXSEQS (bf16 headline config otherwise)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5cap}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
for Q in ${QPS_LIST:-50 51 52}; do
  MXS_BENCH_MAX_SEQS=${MAXSEQS:-512} MXS_BENCH_SERVED=0 timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --qps $Q > $D/bench_q$Q.json 2> $D/bench_q$Q.err
  python3 -c "
import json
d=json.loads(open('$D/bench_q$Q.json').read().strip().splitlines()[-1])
print($Q, d['value'], d['ttft_p50_ms'], d['ttft_p90_ms'], d['itl_p50_ms'], d['itl_p90_ms'], d.get('running_mean'), d['config'].get('global_batch'))
" | tee -a $D/sweep.txt
done
