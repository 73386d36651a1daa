set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sched
for cfg in "48 8192" "48 6144" "50 6144" "50 8192"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --qps $1 --max-num-batched-tokens $2 > gpurun_out/sched/q$1_c$2.json 2> gpurun_out/sched/q$1_c$2.err
done
for f in gpurun_out/sched/*.json; do python3 -c "
import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ttft_p50_ms'],d['ttft_p90_ms'],d['itl_p50_ms'],d['itl_p90_ms'],d['running_mean'],d['steady_state'])"; done
