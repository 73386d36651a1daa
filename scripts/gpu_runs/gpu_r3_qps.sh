# operating point: QPS 42 / 44 / 46 with the current build (20 steps, default chunking), twice each,
# interleaved so box drift hits every rate alike
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/qps
for rep in 1 2; do
  for q in 42 44 46; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --qps $q > gpurun_out/qps/q${q}_r${rep}.json 2> gpurun_out/qps/q${q}_r${rep}.err || exit 1
    python3 - gpurun_out/qps/q${q}_r${rep}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"])
PY
  done
done
