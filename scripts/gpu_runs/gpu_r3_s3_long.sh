# operating point: longer timed windows (60 steps x 50 iterations, ~32 s) at QPS 42 / 44 / 46: is the
# rate sustained (TTFT p90 flat) and where does ITL p90 sit
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/long
for q in 44 46 42; do
  timeout -k 10 420 python3 bench.py --steps 60 --warmup 5 --qps $q > gpurun_out/long/q${q}.json 2> gpurun_out/long/q${q}.err || exit 1
  python3 - gpurun_out/long/q${q}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"], "steady", d["steady_state"], "n_ttft", d["requests_with_first_token"], "ms/step", d["ms_per_step"])
PY
done
