# where the device idles at the operating point: bench QPS 46 under a kernel trace, busy fraction with
# the gaps attributed to their neighbouring kernels and the GPU time split by kernel family; then a
# late-admission A/B (on/off) at QPS 46 and 48, 20 steps each
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/gaps
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gaps/trace -o run -- python3 bench.py --steps 12 --warmup 4 --qps 46 > gpurun_out/gaps/prof_q46.json 2> gpurun_out/gaps/prof_q46.err || exit 1
python3 scripts/gpu_busy.py gpurun_out/gaps/trace/run_results.db --window 6 --attribute > gpurun_out/gaps/busy_q46.json || exit 1
cat gpurun_out/gaps/busy_q46.json
rm -rf gpurun_out/gaps/trace
for q in 46 48; do
  for la in 1 0; do
    MXS_LATE_ADMISSION=$la timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --qps $q > gpurun_out/gaps/q${q}_la${la}.json 2> gpurun_out/gaps/q${q}_la${la}.err || exit 1
    python3 - gpurun_out/gaps/q${q}_la${la}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"])
PY
  done
done
