# GC freeze: the kernel-trace busy fraction at QPS 46 with the start-up heap frozen (the 114 ms
# inter-step gaps of busy_q46.json should be gone), then freeze on/off A/B at QPS 46 and 48
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/gc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gc/trace -o run -- python3 bench.py --steps 12 --warmup 4 --qps 46 > gpurun_out/gc/prof_q46.json 2> gpurun_out/gc/prof_q46.err || exit 1
python3 scripts/gpu_busy.py gpurun_out/gc/trace/run_results.db --window 6 --attribute > gpurun_out/gc/busy_q46_frozen.json || exit 1
cat gpurun_out/gc/busy_q46_frozen.json
rm -rf gpurun_out/gc/trace
for q in 46 48; do
  for fz in 1 0; do
    MXS_GC_FREEZE=$fz timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --qps $q > gpurun_out/gc/q${q}_fz${fz}.json 2> gpurun_out/gc/q${q}_fz${fz}.err || exit 1
    python3 - gpurun_out/gc/q${q}_fz${fz}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"], "gc", d["engine"].get("gc"))
PY
  done
done
