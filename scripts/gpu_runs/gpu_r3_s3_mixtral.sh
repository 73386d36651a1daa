# Mixtral-8x7B on one MI355X at QPS 4 with the chunk budget (ITL targets 30 / 40 ms), the 30 ms run
# under a kernel trace for the per-kernel split; then Llama-3.2-1B QPS 44 with an ITL target of 25 ms
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/mx
MX="--model mistralai/Mixtral-8x7B-Instruct-v0.1 --qps 4 --max-num-seqs 128 --iters-per-step 50 --steps 10 --warmup 3"
summ() { python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["engine"]
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"], "ms/it", round(d["ms_per_step"] / d["engine_iterations_per_step"], 2), "cb", json.dumps(e.get("chunk_budget"))[:400], "gc", e.get("gc"))
PY
}
timeout -k 10 420 python3 bench.py $MX --itl-target-ms 40 > gpurun_out/mx/mixtral_t40.json 2> gpurun_out/mx/mixtral_t40.err || exit 1
summ gpurun_out/mx/mixtral_t40.json
timeout -k 10 480 rocprofv3 --kernel-trace --stats -d gpurun_out/mx/trace -o run -- python3 bench.py $MX --itl-target-ms 30 > gpurun_out/mx/mixtral_t30_prof.json 2> gpurun_out/mx/mixtral_t30_prof.err || exit 1
summ gpurun_out/mx/mixtral_t30_prof.json
python3 scripts/rocpd_stats.py gpurun_out/mx/trace/run_results.db --top 14 > gpurun_out/mx/mixtral_t30_kernel_stats.txt; cat gpurun_out/mx/mixtral_t30_kernel_stats.txt | cut -c1-160
python3 scripts/gpu_busy.py gpurun_out/mx/trace/run_results.db --window 8 --attribute > gpurun_out/mx/mixtral_t30_busy.json; cut -c1-1200 gpurun_out/mx/mixtral_t30_busy.json
rm -rf gpurun_out/mx/trace
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --qps 44 --itl-target-ms 25 > gpurun_out/mx/l1b_q44_t25.json 2> gpurun_out/mx/l1b_q44_t25.err || exit 1
summ gpurun_out/mx/l1b_q44_t25.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --qps 44 > gpurun_out/mx/l1b_q44.json 2> gpurun_out/mx/l1b_q44.err || exit 1
summ gpurun_out/mx/l1b_q44.json
