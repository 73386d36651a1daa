# short-bench variance at QPS 40 vs QPS 42 with a stricter steady-state test
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/bench_repeat2.jsonl; : > $out
for args in "--qps 40" "--qps 40" "--qps 40" "--qps 42 --steady-window-s 5" "--qps 42 --steady-window-s 5"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args 2> gpurun_out/br.err | tail -1 >> $out || exit 1
  tail -1 $out | cut -c1-120
done
