# labelled side data point: the headline workload with an fp8 (e4m3fn) KV cache at higher request rates
export MXS_BENCH_ITERS_PER_STEP=${MXS_BENCH_ITERS_PER_STEP:-1}  # the --steps / --warmup counts below are engine iterations
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/fp8kv_sweep.jsonl; : > $out
for q in ${QPS_LIST:-50 56 62}; do
  echo "== qps $q"
  timeout -k 10 300 python bench.py --kv-cache-dtype fp8 --qps $q --max-num-seqs 512 --steps 1500 --warmup 200 \
    > gpurun_out/fk.log 2> gpurun_out/fk.err || { tail -20 gpurun_out/fk.err; exit 1; }
  tail -1 gpurun_out/fk.log | tee -a $out | cut -c1-200
done
