# fused q RoPE (rope kernel writes K/V only, attention kernels rotate q on load): kernel + engine GPU
# tests, a prefill-chunk kernel profile, then bench A/B (MXS_FUSED_Q_ROPE 1 / 0) at QPS 42 and 46
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/qr
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "rope or paged or engine or Engine or generate" > gpurun_out/qr/tests.log 2>&1 || { tail -30 gpurun_out/qr/tests.log; exit 1; }
tail -2 gpurun_out/qr/tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/qr/trace -o run -- python3 scripts/step_profile.py --which prefill --iters 10 > gpurun_out/qr/prefill.log 2>&1 || { tail -5 gpurun_out/qr/prefill.log; exit 1; }
python3 scripts/rocpd_stats.py gpurun_out/qr/trace/run_results.db --per 10 --top 12 > gpurun_out/qr/prefill_chunk8192_kernel_stats.txt; cut -c1-150 gpurun_out/qr/prefill_chunk8192_kernel_stats.txt
rm -rf gpurun_out/qr/trace
for q in 42 46; do
  for fr in 1 0; do
    MXS_FUSED_Q_ROPE=$fr timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --qps $q > gpurun_out/qr/q${q}_fr${fr}.json 2> gpurun_out/qr/q${q}_fr${fr}.err || exit 1
    python3 - gpurun_out/qr/q${q}_fr${fr}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"])
PY
  done
done
