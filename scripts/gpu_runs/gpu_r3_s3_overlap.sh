# decode || prefill attention on two streams: kernel-level probe, engine GPU tests with the overlap on,
# then the bench at QPS 46 / 48 with MXS_ATTN_OVERLAP 0 / 1
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ov
timeout -k 10 240 python3 scripts/attn_overlap_probe.py > gpurun_out/ov/probe.log 2>&1 || { tail -5 gpurun_out/ov/probe.log; exit 1; }
cat gpurun_out/ov/probe.log
MXS_ATTN_OVERLAP=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ov/engine_tests.log 2>&1 || { tail -20 gpurun_out/ov/engine_tests.log; exit 1; }
tail -2 gpurun_out/ov/engine_tests.log
for q in 46 48; do
  for ov in 1 0; do
    MXS_ATTN_OVERLAP=$ov timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --qps $q > gpurun_out/ov/q${q}_ov${ov}.json 2> gpurun_out/ov/q${q}_ov${ov}.err || exit 1
    python3 - gpurun_out/ov/q${q}_ov${ov}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"])
PY
  done
done
