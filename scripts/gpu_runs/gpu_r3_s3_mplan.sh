# prefill M plans: probe (plan vs F.linear), engine GPU tests, bench A/B MXS_MPLAN 1 / 0 at QPS 44
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/mp
timeout -k 10 200 python3 scripts/mplan_probe.py > gpurun_out/mp/probe.jsonl 2> gpurun_out/mp/probe.err || { tail -5 gpurun_out/mp/probe.err; exit 1; }
cat gpurun_out/mp/probe.jsonl
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mp/tests.log 2>&1 || { tail -30 gpurun_out/mp/tests.log; exit 1; }
tail -1 gpurun_out/mp/tests.log
for r in 1 2; do
  for mp in 1 0; do
    MXS_MPLAN=$mp timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/mp/q44_mp${mp}_r$r.json 2> gpurun_out/mp/q44_mp${mp}_r$r.err || exit 1
    python3 - gpurun_out/mp/q44_mp${mp}_r$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"])
PY
  done
done
