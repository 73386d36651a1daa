# prefill M plans priced with the output copy (all-mm splits): probe, then a prefill+decode mixed-step
# profile at one prompt + 270 decode rows (M = 4270) with the plans on / off
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/mp2
timeout -k 10 200 python3 scripts/mplan_probe.py > gpurun_out/mp2/probe.jsonl 2> gpurun_out/mp2/probe.err || { tail -5 gpurun_out/mp2/probe.err; exit 1; }
cat gpurun_out/mp2/probe.jsonl
for mp in 1 0; do
  MXS_MPLAN=$mp timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/mp2/q44_mp${mp}.json 2> gpurun_out/mp2/q44_mp${mp}.err || exit 1
  python3 - gpurun_out/mp2/q44_mp${mp}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"])
PY
done
