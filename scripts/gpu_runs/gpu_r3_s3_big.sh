# (1) prefill attention A/B HEAD (ab_head/) vs tree; (2) decode GEMM retune with gemm_big candidates
# (lm_head, gate_up at M >= 128) saved to gpurun_out/tuned; (3) bench QPS 42 with that table
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/big gpurun_out/tuned
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "prefill or gemm_big or decode_gemm_tuner" > gpurun_out/big/tests.log 2>&1 || { tail -30 gpurun_out/big/tests.log; exit 1; }
tail -1 gpurun_out/big/tests.log
for r in 1 2; do
  echo "== head"; (cd ab_head && timeout -k 10 120 python3 scripts/prefill_attn_probe.py 2>/dev/null) || exit 1
  echo "== tree"; timeout -k 10 120 python3 scripts/prefill_attn_probe.py 2>/dev/null || exit 1
done
MXS_RETUNE=1 MXS_TUNED_SAVE=1 MXS_TUNED_DIR=gpurun_out/tuned MXS_DECODE_GEMM_REPORT=gpurun_out/big/report.jsonl timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/big/retune.json 2> gpurun_out/big/retune.err || { tail -20 gpurun_out/big/retune.err; exit 1; }
grep -E '"big"|lm_head|gate_up' gpurun_out/big/report.jsonl | cut -c1-240
MXS_TUNED_DIR=gpurun_out/tuned timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/big/q42.json 2> gpurun_out/big/q42.err || exit 1
python3 - gpurun_out/big/q42.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"], d["engine"].get("decode_gemm"))
PY
