# decode table up to the 384 bucket: grow the persisted tables (MXS_TUNED_SAVE into gpurun_out/tuned),
# then bench A/B MXS_DECODE_GEMM_MAX_M 384 / 256 at QPS 42 and 46
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/dec3 gpurun_out/tuned
summ() { python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], d["value"], "ttft", d["ttft_p50_ms"], d["ttft_p90_ms"], "itl", d["itl_p50_ms"], d["itl_p90_ms"], "run", d["running_mean"], "dg", d["engine"].get("decode_gemm"))
PY
}
MXS_TUNED_SAVE=1 MXS_TUNED_DIR=gpurun_out/tuned timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/dec3/save.json 2> gpurun_out/dec3/save.err || exit 1
summ gpurun_out/dec3/save.json; ls -la gpurun_out/tuned
for q in 42 46; do
  for mm in 384 256; do
    MXS_TUNED_DIR=gpurun_out/tuned MXS_DECODE_GEMM_MAX_M=$mm timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --qps $q > gpurun_out/dec3/q${q}_m${mm}.json 2> gpurun_out/dec3/q${q}_m${mm}.err || exit 1
    summ gpurun_out/dec3/q${q}_m${mm}.json
  done
done
