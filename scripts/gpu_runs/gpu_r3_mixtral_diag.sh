# Mixtral QPS 4 with the chunk budget: fit diagnostics; MoE decode table persisted
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/mx gpurun_out/tuned
cp mxserve/ops/tuned/*.json gpurun_out/tuned/ 2>/dev/null
MX="--model mistralai/Mixtral-8x7B-Instruct-v0.1 --qps 4 --max-num-seqs 128 --iters-per-step 50 --steps 10 --warmup 3"
MXS_TUNED_SAVE=1 MXS_TUNED_DIR=gpurun_out/tuned timeout -k 10 420 python3 bench.py $MX --itl-target-ms 40 > gpurun_out/mx/mixtral_t40.json 2> gpurun_out/mx/mixtral_t40.err || exit 1
tail -c 2500 gpurun_out/mx/mixtral_t40.json
