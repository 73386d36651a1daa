# decode-aware chunk budget: Mixtral QPS 4 (bf16 / fp8 KV) and Llama-3.2-1B QPS 42 / 46 with an ITL target
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/budget
MX="--model mistralai/Mixtral-8x7B-Instruct-v0.1 --qps 4 --max-num-seqs 128 --iters-per-step 50 --steps 10 --warmup 3"
timeout -k 10 420 python3 bench.py $MX --itl-target-ms 40 > gpurun_out/budget/mixtral_bf16_t40.json 2> gpurun_out/budget/mixtral_bf16_t40.err || exit 1
tail -c 1500 gpurun_out/budget/mixtral_bf16_t40.json
timeout -k 10 420 python3 bench.py $MX --itl-target-ms 40 --kv-cache-dtype fp8 > gpurun_out/budget/mixtral_fp8_t40.json 2> gpurun_out/budget/mixtral_fp8_t40.err || exit 1
tail -c 1500 gpurun_out/budget/mixtral_fp8_t40.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --itl-target-ms 25 > gpurun_out/budget/l1b_q42_t25.json 2> gpurun_out/budget/l1b_q42_t25.err || exit 1
tail -c 1500 gpurun_out/budget/l1b_q42_t25.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --itl-target-ms 25 --qps 46 --max-num-seqs 512 > gpurun_out/budget/l1b_q46_t25.json 2> gpurun_out/budget/l1b_q46_t25.err || exit 1
tail -c 1500 gpurun_out/budget/l1b_q46_t25.json
