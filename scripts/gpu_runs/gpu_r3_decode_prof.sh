# decode step B=256 ctx 4000 with the engine's tuned GEMMs + fused epilogues: per-kernel breakdown;
# Mixtral QPS 4 with the 40 ms chunk budget (step model on event-timed GPU durations)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/dprof
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof/trace -o run -- python3 scripts/step_profile.py --which decode --iters 20 --tuned > gpurun_out/dprof/decode.log 2>&1 || exit 1
tail -2 gpurun_out/dprof/decode.log
python3 scripts/rocpd_stats.py gpurun_out/dprof/trace/run_results.db --per 20 --top 16 > gpurun_out/dprof/decode_b256_stats.txt && cat gpurun_out/dprof/decode_b256_stats.txt
rm -rf gpurun_out/dprof/trace
MX="--model mistralai/Mixtral-8x7B-Instruct-v0.1 --qps 4 --max-num-seqs 128 --iters-per-step 50 --steps 10 --warmup 3"
timeout -k 10 420 python3 bench.py $MX --itl-target-ms 40 > gpurun_out/dprof/mixtral_t40.json 2> gpurun_out/dprof/mixtral_t40.err || exit 1
tail -c 2500 gpurun_out/dprof/mixtral_t40.json
