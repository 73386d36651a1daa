# mt GEMM tile order (row tiles fastest) at decode M; kernel tests; Mixtral QPS 4 with the NNLS-priced
# chunk budget; 1-GPU bench writing the persisted decode/prefill GEMM tables
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/mt gpurun_out/tuned
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "mt_gemm or decode_gemm" > gpurun_out/mt/tests.log 2>&1; rc=$?; tail -3 gpurun_out/mt/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/mt_gemm_probe.py 128,256 llama-3.2-1b > gpurun_out/mt/probe_1b.jsonl 2> gpurun_out/mt/probe_1b.err || exit 1
cat gpurun_out/mt/probe_1b.jsonl
MXS_TUNED_SAVE=1 MXS_TUNED_DIR=gpurun_out/tuned timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/mt/bench_save.json 2> gpurun_out/mt/bench_save.err || exit 1
tail -c 700 gpurun_out/mt/bench_save.json
MXS_TUNED_DIR=gpurun_out/tuned timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/mt/bench_table.json 2> gpurun_out/mt/bench_table.err || exit 1
tail -c 700 gpurun_out/mt/bench_table.json
MX="--model mistralai/Mixtral-8x7B-Instruct-v0.1 --qps 4 --max-num-seqs 128 --iters-per-step 50 --steps 10 --warmup 3"
MXS_TUNED_SAVE=1 MXS_TUNED_DIR=gpurun_out/tuned timeout -k 10 420 python3 bench.py $MX --itl-target-ms 40 > gpurun_out/mt/mixtral_t40.json 2> gpurun_out/mt/mixtral_t40.err || exit 1
tail -c 1200 gpurun_out/mt/mixtral_t40.json
timeout -k 10 600 python -u -m pytest tests/test_c_tp8_gpu.py tests/test_mgpu_probe_gpu.py tests/test_kernels_gpu.py -x -v --timeout 300 --timeout-method thread -k "ep8_moe_layer or probe_two_ranks or moe_a2a_dispatch" > gpurun_out/mt/ep_tests.log 2>&1; rc=$?; tail -8 gpurun_out/mt/ep_tests.log; [ $rc -eq 0 ] || exit $rc
