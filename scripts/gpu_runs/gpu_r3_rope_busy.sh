set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rope" > gpurun_out/rope_tests.log 2>&1; rc=$?; tail -3 gpurun_out/rope_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_prefill2 -o run -- python3 scripts/step_profile.py --which prefill --iters 10 > gpurun_out/prof_prefill2.log 2>&1 || exit 1
python3 scripts/rocpd_stats.py gpurun_out/prof_prefill2/run_results.db --per 10 --top 12
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit 1
python3 scripts/gpu_busy.py gpurun_out/prof_bench/run_results.db --window 8
rm -rf gpurun_out/prof_bench gpurun_out/prof_prefill2
tail -c 600 gpurun_out/prof_bench.json
