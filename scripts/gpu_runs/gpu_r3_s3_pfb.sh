# prefill attention: row max across the wave halves by permlane32 swap (was an LDS bpermute)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pfb
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "prefill" > gpurun_out/pfb/tests.log 2>&1 || { tail -30 gpurun_out/pfb/tests.log; exit 1; }
tail -2 gpurun_out/pfb/tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pfb/trace -o run -- python3 scripts/step_profile.py --which prefill --iters 10 > gpurun_out/pfb/prefill.log 2>&1 || { tail -5 gpurun_out/pfb/prefill.log; exit 1; }
python3 scripts/rocpd_stats.py gpurun_out/pfb/trace/run_results.db --per 10 --top 8 > gpurun_out/pfb/prefill_stats.txt; cut -c1-150 gpurun_out/pfb/prefill_stats.txt
rm -rf gpurun_out/pfb/trace
timeout -k 10 120 python3 scripts/prefill_attn_probe.py > gpurun_out/pfb/probe.log 2>&1 || { tail -5 gpurun_out/pfb/probe.log; exit 1; }
tail -12 gpurun_out/pfb/probe.log
