# prefill attention: D = 128 row sum of P on the MFMA pipe (ones x P) instead of 32 VALU adds per tile
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pfc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "prefill" > gpurun_out/pfc/tests.log 2>&1 || { tail -30 gpurun_out/pfc/tests.log; exit 1; }
tail -2 gpurun_out/pfc/tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pfc/trace -o run -- python3 scripts/step_profile.py --which prefill --iters 10 > gpurun_out/pfc/prefill.log 2>&1 || { tail -5 gpurun_out/pfc/prefill.log; exit 1; }
python3 scripts/rocpd_stats.py gpurun_out/pfc/trace/run_results.db --per 10 --top 8 > gpurun_out/pfc/prefill_stats.txt; cut -c1-150 gpurun_out/pfc/prefill_stats.txt
rm -rf gpurun_out/pfc/trace
timeout -k 10 120 python3 scripts/prefill_attn_probe.py > gpurun_out/pfc/probe.log 2>&1 || { tail -5 gpurun_out/pfc/probe.log; exit 1; }
tail -12 gpurun_out/pfc/probe.log
