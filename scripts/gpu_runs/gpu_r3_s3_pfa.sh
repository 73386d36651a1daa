# prefill attention with the K fragment reads two ahead of their MFMAs (sched_group_barrier) and the
# occupancy pinned at 4 waves/SIMD for D = 64: kernel tests, then the 8192-token prefill chunk profile
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pfa
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "prefill" > gpurun_out/pfa/tests.log 2>&1 || { tail -30 gpurun_out/pfa/tests.log; exit 1; }
tail -2 gpurun_out/pfa/tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pfa/trace -o run -- python3 scripts/step_profile.py --which prefill --iters 10 > gpurun_out/pfa/prefill.log 2>&1 || { tail -5 gpurun_out/pfa/prefill.log; exit 1; }
python3 scripts/rocpd_stats.py gpurun_out/pfa/trace/run_results.db --per 10 --top 8 > gpurun_out/pfa/prefill_stats.txt; cut -c1-150 gpurun_out/pfa/prefill_stats.txt
rm -rf gpurun_out/pfa/trace
timeout -k 10 120 python3 scripts/prefill_attn_probe.py > gpurun_out/pfa/probe.log 2>&1 || { tail -5 gpurun_out/pfa/probe.log; exit 1; }
tail -12 gpurun_out/pfa/probe.log
