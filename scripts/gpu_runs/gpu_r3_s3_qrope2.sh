# fused q RoPE with 16-byte cos/sin loads: tests + prefill chunk profile, then the Mixtral runs
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/qr2
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "rope or paged or engine or Engine or generate" > gpurun_out/qr2/tests.log 2>&1 || { tail -30 gpurun_out/qr2/tests.log; exit 1; }
tail -2 gpurun_out/qr2/tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/qr2/trace -o run -- python3 scripts/step_profile.py --which prefill --iters 10 > gpurun_out/qr2/prefill.log 2>&1 || { tail -5 gpurun_out/qr2/prefill.log; exit 1; }
python3 scripts/rocpd_stats.py gpurun_out/qr2/trace/run_results.db --per 10 --top 12 > gpurun_out/qr2/prefill_chunk8192_kernel_stats.txt; cut -c1-150 gpurun_out/qr2/prefill_chunk8192_kernel_stats.txt
rm -rf gpurun_out/qr2/trace
bash scripts/gpu_r3_s3_mixtral.sh
