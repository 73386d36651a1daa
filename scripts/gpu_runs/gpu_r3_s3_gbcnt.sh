# gemm_big at mixed-step row counts vs hipBLASLt, and the counters rocprofv3 offers on this box
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/gb
GB_VARIANTS=0 timeout -k 10 240 python3 scripts/gemm_big_probe.py 3300 4300 1300 > gpurun_out/gb/mid.log 2>&1 || { tail -5 gpurun_out/gb/mid.log; exit 1; }
cut -c1-330 gpurun_out/gb/mid.log
timeout -k 10 60 rocprofv3 -L > gpurun_out/gb/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" gpurun_out/gb/counters.txt | sort -u | tr '\n' ' ' | head -c 6000
