# decode table extended to the 320 / 384 graph buckets (MXS_DECODE_GEMM_MAX_M=384): the tuner's picks
# and a decode step profile at B = 320 / 384 with them
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MXS_DECODE_GEMM_MAX_M=384
mkdir -p gpurun_out/dec2
for B in 320 384; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/dec2/t$B -o run -- python3 scripts/step_profile.py --which decode --iters 20 --tuned --batch $B > gpurun_out/dec2/b$B.log 2>&1 || { tail -5 gpurun_out/dec2/b$B.log; exit 1; }
  grep "'proj'" gpurun_out/dec2/b$B.log | head -12
  python3 scripts/rocpd_stats.py gpurun_out/dec2/t$B/run_results.db --per 20 --top 14 > gpurun_out/dec2/decode_b${B}_stats.txt
  echo "== B=$B"; cut -c1-140 gpurun_out/dec2/decode_b${B}_stats.txt
  rm -rf gpurun_out/dec2/t$B
done
