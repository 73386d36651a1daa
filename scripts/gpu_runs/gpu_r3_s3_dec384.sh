# decode steps at the batch the headline actually runs (running set 250-390): B = 256 / 320 / 384,
# ctx 4000, engine-tuned GEMM choices, per-kernel time
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/dec
for B in 256 320 384; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/dec/t$B -o run -- python3 scripts/step_profile.py --which decode --iters 20 --tuned --batch $B > gpurun_out/dec/b$B.log 2>&1 || { tail -5 gpurun_out/dec/b$B.log; exit 1; }
  python3 scripts/rocpd_stats.py gpurun_out/dec/t$B/run_results.db --per 20 --top 14 > gpurun_out/dec/decode_b${B}_stats.txt
  echo "== B=$B"; cut -c1-140 gpurun_out/dec/decode_b${B}_stats.txt
  rm -rf gpurun_out/dec/t$B
done
