set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5dprof}
mkdir -p $D
for B in ${BATCHES:-448 256}; do
  rm -rf /tmp/dprof$B
  timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/dprof$B -o run -- python3 scripts/step_profile.py --which decode --tuned --batch $B --iters 10 > $D/step_b$B.log 2>&1
  DB=$(find /tmp/dprof$B -name "*.db" | head -1)
  python3 scripts/rocpd_stats.py "$DB" --top 40 --per 10 > $D/decode_b${B}_kernel_stats.txt
  head -24 $D/decode_b${B}_kernel_stats.txt
done
