set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5mt}
mkdir -p $D
i=0
while read -r M N K; do
  i=$((i+1))
  rm -rf /tmp/mtp$i
  timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/mtp$i -o run -- python3 scripts/probes/mt_shape_probe.py $M $N $K > $D/mt_$M_$N_$K.log 2>&1
  DB=$(find /tmp/mtp$i -name "*.db" | head -1)
  echo "== M $M N $N K $K" >> $D/mt_probe.txt
  python3 scripts/rocpd_stats.py "$DB" --top 12 --by-grid mt_gemm >> $D/mt_probe.txt
done <<'L'
256 2048 2048
256 2048 512
256 3072 2048
448 2048 2048
L
cat $D/mt_probe.txt
