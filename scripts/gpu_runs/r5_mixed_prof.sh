# kernel breakdown of one mixed step (300 decode rows at ~4.2k context + a 2400-token chunk after 1600 cached)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5mp}
mkdir -p $D
MS_MODES=combined_attn_overlap MS_CASES=${MS_CASES:-300:4250:2400:1600} timeout -k 10 300 \
  rocprofv3 --kernel-trace -d $D/prof -o run -- python3 -u scripts/probes/mixed_step_probe.py > $D/probe.log 2>&1
tail -3 $D/probe.log
DB=$(find $D/prof -name "*.db" | head -1)
python3 scripts/rocpd_stats.py "$DB" --top 45 > $D/kernel_stats.txt
head -30 $D/kernel_stats.txt
