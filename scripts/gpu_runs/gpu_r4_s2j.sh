set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2j
export TMPDIR=/tmp
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/s2jprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/s2j/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/s2j/bench_prof.err
cd $GRAFT_REPO_ROOT
find /tmp/s2jprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/s2j/ \;
ls -la gpurun_out/s2j
tail -c 300 gpurun_out/s2j/bench_prof.json
for cfg in "50 448" "50 512" "52 512"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --qps $1 --max-num-seqs $2 > gpurun_out/s2j/q$1_s$2.json 2> gpurun_out/s2j/q$1_s$2.err
done
