# rocprofv3 kernel statistics of the headline bench (QPS 42, 20 x 50-iteration window); only the stats files are kept
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit $?
find /tmp/prof -name "*stats*" -exec cp {} gpurun_out/prof/ \;
ls gpurun_out/prof
