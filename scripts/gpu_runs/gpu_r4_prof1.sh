set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof1
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rp -o run -- python3 bench.py --steps 20 --warmup 5 --qps 48 > gpurun_out/prof1/bench.json 2> gpurun_out/prof1/bench.err || echo "bench rc=$?"
find /tmp/rp -name "*stats.csv" -exec cp {} gpurun_out/prof1/ \;
ls -la gpurun_out/prof1; tail -3 gpurun_out/prof1/bench.err
