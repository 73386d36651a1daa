set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2e
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s2e/dec -o dec -- python3 $GRAFT_REPO_ROOT/scripts/step_profile.py --which decode --tuned --batch 256 --iters 20 > $GRAFT_REPO_ROOT/gpurun_out/s2e/dec.log 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --qps 50 > gpurun_out/s2e/bench_q50.json 2> gpurun_out/s2e/bench_q50.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --qps 49 > gpurun_out/s2e/bench_q49.json 2> gpurun_out/s2e/bench_q49.err
