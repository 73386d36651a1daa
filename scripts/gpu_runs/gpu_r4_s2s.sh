set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2s/tuned
MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/s2s/tuned timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2s/bench1_tune.json 2> gpurun_out/s2s/bench1_tune.err
ls gpurun_out/s2s/tuned
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2s/bench1_b.json 2> gpurun_out/s2s/bench1_b.err
