set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4b1 gpurun_out/tuned
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/tuned
# baseline (gemm_pf off) vs tuned routing, QPS 44 and 48, driver-shape runs
MXS_GEMM_PF=off timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --qps 48 > gpurun_out/r4b1/off_q48.json 2> gpurun_out/r4b1/off_q48.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --qps 48 > gpurun_out/r4b1/auto_q48.json 2> gpurun_out/r4b1/auto_q48.err
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --qps 44 > gpurun_out/r4b1/auto_q44.json 2> gpurun_out/r4b1/auto_q44.err
tail -c 600 gpurun_out/r4b1/*.json
