set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4b1 gpurun_out/tuned
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_pf" -m gpu 2>&1 | tail -3
GB_PF=0,16 GB_VARIANTS=7 timeout -k 10 300 python -u scripts/gemm_big_probe.py 8192 4240 2048
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/tuned
MXS_GEMM_PF=off timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --qps 48 > gpurun_out/r4b1/off_q48.json 2> gpurun_out/r4b1/off_q48.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --qps 48 > gpurun_out/r4b1/auto_q48.json 2> gpurun_out/r4b1/auto_q48.err
tail -c 1500 gpurun_out/r4b1/*.json
