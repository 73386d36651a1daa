# full --gpus 2 bench (agg + disagg + multi-GPU probe) with 2 ranks sharing the GPU at half rate per rank:
# wall time of the whole job, as the driver's N=2 run would see it
set -o pipefail
export TMPDIR=/tmp MXS_BENCH_VERBOSE=1
t0=$(date +%s)
timeout -k 10 840 python bench.py --gpus 2 --qps 21 --disagg-qps 16 --steps 20 --warmup 5 \
  > gpurun_out/bench2_full.json 2> gpurun_out/bench2_full.err
rc=$?
echo "wall_s=$(( $(date +%s) - t0 )) rc=$rc" | tee gpurun_out/bench2_full.wall
tail -c 3000 gpurun_out/bench2_full.json
exit $rc
