# bench.py --gpus 2 on a 1-GPU box: agg x2 + disagg 1P+1D + the multi-GPU probe (ranks share the GPU,
# so each rank offers half the per-GPU rate)
set -o pipefail
export TMPDIR=/tmp MXS_BENCH_VERBOSE=1
timeout -k 10 900 python bench.py --gpus 2 --steps 20 --warmup 5 --qps 21 --disagg-qps 16 \
  > gpurun_out/s4_bench_g2.json 2> gpurun_out/s4_bench_g2.err && echo BENCH2_OK
tail -c 3000 gpurun_out/s4_bench_g2.json
