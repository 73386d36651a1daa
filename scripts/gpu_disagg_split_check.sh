# disagg phase with one prefill rank serving three decode ranks (4 ranks sharing the GPU, low rate)
set -o pipefail
export TMPDIR=/tmp MXS_BENCH_VERBOSE=1
timeout -k 10 600 python bench.py --gpus 4 --mode disagg --disagg-prefill-ranks 1 --disagg-qps 8 --qps 8 \
  --probe-timeout-s 0 --steps 10 --warmup 2 > gpurun_out/disagg_1p3d.json 2> gpurun_out/disagg_1p3d.err && echo OK
tail -c 2500 gpurun_out/disagg_1p3d.json
