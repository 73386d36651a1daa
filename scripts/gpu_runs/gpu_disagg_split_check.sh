# disagg phase with 2P+2D (every decode rank balances over both prefill ranks) (4 ranks sharing the GPU, low rate)
set -o pipefail
export TMPDIR=/tmp MXS_BENCH_VERBOSE=1
timeout -k 10 600 python bench.py --gpus 4 --mode disagg --disagg-qps 8 --qps 8 \
  --probe-timeout-s 0 --steps 10 --warmup 2 > gpurun_out/disagg_2p2d.json 2> gpurun_out/disagg_2p2d.err && echo OK
tail -c 2500 gpurun_out/disagg_2p2d.json
