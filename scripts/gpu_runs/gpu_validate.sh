set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s4_gpu_suite.log 2>&1 && echo SUITE_OK && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s4_bench20.json 2> gpurun_out/s4_bench20.err && echo BENCH_OK
tail -3 gpurun_out/s4_gpu_suite.log; cat gpurun_out/s4_bench20.json
