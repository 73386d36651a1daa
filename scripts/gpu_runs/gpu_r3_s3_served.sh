# the driver's default 1-GPU line at the new operating point (QPS 44), then the served path at the
# same QPS: frontend (4 processes) -> worker (streamer process) over HTTP/SSE, open-loop client
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/sv
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "prefill or engine or Engine or generate or rope" > gpurun_out/sv/tests.log 2>&1 || { tail -30 gpurun_out/sv/tests.log; exit 1; }
tail -1 gpurun_out/sv/tests.log
timeout -k 10 120 python3 scripts/prefill_attn_probe.py 2>/dev/null || exit 1
timeout -k 10 120 python3 scripts/prefill_attn_probe.py 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/sv/bench_default.json 2> gpurun_out/sv/bench_default.err || exit 1
cut -c1-900 gpurun_out/sv/bench_default.json
timeout -k 10 480 bash scripts/served_bench.sh 44 1800 gpurun_out/sv/served_q44 > gpurun_out/sv/served.log 2>&1 || { tail -30 gpurun_out/sv/served.log; exit 1; }
tail -20 gpurun_out/sv/served.log
ls gpurun_out/sv/served_q44
