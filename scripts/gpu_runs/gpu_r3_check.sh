# round 3: GPU suite, smoke(), the driver's 1-GPU bench line, then a 2-rank shared-GPU bench
# (exercises the wall-budget guard and the probe deadline on the GPU)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_suite.log 2>&1 && echo SUITE_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench1.json 2> gpurun_out/r3_bench1.err && echo BENCH1_OK && \
{ s=$(date +%s); timeout -k 10 560 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r3_bench2.json 2> gpurun_out/r3_bench2.err; r=$?; echo "wall_s=$(( $(date +%s) - s )) rc=$r" > gpurun_out/r3_bench2.wall; [ $r -eq 0 ]; } && echo BENCH2_OK
rc=$?
tail -2 gpurun_out/r3_suite.log; tail -1 gpurun_out/r3_smoke.log; cut -c1-600 gpurun_out/r3_bench1.json; cat gpurun_out/r3_bench2.wall 2>/dev/null
exit $rc
