# current tree on MI355X: full GPU suite, smoke(), the driver's 1-GPU bench line
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/fin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin/suite.log 2>&1 && echo SUITE_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1 && echo SMOKE_OK && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/fin/bench1.json 2> gpurun_out/fin/bench1.err && echo BENCH1_OK
rc=$?
tail -2 gpurun_out/fin/suite.log; tail -1 gpurun_out/fin/smoke.log; cut -c1-600 gpurun_out/fin/bench1.json
exit $rc
