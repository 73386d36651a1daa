# current tree on MI355X: full GPU suite, smoke(), then a mixed prefill+decode run hunting one-off host stalls
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/fin2 gpurun_out/stall
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin2/suite.log 2>&1 && echo SUITE_OK && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin2/smoke.log 2>&1 && echo SMOKE_OK && \
EAGER=0 SLOW_S=0.045 OSL=64 ROUNDS=1 MXS_STEP_TIMING=1 MNBT=8192 timeout -k 10 300 python3 scripts/prefill_capacity_probe.py > gpurun_out/stall/mixed8192.jsonl 2> gpurun_out/stall/mixed8192.err && echo STALL_OK
rc=$?
tail -2 gpurun_out/fin2/suite.log; tail -1 gpurun_out/fin2/smoke.log; cut -c1-1500 gpurun_out/stall/mixed8192.jsonl
exit $rc
