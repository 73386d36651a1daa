# prefill attention A/B: HEAD build (ab_head/) vs the working tree (K reads pipelined), same box,
# alternating, twice each
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pfab
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "prefill" > gpurun_out/pfab/tests.log 2>&1 || { tail -30 gpurun_out/pfab/tests.log; exit 1; }
tail -1 gpurun_out/pfab/tests.log
for r in 1 2; do
  echo "== head"; (cd ab_head && timeout -k 10 120 python3 scripts/prefill_attn_probe.py 2>/dev/null) || exit 1
  echo "== tree"; timeout -k 10 120 python3 scripts/prefill_attn_probe.py 2>/dev/null || exit 1
done
