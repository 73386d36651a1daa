# decode attention A/B: HEAD (ab_head/, occupancy 3) vs tree (D = 64 pinned at 4 waves/SIMD), alternating
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "decode and not gemm" > /tmp/dtests.log 2>&1 || { tail -30 /tmp/dtests.log; exit 1; }
tail -1 /tmp/dtests.log
for r in 1 2; do
  echo "== head"; (cd ab_head && timeout -k 10 120 python3 scripts/decode_attn_probe.py 2>/dev/null) || exit 1
  echo "== tree"; timeout -k 10 120 python3 scripts/decode_attn_probe.py 2>/dev/null || exit 1
done
