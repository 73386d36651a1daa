set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GB_VARIANTS=0,3,4,5
mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_big_probe.py 8192 > gpurun_out/gemm_big_probe2.log 2>&1; rc=$?; grep '^{' gpurun_out/gemm_big_probe2.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['proj'], d['M'], {k:v for k,v in d.items() if k.endswith('_us')})"; exit $rc
