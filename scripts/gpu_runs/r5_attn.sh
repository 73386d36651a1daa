set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5attn}
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill and not gemm" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
PA_VARS=${PA_VARS:-0,2,4,6,3,7} timeout -k 10 240 python -u scripts/prefill_attn_probe.py > $D/probe.jsonl 2>&1
cat $D/probe.jsonl
