# gemm_w4 numerics (GPU tests) then the projection probe against gemm_pf and hipBLASLt
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6w4}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm_w4" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -3 $D/tests.log
timeout -k 10 400 python -u scripts/probes/w4_probe.py > $D/probe.jsonl 2> $D/probe.err
cat $D/probe.jsonl | cut -c1-400
