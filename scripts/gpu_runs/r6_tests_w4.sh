# new GPU tests (long-context prefill forms, TP-4 vs default TP-1 chain, gemm_w4) + the w4 probe
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6tw}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_c_tp8_gpu.py -x -v --timeout 300 --timeout-method thread -k "long_context or gemm_w4 or tp4_engine" > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -3 $D/tests.log
W4_PROJ=gate_up,qkv W4_MS=4096,6592 timeout -k 10 300 python -u scripts/probes/w4_probe.py > $D/probe.jsonl 2> $D/probe.err
cut -c1-300 $D/probe.jsonl
