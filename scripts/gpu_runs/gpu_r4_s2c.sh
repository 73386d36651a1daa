set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2b
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "rope_kv_only or gemm_pf" > gpurun_out/s2b/kt.log 2>&1 || true
grep -E "PASSED|FAILED|Error" gpurun_out/s2b/kt.log | tail -30
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "fused_prefill_chain" > gpurun_out/s2b/et.log 2>&1 || true
grep -E "PASSED|FAILED|Error" gpurun_out/s2b/et.log | tail -10
timeout -k 10 300 python -u scripts/pf_fused_probe.py 2048 4096 6400 8192 > gpurun_out/s2b/pf_fused.jsonl 2> gpurun_out/s2b/pf_fused.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s2b/dec -o dec -- python3 $GRAFT_REPO_ROOT/scripts/step_profile.py --which both --tuned --iters 20 > $GRAFT_REPO_ROOT/gpurun_out/s2b/prof.log 2>&1
