set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2d gpurun_out/s2d/tuned
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "rope_kv_only or gemm_pf" > gpurun_out/s2d/kt.log 2>&1 || true
grep -E "PASSED|FAILED|Error" gpurun_out/s2d/kt.log | tail -40
timeout -k 10 240 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "fused_prefill_chain" > gpurun_out/s2d/et.log 2>&1 || true
grep -E "PASSED|FAILED|Error|assert" gpurun_out/s2d/et.log | tail -10
timeout -k 10 300 python -u scripts/pf_fused_probe.py 2048 6400 > gpurun_out/s2d/pf_fused.jsonl 2> gpurun_out/s2d/pf_fused.err
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/s2d/tuned
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2d/bench_new.json 2> gpurun_out/s2d/bench_new.err
MXS_PF_FUSED=0 MXS_KV_T16_LEGACY=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2d/bench_old.json 2> gpurun_out/s2d/bench_old.err
tail -c 400 gpurun_out/s2d/bench_new.json gpurun_out/s2d/bench_old.json
