set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tpg
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "skinny or decode_gemm_all" > gpurun_out/tpg/tests.log 2>&1
tail -n 2 gpurun_out/tpg/tests.log
timeout -k 10 400 python -u scripts/tp_shard_gemm_probe.py > gpurun_out/tpg/probe.jsonl 2> gpurun_out/tpg/probe.err
cut -c1-600 gpurun_out/tpg/probe.jsonl
for r in 1 2; do
  MXS_PREFILL_PRIO=0 timeout -k 10 120 python scripts/prefill_attn_probe.py > gpurun_out/tpg/attn_prio0_$r.jsonl
  MXS_PREFILL_PRIO=1 timeout -k 10 120 python scripts/prefill_attn_probe.py > gpurun_out/tpg/attn_prio1_$r.jsonl
done
head -n 2 gpurun_out/tpg/attn_prio*.jsonl
