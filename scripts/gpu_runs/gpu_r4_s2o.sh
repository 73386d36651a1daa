set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2o
timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/s2o/stage.jsonl 2>&1
MXS_PF_ATTN_NOSTAGE=1 timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/s2o/nostage.jsonl 2>&1
timeout -k 10 200 python -u scripts/prefill_attn_probe.py > gpurun_out/s2o/stage2.jsonl 2>&1
cat gpurun_out/s2o/stage.jsonl gpurun_out/s2o/nostage.jsonl gpurun_out/s2o/stage2.jsonl | grep "{"
