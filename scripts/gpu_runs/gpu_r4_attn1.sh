set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/attn1
timeout -k 10 120 python scripts/prefill_attn_probe.py > gpurun_out/attn1/probe.jsonl
PA_CASE=1 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d /tmp/pmc1 -o p1 -- python3 scripts/prefill_attn_probe.py > /dev/null 2>&1
PA_CASE=1 timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY --output-format csv -d /tmp/pmc2 -o p2 -- python3 scripts/prefill_attn_probe.py > /dev/null 2>&1
find /tmp/pmc1 /tmp/pmc2 -name "*counter_collection.csv" -exec cp {} gpurun_out/attn1/ \;
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --qps 48 > gpurun_out/attn1/bench_q48.json 2> gpurun_out/attn1/bench_q48.err
cat gpurun_out/attn1/probe.jsonl; ls gpurun_out/attn1
