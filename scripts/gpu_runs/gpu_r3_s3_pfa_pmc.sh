# counters of the prefill attention kernel (probe run): MFMA busy, VALU / LDS activity, bank conflicts
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc/p1 -o run --output-format csv -- python3 scripts/prefill_attn_probe.py > gpurun_out/pmc/p1.log 2>&1 || { tail -5 gpurun_out/pmc/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD -d gpurun_out/pmc/p2 -o run --output-format csv -- python3 scripts/prefill_attn_probe.py > gpurun_out/pmc/p2.log 2>&1 || { tail -5 gpurun_out/pmc/p2.log; exit 1; }
find gpurun_out/pmc -name "*counter_collection*" | head
