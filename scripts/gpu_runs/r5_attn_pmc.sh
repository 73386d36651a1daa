set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5pmc}
mkdir -p $D
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"
for V in 0 16; do
  for i in 1 2; do
    eval PP=\$P$i
    rm -rf /tmp/pmc_${V}_$i
    PA_CASE=1 PA_VARS=$V timeout -s KILL 90 rocprofv3 --pmc $PP --output-format csv -d /tmp/pmc_${V}_$i -o run -- python3 scripts/prefill_attn_probe.py > $D/pmc_${V}_$i.log 2>&1
    f=$(find /tmp/pmc_${V}_$i -name "*counter_collection.csv" | head -1)
    cp "$f" $D/counters_var${V}_pass$i.csv
  done
done
ls -la $D
