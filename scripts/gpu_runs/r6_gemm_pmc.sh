# PMC counters of gemm_w4 vs gemm_pf on the gate_up shape (two passes of 8 SQ counters each)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6pmc}
mkdir -p $D
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU"
for K in w4 pf; do
  for i in 1 2; do
    eval PP=\$P$i
    rm -rf /tmp/pmc_${K}_$i
    timeout -s KILL 90 rocprofv3 --pmc $PP --output-format csv -d /tmp/pmc_${K}_$i -o run -- python3 scripts/probes/gemm_pmc.py $K ${SHAPE:-6592 16384 2048 1} 10 > $D/pmc_${K}_$i.log 2>&1
    f=$(find /tmp/pmc_${K}_$i -name "*counter_collection.csv" | head -1)
    cp "$f" $D/counters_${K}_pass$i.csv
  done
done
ls -la $D
