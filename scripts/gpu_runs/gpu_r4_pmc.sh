set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
P="python3 scripts/gemm_counter_probe.py"
for k in v7 pf lib; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc/a_$k -o run --output-format csv -- $P $k 8192 2048 8192 > gpurun_out/pmc/a_$k.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU -d gpurun_out/pmc/b_$k -o run --output-format csv -- $P $k 8192 2048 8192 > gpurun_out/pmc/b_$k.log 2>&1
done
ls -R gpurun_out/pmc | head -40
