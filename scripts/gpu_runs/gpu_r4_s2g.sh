set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2g
export TMPDIR=/tmp
P="python3 scripts/gemm_pf_counter_probe.py"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/s2g/a -o run --output-format csv -- $P 8192 16384 2048 1 16 > gpurun_out/s2g/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU -d gpurun_out/s2g/b -o run --output-format csv -- $P 8192 16384 2048 1 16 > gpurun_out/s2g/b.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_FLAT -d gpurun_out/s2g/c -o run --output-format csv -- $P 8192 16384 2048 1 16 > gpurun_out/s2g/c.log 2>&1 || true
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/s2g/t -o run -- $P 8192 16384 2048 1 16 20 > gpurun_out/s2g/t.log 2>&1
ls -R gpurun_out/s2g | head -30
