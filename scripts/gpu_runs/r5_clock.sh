# effective clock of the prefill attention and gemm_pf kernels: GRBM_GUI_ACTIVE / 8 XCDs / kernel time
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5clock}
mkdir -p $D
PA_SHAPES=1x8192,2x4096 PA_VARS=256,0 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $D/attn -o run -- python3 scripts/prefill_attn_probe.py > $D/attn.log 2>&1
find $D/attn -name "*.csv" | head
