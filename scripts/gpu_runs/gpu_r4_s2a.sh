set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2a
export TMPDIR=/tmp
GB_PF=0,8,16,32 GB_SHAPES=qkv,o,down,gate_up timeout -k 10 300 python -u scripts/gemm_probe.py 6400 4096 2048 > gpurun_out/s2a/gemm.jsonl 2> gpurun_out/s2a/gemm.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s2a/dec -o dec -- python3 $GRAFT_REPO_ROOT/scripts/step_profile.py --which decode --tuned --iters 20 > $GRAFT_REPO_ROOT/gpurun_out/s2a/dec.log 2>&1
