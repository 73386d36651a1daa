set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dec2
GB_SHAPES=qkv,o,gate_up,down,lm_head GB_PF=0,4,8,16 GB_VARIANTS= timeout -k 10 300 python -u scripts/gemm_big_probe.py 256 384 > gpurun_out/dec2/pf_decode.jsonl
cut -c1-600 gpurun_out/dec2/pf_decode.jsonl
