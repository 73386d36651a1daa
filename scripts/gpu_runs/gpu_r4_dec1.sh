set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dec1
GB_SHAPES=lm_head GB_PF=0,8,16,32 GB_VARIANTS= timeout -k 10 240 python -u scripts/gemm_big_probe.py 128 256 384 512 > gpurun_out/dec1/lmhead.jsonl
MXS_CAPACITY_OUT=gpurun_out/dec1/capacity.json timeout -k 10 600 python -u scripts/decode_capacity_probe.py --rates 60,70,80,90,100 --seconds 10 --write > gpurun_out/dec1/decode_cap.jsonl 2> gpurun_out/dec1/decode_cap.err
tail -n 3 gpurun_out/dec1/*.jsonl
