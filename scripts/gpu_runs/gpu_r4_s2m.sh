set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2m
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2m/new1.json 2> gpurun_out/s2m/new1.err
MXS_ROPE_SPLIT=0 MXS_SAMPLED_QROPE=0 MXS_KV_T16_LEGACY=1 MXS_PF_FUSED=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2m/old.json 2> gpurun_out/s2m/old.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2m/new2.json 2> gpurun_out/s2m/new2.err
