set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2v/tuned
MXS_DECODE_GEMM_MAX_M=448 MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/s2v/tuned timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2v/m448_a.json 2> gpurun_out/s2v/m448_a.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2v/m384.json 2> gpurun_out/s2v/m384.err
MXS_DECODE_GEMM_MAX_M=448 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/s2v/tuned timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2v/m448_b.json 2> gpurun_out/s2v/m448_b.err
ls gpurun_out/s2v/tuned
