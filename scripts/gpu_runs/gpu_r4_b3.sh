set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/b3 gpurun_out/tuned
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/tuned MXS_DECODE_GEMM_REPORT=$GRAFT_REPO_ROOT/gpurun_out/b3/decode_gemm_report.jsonl
timeout -k 10 400 python -u bench.py --steps 40 --warmup 5 --qps 48 > gpurun_out/b3/q48.json 2> gpurun_out/b3/q48.err
grep 128256 gpurun_out/b3/decode_gemm_report.jsonl | cut -c1-300
tail -c 600 gpurun_out/b3/q48.json
