set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3g/tuned
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/s3g/tuned
timeout -k 10 500 python -u scripts/retune_decode_buckets.py > gpurun_out/s3g/retune.jsonl 2> gpurun_out/s3g/retune.err
