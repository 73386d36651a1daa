set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3i/tuned
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/s3i/tuned
timeout -k 10 500 python -u scripts/retune_decode_buckets.py --buckets 96,128,160,192,224,256,320,384,448 > gpurun_out/s3i/retune.jsonl 2> gpurun_out/s3i/retune.err
