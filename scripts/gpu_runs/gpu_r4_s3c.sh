set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3c
timeout -k 10 400 python -u scripts/decode_hb_forms_probe.py > gpurun_out/s3c/probe.jsonl 2> gpurun_out/s3c/probe.err
