set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cup1
timeout -k 10 300 python -u scripts/cu_partition_probe.py > gpurun_out/cup1/probe.jsonl 2> gpurun_out/cup1/probe.err
cat gpurun_out/cup1/probe.jsonl
