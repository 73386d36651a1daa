# Decode attention HBM traffic from the L2's fetch counters (rocprofv3 --pmc FETCH_SIZE) at the
# headline's running-set sizes: bytes fetched per dispatch against the dispatch's duration.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6decpmc}
mkdir -p $D
DP_BATCHES=256,448 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmc -o run -- python3 scripts/probes/decode_plan_probe.py > $D/probe.jsonl 2> $D/probe.err
find /tmp/pmc -name "*.db" -exec cp {} $D/pmc_fetch_size.db \;
ls -la $D
