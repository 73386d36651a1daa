# hipBLASLt solution sweep on the prefill projections (scripts/probes/hblt_probe.py).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6hblt}
mkdir -p $D
timeout -k 10 700 python -u scripts/probes/hblt_probe.py > $D/probe.jsonl 2> $D/probe.err
