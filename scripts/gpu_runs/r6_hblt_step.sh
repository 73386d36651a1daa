# Step-level A/B of the tuned hipBLASLt solutions, tables from profiles/r6/hblt/tuned.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6hblstep}
mkdir -p $D
MXS_TUNED_DIR=$GRAFT_REPO_ROOT/profiles/r6/hblt/tuned timeout -k 10 500 python -u scripts/probes/step_ab_probe.py > $D/step.jsonl 2> $D/step.err
