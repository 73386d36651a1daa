# Step-level A/B: prefill-attention variant choice and the side-stream overlap under the headline's
# mixed steps (scripts/probes/step_ab_probe.py).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6stepab}
mkdir -p $D
STEP_MODES=base,var0,no_overlap,no_overlap_var0 timeout -k 10 500 python -u scripts/probes/step_ab_probe.py > $D/step.jsonl 2> $D/step.err
