# Where the mixed-step attention overlap stops paying: chunk-size sweep, one and two prefill sequences.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6ovl}
mkdir -p $D
MS_CASES="300:4250:3000:0,300:4250:4000:0,300:4250:4500:0,300:4250:5000:0,300:4250:5700:0,400:4250:4600:0,450:4250:5600:0,300:4250:1700:2300+4000:0,400:4250:2000:2000+3500:0,300:4250:800:3200+4000:0+900:0" \
STEP_MODES=base,no_overlap timeout -k 10 500 python -u scripts/probes/step_ab_probe.py > $D/step.jsonl 2> $D/step.err
