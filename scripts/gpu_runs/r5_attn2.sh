set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5attn2}
mkdir -p $D
timeout -k 10 120 python -u scripts/probes/pf_spike_diag.py > $D/diag.txt 2>&1 || { cat $D/diag.txt; exit 1; }
cat $D/diag.txt
PA_VARS=${PA_VARS:-0,2,4,6,3,7} timeout -k 10 240 python -u scripts/prefill_attn_probe.py > $D/probe.jsonl 2>&1
cat $D/probe.jsonl
