# hipBLASLt solution sweep at decode batch sizes (scripts/probes/hblt_probe.py).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6hbltdec}
mkdir -p $D
HB_GRAPH=1 HB_MS=64,128,256,320,384,448 HB_PROJ=qkv,o,down,gate_up timeout -k 10 500 python -u scripts/probes/hblt_probe.py > $D/probe.jsonl 2> $D/probe.err
