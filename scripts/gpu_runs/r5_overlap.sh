# mixed-step attention overlap: the kernel-level probe, then the driver-shape bench with and without it
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5ov}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u scripts/probes/attn_overlap_probe.py > $D/probe.jsonl 2>&1
cat $D/probe.jsonl
for ov in ${OVS:-1 0}; do
  MXS_ATTN_OVERLAP=$ov MXS_BENCH_VERBOSE=1 MXS_BENCH_LOG_DIR=$D/ov$ov timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $D/bench_ov$ov.json 2> $D/bench_ov$ov.err
  echo "overlap $ov"; tail -c 1500 $D/bench_ov$ov.json
done
