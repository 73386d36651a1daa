# Headline rocprofv3 kernel trace with exclusive (overlap-split) family shares, then a short
# saturation sweep (served phase off).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6sweep}
mkdir -p $D
OUT=${OUT:-r6sweep}/prof bash scripts/gpu_runs/r6_prof.sh
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
for q in 49 51 53; do
  MXS_BENCH_SERVED=0 timeout -k 10 400 python -u bench.py --steps 40 --warmup 10 --qps $q > $D/bench_q$q.json 2> $D/bench_q$q.err
  tail -c 200 $D/bench_q$q.json
done
