# The default bench twice more on one box (run-to-run spread of the headline line).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6rep}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
for rep in 1 2; do
  timeout -k 10 600 python -u bench.py > $D/bench_default_r${rep}.json 2> $D/bench_default_r${rep}.err
done
