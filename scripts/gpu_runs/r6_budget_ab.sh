# Same-box A/B of the step budget on the driver's default bench shape (100 steps, 20 warmup; served
# off), packaged tables covering both budgets, interleaved repeats.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6budgetab}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
for rep in 1 2; do
  for b in 6144 7168; do
    MXS_BENCH_SERVED=0 timeout -k 10 500 python -u bench.py --max-num-batched-tokens $b > $D/bench_b${b}_r${rep}.json 2> $D/bench_b${b}_r${rep}.err
  done
done
