# Step token budget at the default rate, interleaved repeats: 6144 / 7168 / 8192 (served phase off).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6mnbt2}
mkdir -p $D
for rep in 1 2; do
  for b in 6144 7168 8192; do
    MXS_BENCH_SERVED=0 timeout -k 10 400 python -u bench.py --steps 40 --warmup 10 --qps 47 --max-num-batched-tokens $b > $D/bench_b${b}_r${rep}.json 2> $D/bench_b${b}_r${rep}.err
    echo "b=$b rep=$rep done"
  done
done
