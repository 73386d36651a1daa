# Step token budget 8192 vs the default 6144 at 47 and 50 req/s (served phase off).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6mnbt}
mkdir -p $D
for q in 47 50; do
  for b in 6144 8192; do
    MXS_BENCH_SERVED=0 timeout -k 10 400 python -u bench.py --steps 40 --warmup 10 --qps $q --max-num-batched-tokens $b > $D/bench_q${q}_b${b}.json 2> $D/bench_q${q}_b${b}.err
    tail -c 150 $D/bench_q${q}_b${b}.json
  done
done
