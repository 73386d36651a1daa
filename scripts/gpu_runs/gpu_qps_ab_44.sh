# operating-point check: the driver's short bench (20 steps of 50 iterations) at QPS 44 vs 42, interleaved on one box
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/qps_ab.jsonl
: > $out
for q in 44 42 44 42; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --qps $q > gpurun_out/qps_$q.json 2> gpurun_out/qps_$q.err || exit $?
  tail -n 1 gpurun_out/qps_$q.json | tee -a $out
done
