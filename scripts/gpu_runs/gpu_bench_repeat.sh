# variance of the driver's short bench: repeated --steps 20 --warmup 5 runs
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
out=gpurun_out/bench_repeat.jsonl; : > $out
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} 2> gpurun_out/br.err | tail -1 >> $out || exit 1
  tail -1 $out | cut -c1-120
done
