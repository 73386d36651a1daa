# gemm_pf 224-row token tiles: numerics, probe against the other heights and hipBLASLt, then a
# retune of the prefill_pf table with the new candidates and a bench on the retuned table.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6pf224}
mkdir -p $D/tuned
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm_pf" > $D/tests.log 2>&1
tail -2 $D/tests.log
W4_MS=6144,6592 W4_PROJ=qkv,o,down,gate_up W4_ROUNDS=5 timeout -k 10 300 python -u scripts/probes/w4_probe.py > $D/probe.jsonl 2> $D/probe.err
MXS_RETUNE=prefill_pf MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 \
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $D/bench_retune.json 2> $D/bench_retune.err
ls $D/tuned
MXS_TUNED_DIR=$GRAFT_REPO_ROOT/$D/tuned MXS_BENCH_SERVED=0 timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $D/bench_after.json 2> $D/bench_after.err
tail -c 600 $D/bench_after.json
