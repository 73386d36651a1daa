# 1-GPU headline bench (with the served phase), then the N = 2 rehearsal (ranks sharing the GPU:
# agg + disagg 1P+1D at QPS 20 per rank, TTFT breakdown), each step under its own limit.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6bm}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
if [ "${SKIP1:-0}" != 1 ]; then
MXS_BENCH_VERBOSE=1 MXS_BENCH_LOG_DIR=$D timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $D/bench1.json 2> $D/bench1.err
tail -c 1200 $D/bench1.json
fi
MXS_BENCH_VERBOSE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 8 --warmup 3 --qps 20 > $D/bench2.json 2> $D/bench2.err
tail -c 1500 $D/bench2.json
