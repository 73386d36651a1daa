set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5c
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 1100 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 8 --warmup 3 --qps 8 > gpurun_out/r5c/bench4.json 2> gpurun_out/r5c/bench4.err
tail -c 3000 gpurun_out/r5c/bench4.json
