# the driver's N=2 command shape on one shared MI355X (2 ranks at QPS 21 each): agg + disagg + probe,
# whole-job wall time, current build
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 MXS_BENCH_VERBOSE=1
mkdir -p gpurun_out/b3
t0=$(date +%s)
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --qps 21 > gpurun_out/b3/bench2.json 2> gpurun_out/b3/bench2.err
rc=$?
echo "wall_s=$(( $(date +%s) - t0 )) rc=$rc" | tee gpurun_out/b3/bench2.wall
tail -c 2500 gpurun_out/b3/bench2.json
exit $rc
