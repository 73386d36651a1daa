set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tp8 gpurun_out/tuned
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/tuned
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29517 -m mxserve.tools.tp_layer_bench --buckets 1,8,32,64,128 --out gpurun_out/tp8/tp8_layer.json > gpurun_out/tp8/tp8_layer.log 2>&1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29518 -m mxserve.tools.tp_layer_bench --buckets 1,8,64 --out gpurun_out/tp8/tp2_layer.json > gpurun_out/tp8/tp2_layer.log 2>&1
grep -h '^{' gpurun_out/tp8/*.log | cut -c1-400
