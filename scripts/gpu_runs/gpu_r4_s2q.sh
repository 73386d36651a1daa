set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2q
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29517 -m mxserve.tools.tp_layer_bench --buckets 1,8,32,64 --out gpurun_out/s2q/tp8_layer.json > gpurun_out/s2q/tp8_layer.log 2>&1
tail -c 3000 gpurun_out/s2q/tp8_layer.json
