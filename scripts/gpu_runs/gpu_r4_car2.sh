set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/car2 gpurun_out/tuned
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_car_norm_gpu.py > gpurun_out/car2/test_car.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_b_tp_gpu.py tests/test_custom_ar_gpu.py > gpurun_out/car2/test_tp.log 2>&1
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/tuned
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29517 -m mxserve.tools.tp_layer_bench --buckets 1,8,32,64,128 --out gpurun_out/car2/tp8_layer.json > gpurun_out/car2/tp8_layer.log 2>&1
tail -n 3 gpurun_out/car2/*.log
