set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3f/tuned
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_car_norm_gpu.py tests/test_b_tp_gpu.py -x -q --timeout 300 --timeout-method thread -k "rope or splitk or norm or decode_gemm or skinny or mt_gemm or car or tp" > gpurun_out/s3f/tests.log 2>&1
tail -2 gpurun_out/s3f/tests.log
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/s3f/tuned
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29517 -m mxserve.tools.tp_layer_bench --buckets 1,8,32,64 --out gpurun_out/s3f/tp8_layer.json > gpurun_out/s3f/tp8_layer.log 2>&1
