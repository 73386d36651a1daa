set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/car1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_car_norm_gpu.py > gpurun_out/car1/test_car.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_b_tp_gpu.py tests/test_custom_ar_gpu.py > gpurun_out/car1/test_tp.log 2>&1
tail -n 5 gpurun_out/car1/*.log
