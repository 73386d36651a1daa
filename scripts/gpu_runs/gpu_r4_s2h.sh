set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2h
timeout -k 10 240 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_c_tp8_gpu.py -k "tp4_engine" > gpurun_out/s2h/tp4.log 2>&1 || true
grep -E "PASSED|FAILED" gpurun_out/s2h/tp4.log | tail -3
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --qps 20 > gpurun_out/s2h/bench2.json 2> gpurun_out/s2h/bench2.err
tail -c 1500 gpurun_out/s2h/bench2.json
