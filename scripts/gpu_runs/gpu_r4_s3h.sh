set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3h
for q in 4 16; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 --qps $q > gpurun_out/s3h/new_q$q.json 2> gpurun_out/s3h/new_q$q.err
MXS_TUNED_DIR=$GRAFT_REPO_ROOT/tmp_ab/old timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 --qps $q > gpurun_out/s3h/old_q$q.json 2> gpurun_out/s3h/old_q$q.err
done
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s3h/engine_tests.log 2>&1
tail -2 gpurun_out/s3h/engine_tests.log
