set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3k
for q in 50 51; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --qps $q > gpurun_out/s3k/bench_q$q.json 2> gpurun_out/s3k/bench_q$q.err
tail -c 200 gpurun_out/s3k/bench_q$q.json
done
