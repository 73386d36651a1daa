set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3j
for i in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s3j/bench_$i.json 2> gpurun_out/s3j/bench_$i.err
tail -c 300 gpurun_out/s3j/bench_$i.json
done
