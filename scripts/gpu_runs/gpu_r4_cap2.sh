set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cap2
MXS_CAPACITY_OUT=gpurun_out/cap2/capacity.json timeout -k 10 420 python -u scripts/decode_capacity_probe.py --batches 256,384,512,640,768 --seconds 4 --write > gpurun_out/cap2/decode_cap.jsonl 2> gpurun_out/cap2/decode_cap.err
for q in 46 48; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --qps $q > gpurun_out/cap2/q$q.json 2> gpurun_out/cap2/q$q.err
done
tail -n 2 gpurun_out/cap2/decode_cap.jsonl
