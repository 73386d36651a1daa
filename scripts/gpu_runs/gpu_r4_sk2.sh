set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sk2 gpurun_out/tuned
export MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/tuned MXS_DECODE_GEMM_REPORT=$GRAFT_REPO_ROOT/gpurun_out/sk2/decode_gemm_report.jsonl
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --qps 48 > gpurun_out/sk2/q48.json 2> gpurun_out/sk2/q48.err
grep '"M": \(1\|2\|4\|8\|16\),' gpurun_out/sk2/decode_gemm_report.jsonl | cut -c1-260
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29518 -m mxserve.tools.tp_layer_bench --buckets 1,8,32,64 --out gpurun_out/sk2/tp2_layer.json > gpurun_out/sk2/tp2_layer.log 2>&1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29519 -m mxserve.tools.tp_layer_bench --buckets 1,8,32,64 --out gpurun_out/sk2/tp8_layer.json > gpurun_out/sk2/tp8_layer.log 2>&1
grep -h '^{' gpurun_out/sk2/tp*_layer.log | cut -c1-500
