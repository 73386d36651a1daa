set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2t/tuned
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "skinny or decode_gemm or linear_rope_and_cache_splitk or linear_add_rms_norm" > gpurun_out/s2t/kt.log 2>&1 || true
tail -5 gpurun_out/s2t/kt.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29517 -m mxserve.tools.tp_layer_bench --buckets 1,8,32,64 --out gpurun_out/s2t/tp8_layer.json > gpurun_out/s2t/tp8_layer.log 2>&1
python - <<'PY'
import json
d = json.load(open("gpurun_out/s2t/tp8_layer.json"))
for r in d["rows"]:
    print(r["M"], r["gemm_chain_us"], round(r["gemm_chain_us"] / r["floor_us"], 2), {k: (v["us"], v["kernel"]) for k, v in r["gemms"].items()})
PY
