set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2r
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 8 --warmup 3 --qps 8 > gpurun_out/s2r/bench4.json 2> gpurun_out/s2r/bench4.err
python - <<'PY'
import json
d = json.loads(open("gpurun_out/s2r/bench4.json").read().strip().splitlines()[-1])
print({k: d.get(k) for k in ("value", "n_gpus", "ttft_p50_ms", "itl_p90_ms")})
print(json.dumps(d.get("agg_vs_disagg"))[:800])
p = d.get("multi_gpu_probe") or {}
print({k: (v.get("status"), v.get("error"), v.get("skipped")) if isinstance(v, dict) else v for k, v in p.items()})
PY
mkdir -p gpurun_out/s2r/tuned
MXS_TUNED_SAVE=1 MXS_TUNED_DIR=$GRAFT_REPO_ROOT/gpurun_out/s2r/tuned timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/s2r/bench1_tune.json 2> gpurun_out/s2r/bench1_tune.err
ls gpurun_out/s2r/tuned
