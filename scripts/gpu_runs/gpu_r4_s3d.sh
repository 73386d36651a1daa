set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3d
timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 10 --warmup 3 --qps 20 > gpurun_out/s3d/bench2.json 2> gpurun_out/s3d/bench2.err
python - <<'PY'
import json
d = json.loads(open("gpurun_out/s3d/bench2.json").read().strip().splitlines()[-1])
p = d.get("multi_gpu_probe") or {}
print({k: (v.get("status"), v.get("error"), v.get("skipped")) if isinstance(v, dict) else v for k, v in p.items()})
PY
