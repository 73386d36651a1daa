# the multi-GPU probe alone with N ranks on this box (ranks share the GPU when it has fewer than N)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
N=${1:-2}
mkdir -p gpurun_out
pids=()
for r in $(seq 0 $((N-1))); do
  (echo "go 29911" | env MASTER_ADDR=127.0.0.1 MASTER_PORT=29911 RANK=$r LOCAL_RANK=$r WORLD_SIZE=$N \
     timeout -k 10 600 python -m mxserve.tools.mgpu_probe > gpurun_out/probe_r$r.out 2> gpurun_out/probe_r$r.err) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
cat gpurun_out/probe_r0.out
exit $rc
