# the driver's N=1 command (defaults) on the current build: agg line + hosted disagg + probe
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/def
t0=$(date +%s)
timeout -k 10 800 python bench.py > gpurun_out/def/bench1.json 2> gpurun_out/def/bench1.err
rc=$?
echo "wall_s=$(( $(date +%s) - t0 )) rc=$rc" | tee gpurun_out/def/bench1.wall
tail -c 1500 gpurun_out/def/bench1.json
exit $rc
