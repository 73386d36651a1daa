# round 3: per-kernel breakdown of prefill / decode steps, then the scheduling operating points
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/sched
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_prefill -o run -- python3 scripts/step_profile.py --which prefill --iters 10 > gpurun_out/prof_prefill.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_decode -o run -- python3 scripts/step_profile.py --which decode --iters 20 > gpurun_out/prof_decode.log 2>&1 || exit 1
for cfg in "42 8192 384" "42 4096 384" "46 8192 384" "46 4096 512" "48 4096 512" "48 8192 512"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --qps $1 --max-num-batched-tokens $2 --max-num-seqs $3 --steps 20 --warmup 5 \
    > gpurun_out/sched/q$1_c$2_s$3.json 2> gpurun_out/sched/q$1_c$2_s$3.err || exit 1
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/sched/q$1_c$2_s$3.json').read().strip().splitlines()[-1]);print('$cfg', d['value'], d['ttft_p50_ms'], d['ttft_p90_ms'], d['itl_p50_ms'], d['itl_p90_ms'], d['running_mean'])"
done
