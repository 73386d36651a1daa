# split-KV prefill attention (VAR 128): tests, then A/B against VAR 0 and the default launch (-1)
# over shapes and split rules (CFGS: "floor:rel" pairs)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r5split}
mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill_split or prefill_softmax_variants or prefill_fp8 or paged_prefill" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
for cfg in ${CFGS:-8:0 8:1 4:1}; do
  MXS_PF_SPLIT_MIN=${cfg%:*} MXS_PF_SPLIT_REL=${cfg#*:} PA_VARS=${PA_VARS:-0,128,-1} \
    PA_SHAPES=${PA_SHAPES:-1x1024,1x2048,1x4096,2x4096,1x6144,4x2048,1x2048x128,1x4096x128,2x4096x128} \
    timeout -k 10 240 python -u scripts/prefill_attn_probe.py > $D/probe_$cfg.jsonl 2>&1
  echo "split rule $cfg"; cat $D/probe_$cfg.jsonl
done
