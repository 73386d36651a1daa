# prefill attention with conflict-free LDS swizzles: kernel tests, probe x2, bank-conflict counters
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/swz
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "prefill" > gpurun_out/swz/tests.log 2>&1 || { tail -30 gpurun_out/swz/tests.log; exit 1; }
tail -1 gpurun_out/swz/tests.log
timeout -k 10 120 python3 scripts/prefill_attn_probe.py 2>/dev/null || exit 1
timeout -k 10 120 python3 scripts/prefill_attn_probe.py 2>/dev/null || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/swz/p1 -o run --output-format csv -- python3 scripts/prefill_attn_probe.py > gpurun_out/swz/p1.log 2>&1 || { tail -5 gpurun_out/swz/p1.log; exit 1; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/swz/p1/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, v in agg.items():
    if "prefill" in k:
        n = cnt[(k, next(iter(v)))]
        print(k, {c: round(x / n) for c, x in v.items()})
PY
