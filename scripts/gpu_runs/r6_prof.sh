set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6prof}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
MXS_BENCH_SERVED=0 timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/prof -o run -- python3 bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $D/bench.json 2> $D/bench.err
DB=$(find /tmp/prof -name "*.db" | head -1)
python3 scripts/rocpd_stats.py "$DB" --top 60 --csv $D/kernel_stats.csv > $D/kernel_stats.txt
python3 scripts/rocpd_stats.py "$DB" --top 80 --by-grid Cijk > $D/hipblaslt_by_grid.txt
python3 scripts/rocpd_stats.py "$DB" --top 40 --by-grid gemm_pf > $D/gemm_pf_by_grid.txt
python3 scripts/rocpd_stats.py "$DB" --top 40 --by-grid paged > $D/attn_by_grid.txt
python3 scripts/rocpd_stats.py "$DB" --busy 1 --top 0 > $D/gpu_busy.txt
python3 scripts/rocpd_stats.py "$DB" --exclusive > $D/kernel_families_exclusive.txt
head -30 $D/kernel_stats.txt
