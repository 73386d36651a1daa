# End-of-round verification: the whole GPU suite (no -x: every failure listed), smoke, the default
# bench (served phase on) and a rocprofv3 kernel trace of the headline bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6final}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $D/suite.log 2>&1
rc=$?
tail -3 $D/suite.log
# 1: test failures (keep going); anything else (timeout, abort, segfault): stop here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo smoke failed; tail -5 $D/smoke.log; exit 3; }
tail -1 $D/smoke.log
timeout -k 10 600 python -u bench.py > $D/bench.json 2> $D/bench.err || { echo bench failed; tail -5 $D/bench.err; exit 4; }
tail -c 400 $D/bench.json
OUT=${OUT:-r6final}/prof bash scripts/gpu_runs/r6_prof.sh
