# The driver's GPU tier on the current tree: the whole GPU suite (-x, as the driver runs it) + smoke.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-r6suitehead}
mkdir -p $D
( while sleep 50; do echo "alive $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/suite.log 2>&1
tail -2 $D/suite.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
tail -1 $D/smoke.log
