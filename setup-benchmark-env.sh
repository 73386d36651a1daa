#!/usr/bin/env bash
# Python environment for run-benchmarks.sh.  Offline-capable: the benchmark harness ships in this
# repo (benchmarks/utils), so nothing is cloned; ./dynamo points at the repo root so the
# reference's `pushd dynamo; python3 -m benchmarks.utils.benchmark` layout keeps working.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
cd "$HERE"
if [[ ! -d .venv ]]; then
  python3 -m venv --system-site-packages .venv
fi
# shellcheck disable=SC1091
source .venv/bin/activate
python3 - <<'PY'
import importlib, sys
missing = [m for m in ("numpy", "httpx", "aiohttp") if importlib.util.find_spec(m) is None]
if missing:
    sys.exit("missing python packages: " + ", ".join(missing) + " (pip install them into .venv)")
PY
[[ -e dynamo ]] && [[ ! -L dynamo ]] && [[ ! -f dynamo/__init__.py ]] && { echo "./dynamo exists and is not ours" >&2; exit 1; }
echo "Benchmark environment ready.  Activate with: source .venv/bin/activate"
