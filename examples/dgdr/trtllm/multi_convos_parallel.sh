#!/usr/bin/env bash
# N parallel 3-turn conversations against /v1/chat/completions with bounded concurrency.
# Env: API_URL MODEL TEMPERATURE(0.7) MAX_TOKENS(200) NUM_CONVOS(10) CONCURRENCY(5); exit 1 on any failure.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
ROOT="$(cd "$HERE/../../.." && pwd)"
exec env PYTHONPATH="${ROOT}${PYTHONPATH:+:$PYTHONPATH}" python3 -m mxserve.clients.multi_convos
