#!/usr/bin/env bash
# Interactive chat against an OpenAI-compatible /v1/chat/completions endpoint (final answers only).
#   ./chat.sh [API_URL] [MODEL]        or   API_URL=... MODEL=... ./chat.sh
# Defaults: API_URL=http://127.0.0.1:8000/v1/chat/completions MODEL=Qwen/Qwen3-0.6B
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
export API_URL="${API_URL:-http://127.0.0.1:8000/v1/chat/completions}"
export MODEL="${MODEL:-Qwen/Qwen3-0.6B}"
exec env PYTHONPATH="${HERE}${PYTHONPATH:+:$PYTHONPATH}" python3 -m mxserve.clients.chat "$@"
