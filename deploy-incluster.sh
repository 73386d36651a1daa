#!/usr/bin/env bash
# Deploy a DynamoGraphDeployment manifest into the cluster and expose its frontend via NodePort.
#   ./deploy-incluster.sh --manifest examples/deploy/vllm/agg.yaml [--namespace NS] [--model M]
#                         [--hf-token T] [--nodeport 30000-32767] [--no-wait]
# Env equivalents: MANIFEST_FILE NAMESPACE MODEL HF_TOKEN NODEPORT NO_WAIT, timeouts PODS_TIMEOUT
# ENDPOINTS_TIMEOUT SERVICES_TIMEOUT DEPLOYMENTS_TIMEOUT.  Uses ~/.kube/config (or in-cluster creds).
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
if [[ "${1:-}" == "-h" || "${1:-}" == "--help" ]]; then
  sed -n '2,7p' "$0"; exit 0
fi
command -v python3 >/dev/null || { echo "ERROR: python3 is required" >&2; exit 1; }
exec env PYTHONPATH="${HERE}${PYTHONPATH:+:$PYTHONPATH}" python3 -m mxserve.k8s.deploy "$@"
