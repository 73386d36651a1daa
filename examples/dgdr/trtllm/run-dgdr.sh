#!/usr/bin/env bash
# Submit the SLA-driven DynamoGraphDeploymentRequest: ConfigMap from the DGD template, apply the
# DGDR (the mxserve operator profiles + renders + applies), expose the frontend on a NodePort.
# Env: NAMESPACE CONFIGMAP_NAME DISAGG_FILE DGDR_FILE FRONTEND_NODEPORT (default 30081)
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
ROOT="$(cd "$HERE/../../.." && pwd)"
export DISAGG_FILE="${DISAGG_FILE:-$HERE/disagg.yaml}" DGDR_FILE="${DGDR_FILE:-$HERE/dgdr.yaml}"
exec env PYTHONPATH="${ROOT}${PYTHONPATH:+:$PYTHONPATH}" python3 -m mxserve.k8s.run_dgdr "$@"
