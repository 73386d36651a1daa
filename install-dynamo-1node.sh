#!/usr/bin/env bash
# Install the mxserve serving platform on a single-node cluster with MI355X GPUs:
#   1) default StorageClass (local-path) for model-cache PVCs
#   2) DGD / DGDR / DCD CRDs (group nvidia.com/v1alpha1, so the example manifests apply unchanged)
#   3) the mxserve operator (replaces the Dynamo operator + etcd + NATS: workers register with the
#      frontend directly, no external state store)
#   4) AMD GPU Operator (or the ROCm k8s-device-plugin DaemonSet) and wait for amd.com/gpu allocatable
# 2) and 3) are two Helm releases when helm is on PATH (deploy/helm/mxserve-crds, mxserve-platform;
# the reference's CRD + platform releases): upgrade = re-run with a new RELEASE_VERSION, rollback =
# `helm rollback mxserve-platform -n $NAMESPACE`, removal = `UNINSTALL=true ./install-dynamo-1node.sh`
# (the CRDs, and with them every DGD, only with PURGE_CRDS=true).  Without helm (MXS_USE_HELM=false
# or no binary) the same objects are applied with kubectl.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"

NAMESPACE="${NAMESPACE:-dynamo-system}"
RELEASE_VERSION="${RELEASE_VERSION:-0.1.0}"                       # mxserve image tag
MXS_IMAGE="${MXS_IMAGE:-mxserve/mxserve-rocm:${RELEASE_VERSION}}"
NAMESPACE_RESTRICTED_OPERATOR="${NAMESPACE_RESTRICTED_OPERATOR:-false}"
PROMETHEUS_ENDPOINT="${PROMETHEUS_ENDPOINT:-http://prometheus-kube-prometheus-prometheus.monitoring.svc.cluster.local:9090}"
LOCAL_PATH_MANIFEST_URL="${LOCAL_PATH_MANIFEST_URL:-https://raw.githubusercontent.com/rancher/local-path-provisioner/master/deploy/local-path-storage.yaml}"
GPU_RESOURCE="${GPU_RESOURCE:-amd.com/gpu}"
GPU_OPERATOR_NS="${GPU_OPERATOR_NS:-kube-amd-gpu}"
GPU_OPERATOR_RELEASE="${GPU_OPERATOR_RELEASE:-amd-gpu-operator}"
AMD_HELM_REPO_NAME="${AMD_HELM_REPO_NAME:-rocm}"
AMD_HELM_REPO_URL="${AMD_HELM_REPO_URL:-https://rocm.github.io/gpu-operator}"
GPU_OPERATOR_MODE="${GPU_OPERATOR_MODE:-operator}"                 # operator | device-plugin | skip
ROCM_DEVICE_PLUGIN_URL="${ROCM_DEVICE_PLUGIN_URL:-https://raw.githubusercontent.com/ROCm/k8s-device-plugin/master/k8s-ds-amdgpu-dp.yaml}"
GPU_OPERATOR_HELM_TIMEOUT="${GPU_OPERATOR_HELM_TIMEOUT:-15m}"
GPU_ALLOCATABLE_WAIT_ATTEMPTS="${GPU_ALLOCATABLE_WAIT_ATTEMPTS:-120}"
GPU_ALLOCATABLE_WAIT_INTERVAL="${GPU_ALLOCATABLE_WAIT_INTERVAL:-5}"
GPU_OPERATOR_POD_WAIT_ATTEMPTS="${GPU_OPERATOR_POD_WAIT_ATTEMPTS:-180}"
GPU_OPERATOR_POD_WAIT_INTERVAL="${GPU_OPERATOR_POD_WAIT_INTERVAL:-5}"
# multi-node gang scheduling (Grove / KAI scheduler): accepted for drop-in compatibility with the
# reference's flags; a single node needs neither, so they are reported and otherwise no-ops
ENABLE_GROVE="${ENABLE_GROVE:-false}"
ENABLE_KAI_SCHEDULER="${ENABLE_KAI_SCHEDULER:-false}"
MXS_USE_HELM="${MXS_USE_HELM:-auto}"                               # auto | true | false
CRD_RELEASE="${CRD_RELEASE:-mxserve-crds}"
PLATFORM_RELEASE="${PLATFORM_RELEASE:-mxserve-platform}"
HELM_TIMEOUT="${HELM_TIMEOUT:-10m}"
UNINSTALL="${UNINSTALL:-false}"
PURGE_CRDS="${PURGE_CRDS:-false}"

say() { printf '\n[install] %s\n' "$*"; }
die() { printf 'ERROR: %s\n' "$*" >&2; exit 1; }
for c in kubectl; do command -v "$c" >/dev/null || die "missing $c"; done
kubectl version >/dev/null 2>&1 || die "cannot reach the cluster (KUBECONFIG?)"

use_helm=false
if [[ "$MXS_USE_HELM" == "true" ]] || { [[ "$MXS_USE_HELM" == "auto" ]] && command -v helm >/dev/null; }; then
  command -v helm >/dev/null || die "MXS_USE_HELM=true but helm is not on PATH"
  use_helm=true
fi

if [[ "$UNINSTALL" == "true" ]]; then
  say "uninstall: operator release / objects in ${NAMESPACE}"
  if $use_helm && helm status "$PLATFORM_RELEASE" -n "$NAMESPACE" >/dev/null 2>&1; then
    helm uninstall "$PLATFORM_RELEASE" -n "$NAMESPACE" --wait
  else
    kubectl delete -n "$NAMESPACE" -f "$HERE/deploy/operator/operator.yaml" --ignore-not-found
  fi
  if [[ "$PURGE_CRDS" == "true" ]]; then
    say "uninstall: CRDs (deletes every DGD / DGDR / DCD)"
    if $use_helm && helm status "$CRD_RELEASE" -n default >/dev/null 2>&1; then
      helm uninstall "$CRD_RELEASE" -n default --wait
    else
      kubectl delete -f "$HERE/deploy/crds/" --ignore-not-found
    fi
  else
    say "CRDs kept (PURGE_CRDS=true removes them and every custom resource)"
  fi
  exit 0
fi

say "configuration"
for v in NAMESPACE RELEASE_VERSION MXS_IMAGE MXS_USE_HELM NAMESPACE_RESTRICTED_OPERATOR ENABLE_GROVE ENABLE_KAI_SCHEDULER \
         PROMETHEUS_ENDPOINT GPU_RESOURCE GPU_OPERATOR_MODE GPU_OPERATOR_NS GPU_OPERATOR_RELEASE GPU_OPERATOR_HELM_TIMEOUT; do
  echo "  ${v}=${!v}"
done
for v in ENABLE_GROVE ENABLE_KAI_SCHEDULER; do
  if [[ "${!v}" == "true" ]]; then
    echo "WARNING: ${v}=true has no effect: mxserve targets one node (8 GPUs, SURVEY §2.4 P07), where the" \
         "operator packs P/D groups into pods itself and no gang scheduler is needed" >&2
  fi
done

say "storage: default StorageClass"
if ! kubectl get storageclass -o jsonpath='{range .items[*]}{.metadata.annotations.storageclass\.kubernetes\.io/is-default-class}{"\n"}{end}' | grep -q true; then
  kubectl apply -f "$LOCAL_PATH_MANIFEST_URL"
  kubectl patch storageclass local-path -p '{"metadata":{"annotations":{"storageclass.kubernetes.io/is-default-class":"true"}}}'
fi

if $use_helm; then
  # `--version` does not select a version of a chart DIRECTORY: package both charts at
  # RELEASE_VERSION (chart version and appVersion) and install the packages, so `helm history` /
  # `helm rollback` track the release version
  charts="$(mktemp -d)"
  trap 'rm -rf "$charts"' EXIT
  for c in mxserve-crds mxserve-platform; do
    helm package "$HERE/deploy/helm/$c" --version "$RELEASE_VERSION" --app-version "$RELEASE_VERSION" \
      -d "$charts" >/dev/null
  done
  say "CRDs: helm release ${CRD_RELEASE} (chart mxserve-crds ${RELEASE_VERSION})"
  helm upgrade --install "$CRD_RELEASE" "$charts/mxserve-crds-${RELEASE_VERSION}.tgz" -n default \
    --wait --timeout "$HELM_TIMEOUT"
  say "operator: helm release ${PLATFORM_RELEASE} in ${NAMESPACE} (${MXS_IMAGE})"
  helm upgrade --install "$PLATFORM_RELEASE" "$charts/mxserve-platform-${RELEASE_VERSION}.tgz" -n "$NAMESPACE" --create-namespace \
    --set image.repository="${MXS_IMAGE%:*}" --set image.tag="${MXS_IMAGE##*:}" \
    --set namespaceRestricted="$NAMESPACE_RESTRICTED_OPERATOR" --set gpuResource="$GPU_RESOURCE" \
    --set prometheusEndpoint="$PROMETHEUS_ENDPOINT" --wait --timeout "$HELM_TIMEOUT"
  helm history "$PLATFORM_RELEASE" -n "$NAMESPACE" --max 3 || true
else
  say "CRDs (kubectl)"
  kubectl apply -f "$HERE/deploy/crds/"
  say "operator ${MXS_IMAGE} in ${NAMESPACE} (kubectl)"
  kubectl create namespace "$NAMESPACE" --dry-run=client -o yaml | kubectl apply -f -
  watch_args='["--interval", "30", "--health-port", "8081"]'
  [[ "$NAMESPACE_RESTRICTED_OPERATOR" == "true" ]] && watch_args="[\"--interval\", \"30\", \"--health-port\", \"8081\", \"--namespace\", \"${NAMESPACE}\"]"
  sed -e "s#IMAGE_PLACEHOLDER#${MXS_IMAGE}#g" -e "s#NAMESPACE_PLACEHOLDER#${NAMESPACE}#g" \
      -e "s#WATCH_ARGS_PLACEHOLDER#${watch_args}#" -e "s#GPU_RESOURCE_PLACEHOLDER#${GPU_RESOURCE}#" \
      -e "s#PROMETHEUS_ENDPOINT_PLACEHOLDER#${PROMETHEUS_ENDPOINT}#" \
      "$HERE/deploy/operator/operator.yaml" | kubectl apply -n "$NAMESPACE" -f -
fi
kubectl -n "$NAMESPACE" rollout status deploy/mxserve-operator --timeout=600s
# the operator hands PROMETHEUS_ENDPOINT to the SLA planners it runs (reference: prometheusEndpoint
# Helm value of the platform chart); workers and frontends are scraped through PodMonitors
say "metrics: PodMonitors per DGD; planners query Prometheus at ${PROMETHEUS_ENDPOINT}"

case "$GPU_OPERATOR_MODE" in
  operator)
    command -v helm >/dev/null || die "helm is required for GPU_OPERATOR_MODE=operator"
    say "AMD GPU Operator (${GPU_OPERATOR_RELEASE} in ${GPU_OPERATOR_NS})"
    helm repo add "$AMD_HELM_REPO_NAME" "$AMD_HELM_REPO_URL" >/dev/null 2>&1 || true
    helm repo update >/dev/null
    helm upgrade --install "$GPU_OPERATOR_RELEASE" "$AMD_HELM_REPO_NAME/gpu-operator-charts" \
      -n "$GPU_OPERATOR_NS" --create-namespace --wait --timeout "$GPU_OPERATOR_HELM_TIMEOUT"
    say "DeviceConfig: device plugin + node labeller + device-metrics-exporter (ServiceMonitor)"
    for f in metrics-exporter-config.yaml deviceconfig.yaml; do
      sed -e "s#GPU_OPERATOR_NS_PLACEHOLDER#${GPU_OPERATOR_NS}#g" "$HERE/deploy/amd-gpu/$f" | kubectl apply -f -
    done
    ;;
  device-plugin)
    say "ROCm k8s-device-plugin DaemonSet"
    kubectl apply -f "$ROCM_DEVICE_PLUGIN_URL"
    ;;
  skip) say "GPU operator installation skipped" ;;
  *) die "GPU_OPERATOR_MODE must be operator|device-plugin|skip" ;;
esac

if [[ "$GPU_OPERATOR_MODE" == "operator" ]]; then
  # the device plugin / node labeller DaemonSets must be up before the GPUs show as allocatable
  say "waiting for the AMD GPU Operator pods in ${GPU_OPERATOR_NS} to be Running/Completed"
  for ((i = 1; i <= GPU_OPERATOR_POD_WAIT_ATTEMPTS; i++)); do
    not_ready="$(kubectl get pods -n "$GPU_OPERATOR_NS" --no-headers 2>/dev/null \
                 | awk '$3 != "Running" && $3 != "Completed" {n++} END {print n + 0}')"
    [[ "$not_ready" == "0" ]] && break
    sleep "$GPU_OPERATOR_POD_WAIT_INTERVAL"
  done
  kubectl get pods -n "$GPU_OPERATOR_NS" || true
fi

say "waiting for ${GPU_RESOURCE} to become allocatable"
for ((i = 1; i <= GPU_ALLOCATABLE_WAIT_ATTEMPTS; i++)); do
  n="$(kubectl get nodes -o jsonpath="{range .items[*]}{.status.allocatable.${GPU_RESOURCE//./\\.}}{\"\\n\"}{end}" \
       | awk '{s += $1} END {print s + 0}')"
  if [[ "$n" -gt 0 ]]; then say "${n} x ${GPU_RESOURCE} allocatable"; exit 0; fi
  sleep "$GPU_ALLOCATABLE_WAIT_INTERVAL"
done
die "no ${GPU_RESOURCE} allocatable after $((GPU_ALLOCATABLE_WAIT_ATTEMPTS * GPU_ALLOCATABLE_WAIT_INTERVAL))s"
