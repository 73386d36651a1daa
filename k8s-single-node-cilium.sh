#!/usr/bin/env bash
# Bootstrap a single-node Kubernetes cluster for an 8x MI355X host: containerd (systemd cgroups),
# kubeadm/kubelet/kubectl, Cilium (+Hubble), Helm, kube-prometheus-stack with open PodMonitor
# selection (the mxserve operator creates PodMonitors in the workload namespaces).
# Run as root: sudo -E ./k8s-single-node-cilium.sh      Re-running on an initialised node is a no-op.
set -euo pipefail

K8S_REPO_MINOR="${K8S_REPO_MINOR:-v1.35}"
CLUSTER_NAME="${CLUSTER_NAME:-k8s-single}"
POD_CIDR="${POD_CIDR:-10.0.0.0/16}"
ENABLE_HUBBLE="${ENABLE_HUBBLE:-true}"
HELM_VERSION="${HELM_VERSION:-v4.1.0}"
INSTALL_HELM="${INSTALL_HELM:-true}"
INSTALL_PROMETHEUS_STACK="${INSTALL_PROMETHEUS_STACK:-true}"
MONITORING_NS="${MONITORING_NS:-monitoring}"

say() { printf '\n[k8s] %s\n' "$*"; }
die() { printf 'ERROR: %s\n' "$*" >&2; exit 1; }

[[ $EUID -eq 0 ]] || die "run as root (sudo -E $0)"
. /etc/os-release 2>/dev/null || true
[[ "${ID:-}" == "ubuntu" ]] || die "Ubuntu is required (found ${ID:-unknown})"
OWNER="${SUDO_USER:-root}"
OWNER_HOME="$(getent passwd "$OWNER" | cut -d: -f6)"
case "$(uname -m)" in x86_64) ARCH=amd64 ;; aarch64) ARCH=arm64 ;; *) die "unsupported arch $(uname -m)" ;; esac

if [[ -f /etc/kubernetes/admin.conf ]]; then
  say "cluster already initialised (/etc/kubernetes/admin.conf exists); nothing to do"
  exit 0
fi

say "OS prerequisites"
apt-get update -y
apt-get install -y apt-transport-https ca-certificates curl gpg conntrack socat containerd
swapoff -a
sed -ri '/\sswap\s/s/^#?/#/' /etc/fstab
printf 'overlay\nbr_netfilter\n' > /etc/modules-load.d/k8s.conf
modprobe overlay; modprobe br_netfilter
cat > /etc/sysctl.d/99-k8s.conf <<SYS
net.bridge.bridge-nf-call-iptables = 1
net.bridge.bridge-nf-call-ip6tables = 1
net.ipv4.ip_forward = 1
SYS
sysctl --system >/dev/null

say "containerd with systemd cgroups"
mkdir -p /etc/containerd
containerd config default > /etc/containerd/config.toml
sed -i 's/SystemdCgroup = false/SystemdCgroup = true/' /etc/containerd/config.toml
systemctl restart containerd && systemctl enable containerd

say "kubeadm/kubelet/kubectl ${K8S_REPO_MINOR}"
install -d -m 0755 /etc/apt/keyrings
curl -fsSL "https://pkgs.k8s.io/core:/stable:/${K8S_REPO_MINOR}/deb/Release.key" \
  | gpg --dearmor --yes -o /etc/apt/keyrings/kubernetes-apt-keyring.gpg
echo "deb [signed-by=/etc/apt/keyrings/kubernetes-apt-keyring.gpg] https://pkgs.k8s.io/core:/stable:/${K8S_REPO_MINOR}/deb/ /" \
  > /etc/apt/sources.list.d/kubernetes.list
apt-get update -y && apt-get install -y kubelet kubeadm kubectl && apt-mark hold kubelet kubeadm kubectl

if [[ "$INSTALL_HELM" == "true" ]] && ! command -v helm >/dev/null; then
  say "helm ${HELM_VERSION}"
  tmp="$(mktemp -d)"
  curl -fsSL -o "$tmp/helm.tgz" "https://get.helm.sh/helm-${HELM_VERSION}-linux-${ARCH}.tar.gz"
  curl -fsSL -o "$tmp/helm.tgz.sha256sum" "https://get.helm.sh/helm-${HELM_VERSION}-linux-${ARCH}.tar.gz.sha256sum"
  (cd "$tmp" && echo "$(cut -d' ' -f1 helm.tgz.sha256sum)  helm.tgz" | sha256sum -c -)
  tar -xzf "$tmp/helm.tgz" -C "$tmp" && install -m 0755 "$tmp/linux-${ARCH}/helm" /usr/local/bin/helm
  rm -rf "$tmp"
fi

NODE_NAME="${NODE_NAME:-$(hostname -s | tr '[:upper:]' '[:lower:]')}"
say "kubeadm init (${CLUSTER_NAME}, node ${NODE_NAME}, pods ${POD_CIDR})"
kubeadm init --pod-network-cidr="$POD_CIDR" --node-name="$NODE_NAME" --skip-phases=addon/kube-proxy
install -d -o "$OWNER" "$OWNER_HOME/.kube"
install -m 0600 -o "$OWNER" /etc/kubernetes/admin.conf "$OWNER_HOME/.kube/config"
export KUBECONFIG=/etc/kubernetes/admin.conf
# the sudo user's shell: `k` alias with kubectl's bash completion on both names
bashrc="$OWNER_HOME/.bashrc"
grep -q 'alias k=kubectl' "$bashrc" 2>/dev/null || echo 'alias k=kubectl' >> "$bashrc"
grep -q 'kubectl completion bash' "$bashrc" 2>/dev/null || cat >> "$bashrc" <<'RC'
source <(kubectl completion bash)
complete -o default -F __start_kubectl k
RC
chown "$OWNER" "$bashrc" 2>/dev/null || true

say "Cilium (kube-proxy replacement, hubble=${ENABLE_HUBBLE})"
CILIUM_CLI_VERSION="$(curl -fsSL https://raw.githubusercontent.com/cilium/cilium-cli/main/stable.txt)"
tmp="$(mktemp -d)"
cilium_url="https://github.com/cilium/cilium-cli/releases/download/${CILIUM_CLI_VERSION}/cilium-linux-${ARCH}.tar.gz"
curl -fsSL -o "$tmp/cilium-linux-${ARCH}.tar.gz" "$cilium_url"
curl -fsSL -o "$tmp/cilium-linux-${ARCH}.tar.gz.sha256sum" "${cilium_url}.sha256sum"
# nothing is unpacked as root before its published checksum matches
(cd "$tmp" && sha256sum --check "cilium-linux-${ARCH}.tar.gz.sha256sum")
tar -xzf "$tmp/cilium-linux-${ARCH}.tar.gz" -C /usr/local/bin cilium
rm -rf "$tmp"
cilium install --set kubeProxyReplacement=true --set cluster.name="$CLUSTER_NAME"
if [[ "$ENABLE_HUBBLE" == "true" ]]; then cilium hubble enable --ui; fi
kubectl taint nodes --all node-role.kubernetes.io/control-plane- 2>/dev/null || true
cilium status --wait

if [[ "$INSTALL_PROMETHEUS_STACK" == "true" ]]; then
  say "kube-prometheus-stack in ${MONITORING_NS}"
  helm repo add prometheus-community https://prometheus-community.github.io/helm-charts >/dev/null
  helm repo update >/dev/null
  helm upgrade --install prometheus prometheus-community/kube-prometheus-stack -n "$MONITORING_NS" --create-namespace \
    --set prometheus.prometheusSpec.podMonitorSelectorNilUsesHelmValues=false \
    --set prometheus.prometheusSpec.serviceMonitorSelectorNilUsesHelmValues=false \
    --set prometheus.prometheusSpec.podMonitorNamespaceSelector={} \
    --set grafana.sidecar.dashboards.enabled=true --set grafana.sidecar.dashboards.searchNamespace=ALL --wait
  pw="$(kubectl -n "$MONITORING_NS" get secret prometheus-grafana -o jsonpath='{.data.admin-password}' | base64 -d)"
  say "Grafana: user admin, password ${pw} (kubectl -n ${MONITORING_NS} port-forward svc/prometheus-grafana 3000:80)"
fi

say "done: kubectl get nodes -o wide; next: make dynamo (installs the mxserve platform + AMD GPU operator)"
