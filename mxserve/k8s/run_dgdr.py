"""Implementation of examples/dgdr/trtllm/run-dgdr.sh (reference run-dgdr.sh:4-54): create the
namespace, (re)create ConfigMap CONFIGMAP_NAME from DISAGG_FILE (under the key the DGDR's
configMapRef names, so DISAGG_FILE=disagg_cache.yaml still lands where the request looks), apply
DGDR_FILE, wait for the generated graph's frontend Service and expose it on FRONTEND_NODEPORT."""
from __future__ import annotations

import os
import sys
import time

import yaml

from .client import KubeClient


def main(k: KubeClient | None = None) -> int:
    e = os.environ
    here = os.path.dirname(os.path.abspath(sys.argv[0])) if sys.argv and sys.argv[0] else "."
    ns = e.get("NAMESPACE", "dynamo-system")
    cm_name = e.get("CONFIGMAP_NAME", "qwen-config")
    disagg = e.get("DISAGG_FILE", os.path.join(here, "disagg.yaml"))
    dgdr_file = e.get("DGDR_FILE", os.path.join(here, "dgdr.yaml"))
    nodeport = int(e.get("FRONTEND_NODEPORT", "30081"))
    timeout = float(e.get("FRONTEND_TIMEOUT", "900"))
    k = k or (KubeClient(e["MXS_KUBE_SERVER"]) if e.get("MXS_KUBE_SERVER") else KubeClient())
    if k.get("Namespace", ns) is None:
        k.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    with open(dgdr_file) as f:
        req = yaml.safe_load(f)
    ref = (((req.get("spec") or {}).get("profilingConfig") or {}).get("configMapRef") or {})
    key = ref.get("key") or os.path.basename(disagg)
    with open(disagg) as f:
        k.apply({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": cm_name, "namespace": ns},
                 "data": {key: f.read()}})
    print(f"==> ConfigMap {cm_name} updated from {disagg} (key {key})")
    req["metadata"]["namespace"] = ns
    k.apply(req)
    print(f"==> applied {dgdr_file}; waiting for the generated frontend Service")
    t0 = time.time()
    while True:
        fe = [s for s in k.list("Service", ns) if "frontend" in s["metadata"]["name"]]
        if fe:
            break
        if time.time() - t0 > timeout:
            print("ERROR: no frontend Service appeared (check `kubectl get dgdr -n %s -o yaml`)" % ns, file=sys.stderr)
            return 1
        time.sleep(float(e.get("MXS_POLL_SECONDS", "5")))
    svc = fe[0]
    ports = [dict(p) for p in svc["spec"]["ports"]]
    ports[0]["nodePort"] = nodeport
    k.merge_patch("Service", svc["metadata"]["name"], ns, {"spec": {"type": "NodePort", "ports": ports}})
    model = req["spec"].get("model", "<model>")
    print(f"""
==> Frontend {svc['metadata']['name']} exposed on NodePort {nodeport}
export DYNAMO_BASE_URL=http://<node-ip>:{nodeport}
curl -s $DYNAMO_BASE_URL/v1/chat/completions -H 'Content-Type: application/json' \\
  -d '{{"model": "{model}", "messages": [{{"role": "user", "content": "Hello"}}], "max_tokens": 64}}'
""")
    return 0


if __name__ == "__main__":
    sys.exit(main())
