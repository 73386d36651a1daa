"""Minimal Kubernetes REST client (no kubernetes-python dependency in the image).

Configuration: in-cluster service account, `$KUBECONFIG` / ~/.kube/config (token or client
certificate), or an explicit server URL (tests use the in-process fake apiserver)."""
from __future__ import annotations

import base64
import os
import tempfile
from typing import Optional

import httpx
import yaml

PLURALS = {
    "Deployment": ("apps/v1", "deployments"), "Service": ("v1", "services"), "ConfigMap": ("v1", "configmaps"),
    "Secret": ("v1", "secrets"), "Pod": ("v1", "pods"), "Endpoints": ("v1", "endpoints"), "Namespace": ("v1", "namespaces"), "Node": ("v1", "nodes"),
    "PersistentVolumeClaim": ("v1", "persistentvolumeclaims"), "Job": ("batch/v1", "jobs"),
    "PodMonitor": ("monitoring.coreos.com/v1", "podmonitors"),
    "ServiceAccount": ("v1", "serviceaccounts"), "Role": ("rbac.authorization.k8s.io/v1", "roles"),
    "RoleBinding": ("rbac.authorization.k8s.io/v1", "rolebindings"),
    "DynamoGraphDeployment": ("nvidia.com/v1alpha1", "dynamographdeployments"),
    "DynamoGraphDeploymentRequest": ("nvidia.com/v1alpha1", "dynamographdeploymentrequests"),
    "DynamoComponentDeployment": ("nvidia.com/v1alpha1", "dynamocomponentdeployments"),
}
CLUSTER_SCOPED = {"Namespace", "Node"}


class ApiError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{status}: {msg}")
        self.status = status


def _path(kind: str, namespace: Optional[str], name: Optional[str] = None, sub: Optional[str] = None,
          api_version: Optional[str] = None) -> str:
    av, plural = PLURALS[kind]
    av = api_version or av
    base = f"/api/{av}" if "/" not in av else f"/apis/{av}"
    if kind not in CLUSTER_SCOPED and namespace:
        base += f"/namespaces/{namespace}"
    p = f"{base}/{plural}"
    if name:
        p += f"/{name}"
    if sub:
        p += f"/{sub}"
    return p


class KubeClient:
    def __init__(self, server: Optional[str] = None, token: Optional[str] = None, verify=True, cert=None):
        if server is None:
            server, token, verify, cert = self._discover()
        headers = {"Authorization": f"Bearer {token}"} if token else {}
        self.http = httpx.Client(base_url=server, headers=headers, verify=verify, cert=cert, timeout=30)

    @staticmethod
    def _discover():
        sa = "/var/run/secrets/kubernetes.io/serviceaccount"
        if os.environ.get("KUBERNETES_SERVICE_HOST") and os.path.exists(f"{sa}/token"):
            host, port = os.environ["KUBERNETES_SERVICE_HOST"], os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            with open(f"{sa}/token") as f:
                return f"https://{host}:{port}", f.read().strip(), f"{sa}/ca.crt", None
        path = os.environ.get("KUBECONFIG", os.path.expanduser("~/.kube/config"))
        with open(path) as f:
            kc = yaml.safe_load(f)
        ctx_name = kc.get("current-context")
        ctx = next(c["context"] for c in kc["contexts"] if c["name"] == ctx_name)
        cl = next(c["cluster"] for c in kc["clusters"] if c["name"] == ctx["cluster"])
        us = next(u["user"] for u in kc["users"] if u["name"] == ctx["user"])

        def _tmp(data_b64: str) -> str:
            fd, p = tempfile.mkstemp()
            os.write(fd, base64.b64decode(data_b64))
            os.close(fd)
            return p
        verify = _tmp(cl["certificate-authority-data"]) if "certificate-authority-data" in cl else \
            cl.get("certificate-authority", not cl.get("insecure-skip-tls-verify", False))
        cert = None
        if "client-certificate-data" in us:
            cert = (_tmp(us["client-certificate-data"]), _tmp(us["client-key-data"]))
        return cl["server"], us.get("token"), verify, cert

    def _req(self, method: str, path: str, **kw):
        r = self.http.request(method, path, **kw)
        if r.status_code >= 400:
            raise ApiError(r.status_code, r.text[:300])
        return r.json() if r.content else {}

    def get(self, kind: str, name: str, namespace: Optional[str] = None) -> Optional[dict]:
        try:
            return self._req("GET", _path(kind, namespace, name))
        except ApiError as e:
            if e.status == 404:
                return None
            raise

    def list(self, kind: str, namespace: Optional[str] = None, label_selector: Optional[str] = None) -> list:
        params = {"labelSelector": label_selector} if label_selector else None
        return self._req("GET", _path(kind, namespace), params=params).get("items", [])

    def create(self, obj: dict) -> dict:
        ns = obj.get("metadata", {}).get("namespace")
        return self._req("POST", _path(obj["kind"], ns, api_version=obj.get("apiVersion")), json=obj)

    def merge_patch(self, kind: str, name: str, namespace: Optional[str], patch: dict, sub: Optional[str] = None):
        return self._req("PATCH", _path(kind, namespace, name, sub), json=patch,
                         headers={"Content-Type": "application/merge-patch+json"})

    def apply(self, obj: dict) -> dict:
        """Create, or merge-patch the spec/labels/owners of an existing object."""
        meta = obj["metadata"]
        cur = self.get(obj["kind"], meta["name"], meta.get("namespace"))
        if cur is None:
            return self.create(obj)
        patch = {k: v for k, v in obj.items() if k not in ("apiVersion", "kind", "status")}
        return self.merge_patch(obj["kind"], meta["name"], meta.get("namespace"), patch)

    def delete(self, kind: str, name: str, namespace: Optional[str] = None) -> None:
        try:
            self._req("DELETE", _path(kind, namespace, name))
        except ApiError as e:
            if e.status != 404:
                raise

    def patch_status(self, kind: str, name: str, namespace: Optional[str], status: dict) -> None:
        try:
            self.merge_patch(kind, name, namespace, {"status": status}, sub="status")
        except ApiError as e:
            if e.status != 404:
                raise
