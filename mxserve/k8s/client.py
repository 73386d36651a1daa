"""Minimal Kubernetes REST client (no kubernetes-python dependency in the image).

Configuration: in-cluster service account, `$KUBECONFIG` / ~/.kube/config (token or client
certificate), or an explicit server URL (tests use the in-process fake apiserver)."""
from __future__ import annotations

import base64
import hashlib
import json
import os
import tempfile
from typing import Iterator, Optional

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
    "Event": ("v1", "events"),
    "Lease": ("coordination.k8s.io/v1", "leases"),
}
# annotation carrying the hash of the spec the operator last applied (apply() skips unchanged objects)
HASH_ANNOTATION = "mxserve.io/spec-hash"


def spec_hash(obj: dict) -> str:
    """Hash of everything apply() would write (the object minus status and the hash itself)."""
    body = {k: v for k, v in obj.items() if k != "status"}
    meta = dict(body.get("metadata") or {})
    ann = {k: v for k, v in (meta.get("annotations") or {}).items() if k != HASH_ANNOTATION}
    meta["annotations"] = ann
    body["metadata"] = meta
    return hashlib.sha256(json.dumps(body, sort_keys=True, default=str).encode()).hexdigest()[:20]
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
        """Create, or merge-patch the spec/labels/owners of an existing object.  The object is stamped
        with a hash of what is written; an existing object carrying the same hash is left alone (no
        write), so a reconcile of an unchanged graph costs reads only.  A patch the apiserver refuses
        as invalid (422: e.g. a Deployment's immutable selector changed) deletes and recreates."""
        meta = obj["metadata"]
        h = spec_hash(obj)
        obj = dict(obj, metadata=dict(meta, annotations={**(meta.get("annotations") or {}), HASH_ANNOTATION: h}))
        cur = self.get(obj["kind"], meta["name"], meta.get("namespace"))
        if cur is None:
            return self.create(obj)
        if ((cur.get("metadata") or {}).get("annotations") or {}).get(HASH_ANNOTATION) == h:
            return cur
        patch = {k: v for k, v in obj.items() if k not in ("apiVersion", "kind", "status")}
        try:
            return self.merge_patch(obj["kind"], meta["name"], meta.get("namespace"), patch)
        except ApiError as e:
            if e.status != 422:
                raise
            self.delete(obj["kind"], meta["name"], meta.get("namespace"))
            return self.create(obj)

    def list_rv(self, kind: str, namespace: Optional[str] = None, label_selector: Optional[str] = None) -> tuple:
        """(items, the list's resourceVersion) -- the starting point of a watch."""
        params = {"labelSelector": label_selector} if label_selector else None
        out = self._req("GET", _path(kind, namespace), params=params)
        return out.get("items", []), str((out.get("metadata") or {}).get("resourceVersion") or "")

    def watch(self, kind: str, namespace: Optional[str] = None, resource_version: str = "",
              timeout_s: int = 60, label_selector: Optional[str] = None) -> Iterator[dict]:
        """Stream watch events ({"type": ADDED|MODIFIED|DELETED|BOOKMARK|ERROR, "object": ...}) from
        resource_version on, for at most timeout_s seconds (the apiserver closes the stream then)."""
        params = {"watch": "true", "timeoutSeconds": str(int(timeout_s)), "allowWatchBookmarks": "true"}
        if resource_version:
            params["resourceVersion"] = resource_version
        if label_selector:
            params["labelSelector"] = label_selector
        with self.http.stream("GET", _path(kind, namespace), params=params, timeout=timeout_s + 10) as r:
            if r.status_code >= 400:
                r.read()
                raise ApiError(r.status_code, r.text[:300])
            for line in r.iter_lines():
                if line.strip():
                    yield json.loads(line)

    def event(self, involved: dict, reason: str, message: str, kind: str = "Normal") -> None:
        """Record a core/v1 Event on `involved` (best effort: an Event failing never fails a reconcile)."""
        meta = involved.get("metadata") or {}
        ns = meta.get("namespace") or "default"
        try:
            self.create({"apiVersion": "v1", "kind": "Event",
                         "metadata": {"generateName": f"{meta.get('name', 'obj')}.", "namespace": ns,
                                      "name": f"{meta.get('name', 'obj')}.{os.urandom(6).hex()}"},
                         "involvedObject": {"apiVersion": involved.get("apiVersion"), "kind": involved.get("kind"),
                                            "name": meta.get("name"), "namespace": ns, "uid": meta.get("uid")},
                         "reason": reason, "message": message, "type": kind,
                         "source": {"component": "mxserve-operator"}})
        except (ApiError, OSError, httpx.HTTPError):
            pass

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
