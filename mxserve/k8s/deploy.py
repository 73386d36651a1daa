"""Implementation of `deploy-incluster.sh` (reference deploy-incluster.sh:14-659, same flags, env
and printed quick test) over the REST client instead of kubectl text parsing:

  --manifest FILE  --namespace NS (dynamo-system)  --model M  --hf-token T  --nodeport P  --no-wait
  env: MANIFEST_FILE NAMESPACE MODEL HF_TOKEN NODEPORT NO_WAIT PODS_TIMEOUT ENDPOINTS_TIMEOUT
       SERVICES_TIMEOUT DEPLOYMENTS_TIMEOUT

Steps: validate -> warn if no allocatable amd.com/gpu -> ensure namespace -> hf-token-secret (keys
HF_TOKEN, HUGGING_FACE_HUB_TOKEN, token; "dummy" when no token) -> apply the manifest as-is ->
find Deployments by `nvidia.com/dynamo-namespace=<ns>-<dgd>` and Services by `<dgd>-` prefix ->
NodePort for every non-headless Service (fixed port for the frontend if given) -> wait for every
Deployment ready (all replicas, not just the first pod) -> wait for the frontend's Endpoints ->
print the quick test.  With a token, every DGD service gets envFromSecret: hf-token-secret.
While it waits it prints, every MXS_PROGRESS_SECONDS (15), each Deployment's ready count, each pod's
phase and container waiting reasons (ImagePullBackOff, CrashLoopBackOff, ...) and the namespace's
recent Warning events (e.g. FailedScheduling: Insufficient amd.com/gpu), as the reference's wait loop
does (deploy-incluster.sh:511-605); a timeout error carries the same report.
Fixes the reference quirks listed in SURVEY.md Appendix B items 2, 3 and 5.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import Optional

import yaml

from .client import ApiError, KubeClient
from .resources import GPU_RESOURCE, NS_LABEL


def log(msg: str) -> None:
    print(f"\n==> {msg}\n", flush=True)


def warn(msg: str) -> None:
    print(f"WARN: {msg}\n", file=sys.stderr, flush=True)


class DeployError(RuntimeError):
    pass


def parse_args(argv=None) -> argparse.Namespace:
    e = os.environ
    ap = argparse.ArgumentParser(prog="deploy-incluster.sh", description="Deploy a DynamoGraphDeployment manifest")
    ap.add_argument("--manifest", default=e.get("MANIFEST_FILE", ""))
    ap.add_argument("--namespace", default=e.get("NAMESPACE", "dynamo-system"))
    ap.add_argument("--model", default=e.get("MODEL", ""))
    ap.add_argument("--hf-token", default=e.get("HF_TOKEN", ""))
    ap.add_argument("--nodeport", default=e.get("NODEPORT", ""))
    ap.add_argument("--no-wait", action="store_true", default=e.get("NO_WAIT", "false") == "true")
    ap.add_argument("--server", default=e.get("MXS_KUBE_SERVER"), help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    a.pods_timeout = int(e.get("PODS_TIMEOUT", "1200"))
    a.endpoints_timeout = int(e.get("ENDPOINTS_TIMEOUT", "300"))
    a.services_timeout = int(e.get("SERVICES_TIMEOUT", "180"))
    a.deployments_timeout = int(e.get("DEPLOYMENTS_TIMEOUT", "180"))
    a.poll = float(e.get("MXS_POLL_SECONDS", "3"))
    a.progress = float(e.get("MXS_PROGRESS_SECONDS", "15"))
    return a


def _poll(fn, timeout: float, interval: float, what: str, report=None, every: float = 15.0):
    """Call fn until it returns something truthy.  `report()` (a list of lines) is printed every
    `every` seconds while waiting and appended to the timeout error."""
    t0 = last = time.time()
    while True:
        v = fn()
        if v:
            return v
        now = time.time()
        if now - t0 > timeout:
            lines = report() if report else []
            raise DeployError(f"timed out after {timeout:.0f}s waiting for {what}" +
                              ("".join("\n  " + ln for ln in lines) if lines else ""))
        if report and now - last >= every:
            last = now
            print(f"... waiting for {what} ({now - t0:.0f}s / {timeout:.0f}s)", flush=True)
            for ln in report():
                print("    " + ln, flush=True)
        time.sleep(interval)


def _ts(ev: dict) -> str:
    return str(ev.get("lastTimestamp") or ev.get("eventTime") or (ev.get("metadata") or {}).get("creationTimestamp")
               or "")


def status_report(k: KubeClient, ns: str, sel: str, max_events: int = 6) -> list:
    """Human-readable state of a graph's Deployments, pods and recent Warning events."""
    out = []
    try:
        names = set()
        for d in k.list("Deployment", ns, sel):
            st = d.get("status") or {}
            names.add(d["metadata"]["name"])
            out.append(f"deployment {d['metadata']['name']}: ready {int(st.get('readyReplicas', 0) or 0)}/"
                       f"{int(d['spec'].get('replicas', 1))}")
        for p in k.list("Pod", ns, sel):
            names.add(p["metadata"]["name"])
            st = p.get("status") or {}
            cs = st.get("containerStatuses") or []
            ready = sum(1 for c in cs if c.get("ready"))
            why = []
            for c in cs:
                for state in ("waiting", "terminated"):
                    w = (c.get("state") or {}).get(state)
                    if w and w.get("reason"):
                        why.append(f"{c.get('name')}: {w['reason']}" + (f" ({w['message'][:120]})" if w.get("message")
                                                                       else ""))
                if c.get("restartCount"):
                    why.append(f"{c.get('name')}: {c['restartCount']} restarts")
            for cond in st.get("conditions") or []:
                if cond.get("type") == "PodScheduled" and cond.get("status") == "False":
                    why.append(f"unschedulable: {cond.get('message', cond.get('reason', ''))[:160]}")
            out.append(f"pod {p['metadata']['name']}: {st.get('phase', '?')} {ready}/{len(cs) or 1}"
                       + (" -- " + "; ".join(why) if why else ""))
        evs = [e for e in k.list("Event", ns) if e.get("type") == "Warning"
               and any(((e.get("involvedObject") or {}).get("name") or "").startswith(n) for n in names)]
        for e in sorted(evs, key=_ts)[-max_events:]:
            io = e.get("involvedObject") or {}
            out.append(f"event {io.get('kind', '')}/{io.get('name', '')}: {e.get('reason', '')}: "
                       f"{(e.get('message') or '')[:160]}")
    except (ApiError, OSError) as e:  # a report never turns into the error itself
        out.append(f"(status unavailable: {e})")
    return out


def run(a: argparse.Namespace, k: Optional[KubeClient] = None) -> dict:
    if not a.manifest:
        raise DeployError("--manifest is required")
    if not os.path.isfile(a.manifest):
        raise DeployError(f"manifest not found: {a.manifest}")
    if a.nodeport and not (a.nodeport.isdigit() and 30000 <= int(a.nodeport) <= 32767):
        raise DeployError(f"--nodeport must be in 30000-32767, got {a.nodeport}")
    with open(a.manifest) as f:
        docs = [d for d in yaml.safe_load_all(f) if isinstance(d, dict)]
    if not docs:
        raise DeployError("manifest contains no objects")
    k = k or (KubeClient(a.server) if a.server else KubeClient())
    ns = a.namespace

    nodes = k.list("Node")
    gpus = sum(int((n.get("status") or {}).get("allocatable", {}).get(GPU_RESOURCE, 0) or 0) for n in nodes)
    if gpus == 0:
        warn(f"no allocatable {GPU_RESOURCE} on any node (is the AMD GPU Operator / device plugin running?)")
    else:
        log(f"cluster has {gpus} allocatable {GPU_RESOURCE}")

    if k.get("Namespace", ns) is None:
        k.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
    tok = a.hf_token or "dummy"
    k.apply({"apiVersion": "v1", "kind": "Secret", "metadata": {"name": "hf-token-secret", "namespace": ns},
             "type": "Opaque", "stringData": {"HF_TOKEN": tok, "HUGGING_FACE_HUB_TOKEN": tok, "token": tok}})
    log(f"applying {a.manifest} to namespace {ns}")
    dgds = []
    for d in docs:
        d.setdefault("metadata", {})["namespace"] = ns
        if d.get("kind") == "DynamoGraphDeployment" and a.hf_token:
            # reference :233-247 + :648-655 (envFromSecret patch, then `kubectl set env
            # --from=secret`): every service of THIS graph gets the token secret (the reference's
            # fixed service names added stray services to SGLang/TRT-LLM graphs, Appendix B item 2),
            # and the operator renders it as envFrom on the pods
            for svc in ((d.get("spec") or {}).get("services") or {}).values():
                svc.setdefault("envFromSecret", "hf-token-secret")
        k.apply(d)
        if d.get("kind") == "DynamoGraphDeployment":
            dgds.append(d["metadata"]["name"])
    result = {"namespace": ns, "graphs": {}}
    for g in dgds:
        sel = f"{NS_LABEL}={ns}-{g}"
        deps = _poll(lambda: k.list("Deployment", ns, sel), a.deployments_timeout, a.poll, f"deployments of {g}")
        svcs = _poll(lambda: [s for s in k.list("Service", ns) if s["metadata"]["name"].startswith(g + "-")],
                     a.services_timeout, a.poll, f"services of {g}")
        fe = [s for s in svcs if "frontend" in s["metadata"]["name"]]
        if not fe:
            raise DeployError(f"no frontend service for {g}")
        ports = {}
        for s in svcs:
            if (s.get("spec") or {}).get("clusterIP") == "None":
                continue  # headless worker services are not exposed
            name = s["metadata"]["name"]
            pl = [dict(p) for p in s["spec"]["ports"]]
            if a.nodeport and s is fe[0]:
                pl[0]["nodePort"] = int(a.nodeport)
            cur = k.merge_patch("Service", name, ns, {"spec": {"type": "NodePort", "ports": pl}})
            ports[name] = (cur.get("spec") or {}).get("ports", [{}])[0].get("nodePort")
        if not a.no_wait:
            def ready():
                ds = k.list("Deployment", ns, sel)
                return all(int((d.get("status") or {}).get("readyReplicas", 0) or 0) >= int(d["spec"].get("replicas", 1))
                           for d in ds) and ds
            _poll(ready, a.pods_timeout, a.poll, f"all pods of {g} ready",
                  report=lambda: status_report(k, ns, sel), every=a.progress)
            for ln in status_report(k, ns, sel):
                print("    " + ln, flush=True)
            # reference wait_endpoints (:94-108, :573): the frontend Service routes to a ready pod
            fe_name = fe[0]["metadata"]["name"]

            def has_endpoints():
                ep = k.get("Endpoints", fe_name, ns) or {}
                return any(ss.get("addresses") for ss in ep.get("subsets") or [])
            _poll(has_endpoints, a.endpoints_timeout, a.poll, f"endpoints of {fe_name}",
                  report=lambda: status_report(k, ns, sel), every=a.progress)
        result["graphs"][g] = {"deployments": sorted(d["metadata"]["name"] for d in deps),
                               "services": sorted(s["metadata"]["name"] for s in svcs),
                               "frontend": fe[0]["metadata"]["name"], "nodeports": ports}
    node_ip = "<node-ip>"
    for n in nodes:
        for ad in (n.get("status") or {}).get("addresses", []):
            if ad.get("type") == "InternalIP":
                node_ip = ad["address"]
    result["node_ip"] = node_ip
    print_quick_test(result, a.model)
    return result


def print_quick_test(result: dict, model: str) -> None:
    for g, info in result["graphs"].items():
        port = info["nodeports"].get(info["frontend"])
        base = f"http://{result['node_ip']}:{port}"
        m = model or "<model>"
        print(f"""
==> Quick test for {g} (namespace {result['namespace']})

export DYNAMO_BASE_URL={base}
curl -s $DYNAMO_BASE_URL/v1/models | python3 -m json.tool
curl -s $DYNAMO_BASE_URL/v1/chat/completions -H 'Content-Type: application/json' \\
  -d '{json.dumps({"model": m, "messages": [{"role": "user", "content": "Hello!"}], "max_tokens": 64})}'
./chat.sh $DYNAMO_BASE_URL/v1/chat/completions {m}
""", flush=True)


def main(argv=None) -> int:
    a = parse_args(argv)
    try:
        run(a)
        return 0
    except (DeployError, ApiError) as e:
        print(f"ERROR: {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
