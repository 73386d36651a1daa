"""In-process fake Kubernetes apiserver: the REST subset the operator and deploy scripts use
(CRUD, merge-patch, /status, labelSelector lists, list + watch from a resourceVersion,
ownerReference-free storage).  Used by the
operator tests and the script tests; `python -m mxserve.k8s.fake_apiserver
--port P` runs it standalone.  Optionally marks Deployments ready (simulated kubelet)."""
from __future__ import annotations

import argparse
import asyncio
import copy
import itertools
import json
import os
import threading
import time
import uuid

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, StreamingResponse


def _merge(dst: dict, patch: dict) -> dict:
    for k, v in patch.items():
        if v is None:
            dst.pop(k, None)
        elif isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _match(labels: dict, selector: str | None) -> bool:
    if not selector:
        return True
    for term in selector.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            if labels.get(k) == v:
                return False
        elif "=" in term:
            k, v = term.split("=", 1)
            if labels.get(k) != v.lstrip("="):
                return False
        elif labels.get(term) is None:
            return False
    return True


class FakeApiServer:
    def __init__(self, auto_ready: bool = True, nodes: int = 1, gpus_per_node: int = 8,
                 gpu_resource: str = "amd.com/gpu"):
        self.store: dict[tuple, dict] = {}  # (group/version, plural, ns, name) -> obj
        self.auto_ready = auto_ready
        self.endpoints_ready = True  # tests flip it to simulate pods that never become endpoints
        # Jobs: `job_runner(job)` runs in a thread when a Job is created (default: run the mxserve
        # profiler's command in-process against this server, needs `url`), then the Job succeeds
        self.url: str | None = None
        self.job_runner = self._run_profiler_job
        self.jobs_run: list = []
        self.log: list = []
        self.events: list = []  # (resourceVersion, type, gv, plural, ns, obj) for watches
        self._rv = itertools.count(1)
        for i in range(nodes):
            self._put("v1", "nodes", None, {
                "apiVersion": "v1", "kind": "Node", "metadata": {"name": f"node-{i}", "labels": {}},
                "status": {"allocatable": {gpu_resource: str(gpus_per_node), "cpu": "128"},
                           "addresses": [{"type": "InternalIP", "address": f"10.0.0.{i + 10}"}]}})
        self.app = self._build()

    def _put(self, gv, plural, ns, obj):
        meta = obj.setdefault("metadata", {})
        meta.setdefault("uid", str(uuid.uuid4()))
        meta.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
        meta["resourceVersion"] = str(next(self._rv))
        if ns:
            meta["namespace"] = ns
        if plural == "deployments" and self.auto_ready:
            r = int(obj.get("spec", {}).get("replicas", 1))
            obj["status"] = {"replicas": r, "readyReplicas": r, "availableReplicas": r}
        if plural == "services" and obj.get("spec", {}).get("type") == "NodePort":
            used = {p.get("nodePort") for o in self.objects("services") for p in o["spec"].get("ports", [])}
            for p in obj["spec"].get("ports", []):
                if not p.get("nodePort"):
                    p["nodePort"] = next(n for n in range(30000, 32768) if n not in used)
                    used.add(p["nodePort"])
        kind = "MODIFIED" if (gv, plural, ns, meta["name"]) in self.store else "ADDED"
        self.store[(gv, plural, ns, meta["name"])] = obj
        self.events.append((int(meta["resourceVersion"]), kind, gv, plural, ns, copy.deepcopy(obj)))
        if plural == "services" and self.auto_ready and obj.get("spec", {}).get("selector"):
            # the endpoints controller: a ready address per selected pod (one, here)
            ports = [{"name": p.get("name"), "port": p.get("targetPort", p.get("port"))}
                     for p in obj["spec"].get("ports", [])]
            self.store[("v1", "endpoints", ns, meta["name"])] = {
                "apiVersion": "v1", "kind": "Endpoints",
                "metadata": {"name": meta["name"], "namespace": ns, "uid": str(uuid.uuid4()),
                             "resourceVersion": str(next(self._rv))},
                "subsets": [{"addresses": [{"ip": "10.244.0.10"}], "ports": ports}] if self.endpoints_ready else []}
        return obj

    def _run_profiler_job(self, job: dict) -> None:
        cmd = job["spec"]["template"]["spec"]["containers"][0]["command"]
        if cmd[:3] != ["python3", "-m", "mxserve.profiler.sla"] or self.url is None:
            return
        args = list(cmd[3:])
        try:
            import torch
            if "--measure" in args and not torch.cuda.is_available():
                args.remove("--measure")  # CPU test box: the roofline stands in for the live timings
        except ImportError:
            pass
        os.environ["MXS_KUBE_SERVER"] = self.url
        from ..profiler import sla
        sla.main(args)

    def _start_job(self, gv, ns, job: dict) -> None:
        name = job["metadata"]["name"]

        def run():
            ok = True
            try:
                self.job_runner(copy.deepcopy(job))
            except BaseException:  # noqa: BLE001 - a failing Job
                ok = False
            self.jobs_run.append((name, ok))
            cur = self.store.get((gv, "jobs", ns, name))
            if cur is not None:
                cur["status"] = {"succeeded": 1} if ok else {"failed": 2}
        threading.Thread(target=run, daemon=True).start()

    def writes(self) -> list:
        """Mutating requests received (method, gv, plural, ns, name, sub)."""
        return [e for e in self.log if e[0] in ("POST", "PUT", "PATCH", "DELETE")]

    def objects(self, plural: str, ns: str | None = None) -> list:
        return [o for (gv, p, n, _), o in self.store.items() if p == plural and (ns is None or n == ns)]

    def _build(self) -> FastAPI:
        app = FastAPI()
        srv = self

        def handle(method: str, gv: str, plural: str, ns, name, sub, body, params):
            srv.log.append((method, gv, plural, ns, name, sub))
            key = (gv, plural, ns, name)
            if name is None:
                if method == "GET":
                    items = [copy.deepcopy(o) for (g, p, n, _), o in srv.store.items()
                             if g == gv and p == plural and (ns is None or n == ns)
                             and _match(o["metadata"].get("labels") or {}, params.get("labelSelector"))]
                    last = srv.events[-1][0] if srv.events else 0
                    return 200, {"kind": "List", "apiVersion": gv, "metadata": {"resourceVersion": str(last)},
                                 "items": items}
                if method == "POST":
                    nm = body["metadata"]["name"]
                    if (gv, plural, ns, nm) in srv.store:
                        return 409, {"kind": "Status", "reason": "AlreadyExists", "message": f"{nm} exists"}
                    obj = srv._put(gv, plural, ns, copy.deepcopy(body))
                    if plural == "jobs" and srv.job_runner is not None:
                        srv._start_job(gv, ns, obj)
                    return 201, copy.deepcopy(obj)
                return 405, {}
            cur = srv.store.get(key)
            if cur is None:
                if method == "PUT":
                    return 201, copy.deepcopy(srv._put(gv, plural, ns, copy.deepcopy(body)))
                return 404, {"kind": "Status", "reason": "NotFound", "message": f"{plural} {name} not found"}
            if method == "GET":
                return 200, copy.deepcopy(cur)
            if method == "DELETE":
                del srv.store[key]
                srv.events.append((next(srv._rv), "DELETED", gv, plural, ns, copy.deepcopy(cur)))
                return 200, {"kind": "Status", "status": "Success"}
            if method == "PATCH":
                if sub == "status":
                    cur.setdefault("status", {})
                    _merge(cur["status"], body.get("status", {}))
                    cur["metadata"]["resourceVersion"] = str(next(srv._rv))
                    srv.events.append((int(cur["metadata"]["resourceVersion"]), "MODIFIED", gv, plural, ns,
                                       copy.deepcopy(cur)))
                else:
                    body = {k: v for k, v in body.items() if k != "status"}
                    _merge(cur, body)
                    srv._put(gv, plural, ns, cur)
                return 200, copy.deepcopy(cur)
            if method == "PUT":
                return 200, copy.deepcopy(srv._put(gv, plural, ns, copy.deepcopy(body)))
            return 405, {}

        async def core(request: Request, path: str):
            parts = [p for p in path.split("/") if p]
            # api/v1[/namespaces/ns]/plural[/name][/sub]  |  apis/group/version[/namespaces/ns]/plural[...]
            if parts[0] == "api":
                gv, rest = parts[1], parts[2:]
            else:
                gv, rest = f"{parts[1]}/{parts[2]}", parts[3:]
            ns = None
            if len(rest) >= 2 and rest[0] == "namespaces" and len(rest) > 2:
                ns, rest = rest[1], rest[2:]
            plural = rest[0]
            name = rest[1] if len(rest) > 1 else None
            sub = rest[2] if len(rest) > 2 else None
            body = None
            if request.method in ("POST", "PUT", "PATCH"):
                body = await request.json()
            q = dict(request.query_params)
            if request.method == "GET" and name is None and q.get("watch") in ("true", "1"):
                return StreamingResponse(watch(gv, plural, ns, q), media_type="application/json")
            code, out = handle(request.method, gv, plural, ns, name, sub, body, dict(request.query_params))
            return JSONResponse(out, status_code=code)

        async def watch(gv, plural, ns, q):
            """Newline-delimited watch events after resourceVersion, until timeoutSeconds."""
            srv.log.append(("WATCH", gv, plural, ns, None, None))
            rv = int(q.get("resourceVersion") or 0)
            deadline = time.monotonic() + float(q.get("timeoutSeconds") or 30)
            sel = q.get("labelSelector")
            while time.monotonic() < deadline:
                for ev_rv, kind, g, p, n, obj in list(srv.events):
                    if ev_rv <= rv or g != gv or p != plural or (ns is not None and n != ns):
                        continue
                    rv = ev_rv
                    if _match(obj["metadata"].get("labels") or {}, sel):
                        yield json.dumps({"type": kind, "object": obj}) + "\n"
                await asyncio.sleep(0.05)

        app.add_api_route("/{path:path}", core, methods=["GET", "POST", "PUT", "PATCH", "DELETE"])
        return app


def main(argv=None) -> None:
    import uvicorn
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=16443)
    ap.add_argument("--no-auto-ready", action="store_true")
    a = ap.parse_args(argv)
    uvicorn.run(FakeApiServer(auto_ready=not a.no_auto_ready).app, host="127.0.0.1", port=a.port, log_level="warning")


if __name__ == "__main__":
    main()
