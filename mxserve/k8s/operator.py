"""The mxserve operator: reconciles DynamoGraphDeployment(Request)s (replaces the Dynamo operator
controller-manager).

Level-triggered polling reconcile (robust to missed events, no watch-resume bookkeeping):
  DGDR -> profiling Job from `profilerImage` running mxserve.profiler.sla (live timings on one GPU
          when useAiConfigurator is false, else the MI355X roofline), results published in a
          ConfigMap (state Profiling until the Job ends) -> DGD rendered from the request's ConfigMap
          template (+ workersImage override) -> applied if autoApply; results in status.
          MXS_PROFILER_MODE=inline (or no profilerImage) runs the roofline in the operator instead.
  DGD  -> DCD per service -> Deployment + Service + PodMonitor; DGD status.state = successful once
          every Deployment has its replicas ready
Orphans (children whose DGD is gone) are deleted, as the Kubernetes garbage collector would via
ownerReferences.  `python -m mxserve.k8s.operator [--namespace NS] [--interval S] [--server URL]`.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import time
from typing import Optional

import yaml

from ..profiler import sla
from .client import ApiError, KubeClient
from .resources import (API_VERSION, DCD_KIND, DGD_KIND, DGDR_KIND, NS_LABEL, ValidationError,
                        apply_plan_to_template, parse_dgd, parse_dgdr, render_children, render_dcds,
                        render_profiler_job)

log = logging.getLogger("mxserve.operator")


class Operator:
    def __init__(self, client: KubeClient, namespace: Optional[str] = None, podmonitors: bool = True):
        self.k = client
        self.ns = namespace
        self.podmonitors = podmonitors
        self._pm_disabled = False

    # ------------------------------------------------------------------ DGD
    def reconcile_dgd(self, obj: dict) -> dict:
        ns = obj["metadata"].get("namespace") or self.ns or "default"
        try:
            g = parse_dgd(obj, ns)
        except ValidationError as e:
            st = {"state": "failed", "conditions": [{"type": "Ready", "status": "False", "reason": "InvalidSpec",
                                                      "message": str(e)}]}
            self.k.patch_status(DGD_KIND, obj["metadata"]["name"], ns, st)
            return st
        uids = {}
        for dcd in render_dcds(g):
            cur = self.k.apply(dcd)
            uids[dcd["metadata"]["name"]] = (cur.get("metadata") or {}).get("uid")
        want = set()
        for child in render_children(g, uids):
            if child["kind"] == "PodMonitor" and (not self.podmonitors or self._pm_disabled):
                continue
            try:
                self.k.apply(child)
                want.add((child["kind"], child["metadata"]["name"]))
            except ApiError as e:
                if child["kind"] == "PodMonitor" and e.status == 404:
                    log.info("PodMonitor CRD not installed; skipping PodMonitors")
                    self._pm_disabled = True
                    continue
                raise
        # drop children of services that left the graph
        sel = f"{NS_LABEL}={ns}-{g.name}"
        for kind in ("Deployment", "Service", DCD_KIND):
            for o in self.k.list(kind, ns, sel):
                n = o["metadata"]["name"]
                if kind == DCD_KIND:
                    if n not in uids:
                        self.k.delete(kind, n, ns)
                elif (kind, n) not in want:
                    self.k.delete(kind, n, ns)
        # status
        services, ready_all = {}, True
        for s in g.services:
            name = f"{g.name}-{s.dns_name}"
            d = self.k.get("Deployment", name, ns) or {}
            ready = int((d.get("status") or {}).get("readyReplicas", 0) or 0)
            services[s.key] = {"componentType": s.component_type, "replicas": s.replicas, "readyReplicas": ready}
            ready_all &= ready >= s.replicas
        st = {"state": "successful" if ready_all else "pending", "services": services,
              "conditions": [{"type": "Ready", "status": "True" if ready_all else "False",
                              "reason": "AllServicesReady" if ready_all else "WaitingForReplicas"}]}
        self.k.patch_status(DGD_KIND, g.name, ns, st)
        for dname, uid in uids.items():
            self.k.patch_status(DCD_KIND, dname, ns, {"state": st["state"]})
        return st

    # ------------------------------------------------------------------ DGDR
    def reconcile_dgdr(self, obj: dict) -> dict:
        ns = obj["metadata"].get("namespace") or self.ns or "default"
        if (obj.get("status") or {}).get("state") in ("Successful", "Deployed"):
            return obj["status"]
        try:
            r = parse_dgdr(obj, ns)
        except ValidationError as e:
            st = {"state": "Failed", "message": str(e)}
            self.k.patch_status(DGDR_KIND, obj["metadata"]["name"], ns, st)
            return st
        if r.profiler_image and os.environ.get("MXS_PROFILER_MODE", "job") == "job":
            p = self._profiling_job(r, ns)
            if isinstance(p, dict) and "state" in p:  # still profiling, or the Job failed
                self.k.patch_status(DGDR_KIND, r.name, ns, p)
                return p
        else:
            p = sla.plan(r.model, r.isl, r.osl, r.ttft_ms, r.itl_ms, system="mi355x")
        if not p["feasible"]:
            st = {"state": "Failed", "message": "SLA not reachable on one node", "profilingResults": p}
            self.k.patch_status(DGDR_KIND, r.name, ns, st)
            return st
        roles = {}
        if p["disagg"]:
            roles = {"prefill": p["disagg"]["prefill"], "decode": p["disagg"]["decode"]}
        if p["agg"]:
            roles["agg"] = p["agg"]
        template = None
        if r.config_map:
            cm = self.k.get("ConfigMap", r.config_map, ns)
            if cm is None:
                st = {"state": "Pending", "message": f"ConfigMap {r.config_map} not found"}
                self.k.patch_status(DGDR_KIND, r.name, ns, st)
                return st
            template = yaml.safe_load((cm.get("data") or {}).get(r.config_key or "disagg.yaml", ""))
        if template is None:
            template = default_template(r.model)
        dgd = apply_plan_to_template(template, roles, r)
        if r.uid:
            dgd["metadata"]["ownerReferences"] = [{"apiVersion": API_VERSION, "kind": DGDR_KIND, "name": r.name,
                                                   "uid": r.uid, "controller": True}]
        st = {"state": "Successful", "profilingResults": p, "generatedDeployment": dgd,
              "deployment": {"name": dgd["metadata"]["name"], "applied": r.auto_apply}}
        if r.auto_apply:
            self.k.apply(dgd)
        self.k.patch_status(DGDR_KIND, r.name, ns, st)
        return st

    def _profiling_job(self, r, ns: str) -> dict:
        """Start the DGDR's profiling Job once; return its results, or a status while it runs."""
        job_name, cm_name = f"{r.name}-profile", f"{r.name}-profiling-results"
        job = self.k.get("Job", job_name, ns)
        if job is None:
            for obj in render_profiler_job(r, job_name, cm_name):
                self.k.apply(obj)
            log.info("DGDR %s/%s: profiling Job %s started (%s)", ns, r.name, job_name,
                     "live on 1 GPU" if r.measure else "roofline")
            return {"state": "Profiling", "message": f"Job {job_name} started", "profilingJob": job_name}
        js = job.get("status") or {}
        if int(js.get("succeeded") or 0) >= 1:
            cm = self.k.get("ConfigMap", cm_name, ns)
            if cm is None or "results.json" not in (cm.get("data") or {}):
                return {"state": "Failed", "message": f"Job {job_name} succeeded without publishing {cm_name}"}
            return json.loads(cm["data"]["results.json"])
        if int(js.get("failed") or 0) > int((job.get("spec") or {}).get("backoffLimit", 1)):
            return {"state": "Failed", "message": f"profiling Job {job_name} failed", "profilingJob": job_name}
        return {"state": "Profiling", "message": f"Job {job_name} running", "profilingJob": job_name}

    # ------------------------------------------------------------------ loop
    def gc_orphans(self) -> None:
        """Delete DCDs (and their children) whose DGD no longer exists."""
        for dcd in self.k.list(DCD_KIND, self.ns):
            owners = dcd["metadata"].get("ownerReferences") or []
            ns = dcd["metadata"].get("namespace")
            for o in owners:
                if o.get("kind") == DGD_KIND and self.k.get(DGD_KIND, o["name"], ns) is None:
                    n = dcd["metadata"]["name"]
                    for kind in ("Deployment", "Service", "PodMonitor"):
                        try:
                            self.k.delete(kind, n, ns)
                        except ApiError:
                            pass
                    self.k.delete(DCD_KIND, n, ns)

    def reconcile_all(self) -> None:
        for obj in self.k.list(DGDR_KIND, self.ns):
            try:
                self.reconcile_dgdr(obj)
            except Exception:  # noqa: BLE001 - keep reconciling the others
                log.exception("DGDR %s", obj["metadata"].get("name"))
        for obj in self.k.list(DGD_KIND, self.ns):
            try:
                self.reconcile_dgd(obj)
            except Exception:  # noqa: BLE001
                log.exception("DGD %s", obj["metadata"].get("name"))
        self.gc_orphans()

    def run(self, interval: float = 5.0) -> None:
        while True:
            try:
                self.reconcile_all()
            except Exception:  # noqa: BLE001 - apiserver hiccup
                log.exception("reconcile pass failed")
            time.sleep(interval)


def default_template(model: str) -> dict:
    """Disaggregated graph used when a DGDR names no ConfigMap template."""
    def worker(role: str) -> dict:
        return {"componentType": "worker", "subComponentType": role, "replicas": 1, "resources": {"limits": {"gpu": "1"}},
                "envFromSecret": "hf-token-secret",
                "extraPodSpec": {"mainContainer": {"command": ["python3", "-m", "dynamo.vllm"],
                                                   "args": ["--model", model, f"--is-{role}-worker"]}}}
    return {"apiVersion": API_VERSION, "kind": DGD_KIND, "metadata": {"name": "sla-disagg"},
            "spec": {"services": {"Frontend": {"componentType": "frontend", "replicas": 1},
                                  "VllmPrefillWorker": worker("prefill"), "VllmDecodeWorker": worker("decode")}}}


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(prog="python -m mxserve.k8s.operator")
    ap.add_argument("--namespace", default=None, help="watch one namespace (default: all)")
    ap.add_argument("--interval", type=float, default=5.0)
    ap.add_argument("--server", default=None, help="apiserver URL (default: in-cluster / kubeconfig)")
    ap.add_argument("--no-podmonitors", action="store_true")
    a = ap.parse_args(argv)
    from ..utils.logs import setup_logging
    setup_logging()
    op = Operator(KubeClient(a.server) if a.server else KubeClient(), a.namespace, not a.no_podmonitors)
    op.run(a.interval)


if __name__ == "__main__":
    main()
