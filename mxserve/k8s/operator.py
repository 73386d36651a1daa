"""The mxserve operator: reconciles DynamoGraphDeployment(Request)s (replaces the Dynamo operator
controller-manager).

Level-triggered reconcile, woken by watches and re-run as a periodic resync (robust to missed
events: a watch only shortens the wait, the full pass always reads the current state):
  DGDR -> profiling Job from `profilerImage` running mxserve.profiler.sla (live timings on one GPU
          when useAiConfigurator is false, else the MI355X roofline), results published in a
          ConfigMap (state Profiling until the Job ends) -> DGD rendered from the request's ConfigMap
          template (+ workersImage override) -> applied if autoApply; results in status.
          MXS_PROFILER_MODE=inline (or no profilerImage) runs the roofline in the operator instead.
  DGD  -> DCD per service -> Deployment + Service + PodMonitor; DGD status.state = successful once
          every Deployment has its replicas ready (P/D group pods: every shape Deployment's pods)
Writes are skipped when nothing changed (a spec hash on every child, status compared before it is
patched), so an idle operator only reads; state transitions and image rewrites are recorded as
Events.
Orphans (children whose DGD is gone) are deleted, as the Kubernetes garbage collector would via
ownerReferences.  `python -m mxserve.k8s.operator [--namespace NS] [--interval S] [--server URL]`.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import threading
import time
from typing import Optional

import yaml

from ..profiler import sla
from .client import ApiError, KubeClient
from .resources import (API_VERSION, DCD_KIND, DGD_KIND, DGDR_KIND, NS_LABEL, ValidationError,
                        apply_plan_to_template, group_deployment_name, group_shapes, image_rewrites, parse_dgd,
                        parse_dgdr, pd_groups, pd_pairs, render_children, render_dcds, render_profiler_job)

log = logging.getLogger("mxserve.operator")


class LeaderElector:
    """Lease-based leader election (coordination.k8s.io/v1 Lease, the client-go protocol's fields):
    the holder renews spec.renewTime well inside leaseDurationSeconds; another replica takes the
    lease over only once it has expired.  Writes carry the lease's resourceVersion, so two replicas
    racing for an expired lease cannot both win (the apiserver answers the loser 409)."""

    def __init__(self, client: KubeClient, namespace: str, name: str = "mxserve-operator",
                 identity: Optional[str] = None, lease_s: float = 30.0):
        import socket
        self.k, self.ns, self.name = client, namespace, name
        self.id = identity or f"{socket.gethostname()}-{os.getpid()}"
        self.lease_s = lease_s
        self.leader = False
        self.observed = False  # one election step reached the apiserver (leader or healthy standby)

    @staticmethod
    def _now() -> str:
        return time.strftime("%Y-%m-%dT%H:%M:%S.000000Z", time.gmtime())

    @staticmethod
    def _parse(ts: Optional[str]) -> float:
        if not ts:
            return 0.0
        import calendar
        return calendar.timegm(time.strptime(ts.split(".")[0].rstrip("Z"), "%Y-%m-%dT%H:%M:%S"))

    def step(self) -> bool:
        """Acquire or renew; returns whether this replica leads now."""
        try:
            lease = self.k.get("Lease", self.name, self.ns)
            spec = {"holderIdentity": self.id, "leaseDurationSeconds": int(self.lease_s), "renewTime": self._now()}
            if lease is None:
                self.k.create({"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                               "metadata": {"name": self.name, "namespace": self.ns},
                               "spec": dict(spec, acquireTime=spec["renewTime"], leaseTransitions=0)})
                self.leader = self.observed = True
                return True
            cur = lease.get("spec") or {}
            holder = cur.get("holderIdentity")
            expired = time.time() > self._parse(cur.get("renewTime")) + float(cur.get("leaseDurationSeconds") or
                                                                               self.lease_s)
            self.observed = True
            if holder != self.id and not expired:
                self.leader = False
                return False
            if holder != self.id:
                spec.update(acquireTime=spec["renewTime"], leaseTransitions=int(cur.get("leaseTransitions") or 0) + 1)
            self.k.merge_patch("Lease", self.name, self.ns,
                               {"metadata": {"resourceVersion": lease["metadata"].get("resourceVersion")},
                                "spec": spec})
            self.leader = True
        except ApiError as e:
            log.info("leader election: %s", e)
            self.leader = False
        return self.leader

    def release(self) -> bool:
        """Give the lease up (SIGTERM of the leader): clear the holder and back-date renewTime, so a
        standby takes over at its next step instead of after leaseDurationSeconds (the client-go
        ReleaseOnCancel behaviour).  Returns whether this replica held it."""
        if not self.leader:
            return False
        try:
            lease = self.k.get("Lease", self.name, self.ns)
            if lease is None or (lease.get("spec") or {}).get("holderIdentity") != self.id:
                return False
            self.k.merge_patch("Lease", self.name, self.ns,
                               {"metadata": {"resourceVersion": lease["metadata"].get("resourceVersion")},
                                "spec": {"holderIdentity": "", "leaseDurationSeconds": 1,
                                         "renewTime": "1970-01-01T00:00:00.000000Z"}})
            return True
        except ApiError as e:
            log.info("lease release: %s", e)
            return False
        finally:
            self.leader = False


class Operator:
    def __init__(self, client: KubeClient, namespace: Optional[str] = None, podmonitors: bool = True):
        self.k = client
        self.ns = namespace
        self.podmonitors = podmonitors
        self._pm_disabled = False
        self._wake = threading.Event()
        self.watch_errors = 0
        # liveness: each watch thread and the reconcile loop stamp a beat every cycle; /healthz fails
        # when one has not cycled within twice its period (a hung watch thread is otherwise invisible)
        self.watch_timeout_s = 60.0
        self.interval = 30.0
        self.beats: dict = {}
        self.last_pass: Optional[float] = None
        self.elector: Optional[LeaderElector] = None

    def _set_status(self, kind: str, obj: Optional[dict], name: str, ns: str, st: dict) -> None:
        """Patch status only when it differs from what the object already carries."""
        cur = (obj or {}).get("status") or {}
        if all(cur.get(k) == v for k, v in st.items()):
            return
        self.k.patch_status(kind, name, ns, st)
        if obj is not None and cur.get("state") != st.get("state") and st.get("state"):
            self.k.event(obj, f"State{str(st['state']).capitalize()}",
                         f"{kind} {name}: state {cur.get('state') or 'none'} -> {st['state']}",
                         "Warning" if str(st["state"]).lower() == "failed" else "Normal")

    def _service_ready(self, g, ns: str) -> dict:
        """{service key: (ready workers/replicas, wanted)}.  A P/D-grouped decode service runs its
        workers AND the prefill service's in group pods, one Deployment per pod shape: ready decode
        (prefill) workers = sum over shapes of ready pods x decode (prefill) workers per pod."""
        out = {}
        pair = pd_pairs(g)
        if pair is not None:
            dec, pre = pair
            name = f"{g.name}-{dec.dns_name}"
            rd = rp = 0
            for k, (n_pre, n_dec, count) in enumerate(group_shapes(pd_groups(dec, pre))):
                d = self.k.get("Deployment", group_deployment_name(name, k), ns) or {}
                ready = min(count, int((d.get("status") or {}).get("readyReplicas", 0) or 0))
                rd += ready * n_dec
                rp += ready * n_pre
            out[dec.key] = (rd, dec.replicas)
            out[pre.key] = (rp, pre.replicas)
        for s in g.services:
            if s.key in out:
                continue
            d = self.k.get("Deployment", f"{g.name}-{s.dns_name}", ns) or {}
            out[s.key] = (int((d.get("status") or {}).get("readyReplicas", 0) or 0), s.replicas)
        return out

    # ------------------------------------------------------------------ DGD
    def reconcile_dgd(self, obj: dict) -> dict:
        ns = obj["metadata"].get("namespace") or self.ns or "default"
        try:
            g = parse_dgd(obj, ns)
            render_children(g)  # layout errors (e.g. a P/D group that cannot fit) surface as InvalidSpec
        except ValidationError as e:
            st = {"state": "failed", "conditions": [{"type": "Ready", "status": "False", "reason": "InvalidSpec",
                                                      "message": str(e)}]}
            self._set_status(DGD_KIND, obj, obj["metadata"]["name"], ns, st)
            return st
        uids, dcd_objs = {}, {}
        for dcd in render_dcds(g):
            cur = self.k.apply(dcd)
            uids[dcd["metadata"]["name"]] = (cur.get("metadata") or {}).get("uid")
            dcd_objs[dcd["metadata"]["name"]] = cur
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
        ready = self._service_ready(g, ns)
        for s in g.services:
            r, want = ready[s.key]
            services[s.key] = {"componentType": s.component_type, "replicas": s.replicas, "readyReplicas": r}
            ready_all &= r >= want
        st = {"state": "successful" if ready_all else "pending", "services": services,
              "conditions": [{"type": "Ready", "status": "True" if ready_all else "False",
                              "reason": "AllServicesReady" if ready_all else "WaitingForReplicas"}]}
        self._set_status(DGD_KIND, obj, g.name, ns, st)
        rewrites = image_rewrites(g)
        for s in g.services:
            dname = f"{g.name}-{s.dns_name}"
            dst = {"state": st["state"]}
            if s.key in rewrites:  # an image the node cannot run, replaced (resources.map_image)
                dst["imageRewrite"] = rewrites[s.key]
            cur = dcd_objs.get(dname)
            if cur is not None and "imageRewrite" in dst and ((cur.get("status") or {}).get("imageRewrite")
                                                               != dst["imageRewrite"]):
                self.k.event(cur, "ImageRewritten", f"{dst['imageRewrite']['from']} -> {dst['imageRewrite']['to']}")
            self._set_status(DCD_KIND, cur, dname, ns, dst)
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
            self._set_status(DGDR_KIND, obj, obj["metadata"]["name"], ns, st)
            return st
        if r.profiler_image and os.environ.get("MXS_PROFILER_MODE", "job") == "job":
            p = self._profiling_job(r, ns)
            if isinstance(p, dict) and "state" in p:  # still profiling, or the Job failed
                self._set_status(DGDR_KIND, obj, r.name, ns, p)
                return p
        else:
            p = sla.plan(r.model, r.isl, r.osl, r.ttft_ms, r.itl_ms, system="mi355x")
        if not p["feasible"]:
            st = {"state": "Failed", "message": "SLA not reachable on one node", "profilingResults": p}
            self._set_status(DGDR_KIND, obj, r.name, ns, st)
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
                self._set_status(DGDR_KIND, obj, r.name, ns, st)
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
        self._set_status(DGDR_KIND, obj, r.name, ns, st)
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

    def _watch_loop(self, kind: str, stop: threading.Event) -> None:
        """List + watch `kind` from the list's resourceVersion; every event wakes the reconcile loop.
        Re-lists on expiry (410) and backs off on errors; an apiserver without watch support leaves
        the operator on its resync interval."""
        rv, backoff = "", 1.0
        while not stop.is_set():
            self.beats[kind] = time.monotonic()
            try:
                if not rv:
                    _, rv = self.k.list_rv(kind, self.ns)
                for ev in self.k.watch(kind, self.ns, rv, timeout_s=self.watch_timeout_s):
                    self.beats[kind] = time.monotonic()
                    if ev.get("type") == "ERROR":
                        rv = ""  # expired resourceVersion: re-list
                        break
                    rv = str(((ev.get("object") or {}).get("metadata") or {}).get("resourceVersion") or rv)
                    if ev.get("type") != "BOOKMARK":
                        self._wake.set()
                    if stop.is_set():
                        return
                backoff = 1.0
            except Exception as e:  # noqa: BLE001 - apiserver hiccup / no watch support
                self.watch_errors += 1
                rv = ""
                log.debug("watch %s: %s", kind, e)
                if stop.wait(backoff):
                    return
                backoff = min(self.watch_timeout_s, backoff * 2)

    def start_watches(self, kinds=(DGD_KIND, DGDR_KIND, "Deployment", "Job")) -> threading.Event:
        stop = threading.Event()
        now = time.monotonic()
        for kind in kinds:
            self.beats[kind] = now
            threading.Thread(target=self._watch_loop, args=(kind, stop), name=f"watch-{kind}", daemon=True).start()
        return stop

    def run(self, interval: float = 30.0, watch: bool = True, stop: Optional[threading.Event] = None) -> None:
        """Reconcile on every watch event (coalesced) and at least every `interval` seconds."""
        stop = stop or threading.Event()
        self.interval = interval
        wstop = self.start_watches() if watch else None
        try:
            while not stop.is_set():
                self._wake.clear()
                self.beats["reconcile"] = time.monotonic()
                if self.elector is not None and not self.elector.step():
                    stop.wait(min(interval, self.elector.lease_s / 3))  # standby: retry for the lease
                    continue
                try:
                    self.reconcile_all()
                    self.last_pass = time.monotonic()
                except Exception:  # noqa: BLE001 - apiserver hiccup
                    log.exception("reconcile pass failed")
                wait = interval if self.elector is None else min(interval, self.elector.lease_s / 3)
                self._wake.wait(wait)  # a leader wakes at least every third of its lease to renew it
                time.sleep(0.2)  # coalesce a burst of events into one pass
        finally:
            if wstop is not None:
                wstop.set()


    # ------------------------------------------------------------------ probes
    def health(self) -> tuple:
        """(alive, detail): every watch thread and the reconcile loop cycled within twice its period."""
        now = time.monotonic()
        detail, ok = {}, True
        for name, t in sorted(self.beats.items()):
            limit = 2 * (self.interval + 5 if name == "reconcile" else self.watch_timeout_s)
            age = now - t
            detail[name] = round(age, 1)
            if age > limit:
                ok = False
                detail.setdefault("stalled", []).append(name)
        return ok, detail

    def ready(self) -> bool:
        """Ready once this replica works: a reconcile pass completed, or -- with leader election -- an
        election step reached the apiserver (the leader after its first pass, a standby as soon as it
        sees the lease held).  Leadership only gates reconciling: a standby reporting unready would
        stall a RollingUpdate (maxUnavailable 0) for as long as the old leader renews its lease."""
        if self.elector is None:
            return self.last_pass is not None
        if self.elector.leader:
            return self.last_pass is not None
        return self.elector.observed

    def serve_probes(self, port: int, host: str = "0.0.0.0"):
        """/healthz (liveness) and /readyz (readiness) on a daemon thread; returns the server."""
        import http.server
        import json as _json
        op = self

        class H(http.server.BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802
                if self.path.startswith("/healthz"):
                    ok, detail = op.health()
                elif self.path.startswith("/readyz"):
                    ok, detail = op.ready(), {"last_pass": op.last_pass is not None}
                else:
                    ok, detail = False, {"error": "not found"}
                body = _json.dumps({"ok": ok, **detail}).encode()
                self.send_response(200 if ok else (404 if "error" in detail else 503))
                self.send_header("content-type", "application/json")
                self.send_header("content-length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):
                pass

        srv = http.server.ThreadingHTTPServer((host, port), H)
        threading.Thread(target=srv.serve_forever, name="operator-probes", daemon=True).start()
        return srv


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
    ap.add_argument("--interval", type=float, default=30.0, help="resync period (watch events reconcile at once)")
    ap.add_argument("--no-watch", action="store_true", help="poll every --interval instead of watching")
    ap.add_argument("--server", default=None, help="apiserver URL (default: in-cluster / kubeconfig)")
    ap.add_argument("--no-podmonitors", action="store_true")
    ap.add_argument("--health-port", type=int, default=int(os.environ.get("MXS_OPERATOR_HEALTH_PORT", "8081")),
                    help="/healthz and /readyz (0: off)")
    ap.add_argument("--leader-elect", action="store_true", help="Lease-based leader election (replicas > 1)")
    ap.add_argument("--lease-namespace", default=os.environ.get("POD_NAMESPACE", "default"))
    a = ap.parse_args(argv)
    from ..utils.logs import setup_logging
    setup_logging()
    client = KubeClient(a.server) if a.server else KubeClient()
    op = Operator(client, a.namespace, not a.no_podmonitors)
    if a.leader_elect:
        op.elector = LeaderElector(client, a.lease_namespace)
    if a.health_port:
        op.serve_probes(a.health_port)
    stop = threading.Event()

    def on_term(signum, frame):  # noqa: ARG001
        stop.set()
        op._wake.set()
    import signal
    signal.signal(signal.SIGTERM, on_term)
    try:
        op.run(a.interval, watch=not a.no_watch, stop=stop)
    finally:
        if op.elector is not None and op.elector.release():
            log.info("released the operator lease")


if __name__ == "__main__":
    main()
