"""DynamoGraphDeployment (DGD) / DynamoGraphDeploymentRequest (DGDR) schema + rendering.

Same group/version/kinds as the reference manifests (`nvidia.com/v1alpha1`, examples/deploy/vllm/
agg.yaml:6-7, examples/dgdr/trtllm/dgdr.yaml:6-7) so they apply unchanged; SURVEY.md Appendix A.3
lists the fields honoured here.  Rendering (pure functions, unit-tested without a cluster):

  DGD  -> one DynamoComponentDeployment (DCD) per service (owned by the DGD)
  DCD  -> Deployment + Service (+ PodMonitor), names `<dgd>-<service key lowercased>`, label
          `nvidia.com/dynamo-namespace=<ns>-<dgd>` (what deploy-incluster.sh:252-256 selects on),
          single-container pods, `resources.limits.gpu` -> `amd.com/gpu` (AMD GPU Operator / ROCm
          device plugin), readiness = /health (true only once the model is servable).
"""
from __future__ import annotations

import copy
import fnmatch
import json
import os
import re
from dataclasses import dataclass, field
from typing import Optional

GROUP = "nvidia.com"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"
DGD_KIND = "DynamoGraphDeployment"
DGDR_KIND = "DynamoGraphDeploymentRequest"
DCD_KIND = "DynamoComponentDeployment"
NS_LABEL = "nvidia.com/dynamo-namespace"
COMPONENT_LABEL = "nvidia.com/dynamo-component"
TYPE_LABEL = "nvidia.com/dynamo-component-type"
SUBTYPE_LABEL = "nvidia.com/dynamo-sub-component-type"
GPU_RESOURCE = os.environ.get("MXS_GPU_RESOURCE", "amd.com/gpu")
DEFAULT_IMAGE = os.environ.get("MXS_DEFAULT_IMAGE", "mxserve/mxserve-rocm:0.1.0")
# set on the operator Deployment by install-dynamo-1node.sh; passed to every component it renders
PROMETHEUS_ENDPOINT = os.environ.get("PROMETHEUS_ENDPOINT", "")
FRONTEND_PORT = 8000
WORKER_PORT = 8081
# The reference pins NVIDIA's CUDA runtime images on every service
# (/root/reference/examples/deploy/vllm/agg.yaml:17,27; examples/dgdr/trtllm/disagg.yaml:17,28,53);
# scheduled unchanged on an MI355X node they cannot run.  Such images are rewritten to the mxserve
# image (which also provides the reference's /workspace layout, docker/Dockerfile), and the rewrite is
# recorded in the DCD status.  MXS_IMAGE_MAP="<glob>=<image>;..." adds mappings (checked first);
# MXS_IMAGE_MAP=off keeps every image as written.
BUILTIN_IMAGE_MAP = [("nvcr.io/nvidia/ai-dynamo/*-runtime:*", None), ("nvcr.io/nvidia/ai-dynamo/*", None)]

_DNS = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$")


class ValidationError(ValueError):
    pass


@dataclass
class ServiceSpec:
    key: str
    component_type: str  # frontend | worker | planner | ...
    sub_component_type: Optional[str] = None  # prefill | decode
    replicas: int = 1
    gpus: int = 0
    env_from_secret: Optional[str] = None
    envs: list = field(default_factory=list)
    volume_mounts: list = field(default_factory=list)
    image: Optional[str] = None
    working_dir: Optional[str] = None
    command: Optional[list] = None
    args: Optional[list] = None

    @property
    def dns_name(self) -> str:
        return self.key.lower()


@dataclass
class GraphSpec:
    name: str
    namespace: str
    services: list
    pvcs: list = field(default_factory=list)
    uid: Optional[str] = None


def _int(v, what: str) -> int:
    try:
        return int(str(v))
    except (TypeError, ValueError):
        raise ValidationError(f"{what} must be an integer, got {v!r}") from None


def parse_dgd(obj: dict, namespace: Optional[str] = None) -> GraphSpec:
    if obj.get("apiVersion") != API_VERSION or obj.get("kind") != DGD_KIND:
        raise ValidationError(f"expected {API_VERSION} {DGD_KIND}, got {obj.get('apiVersion')} {obj.get('kind')}")
    meta = obj.get("metadata") or {}
    name = meta.get("name")
    if not name or not _DNS.match(name):
        raise ValidationError(f"metadata.name {name!r} is not a DNS-1123 label")
    spec = obj.get("spec") or {}
    svcs = spec.get("services") or {}
    if not isinstance(svcs, dict) or not svcs:
        raise ValidationError("spec.services must be a non-empty map")
    out = []
    for key, s in svcs.items():
        s = s or {}
        ctype = s.get("componentType")
        if ctype not in ("frontend", "worker", "planner", "main"):
            raise ValidationError(f"services.{key}.componentType must be frontend|worker|planner, got {ctype!r}")
        sub = s.get("subComponentType")
        if sub is not None and sub not in ("prefill", "decode"):
            raise ValidationError(f"services.{key}.subComponentType must be prefill|decode")
        lim = ((s.get("resources") or {}).get("limits") or {})
        mc = ((s.get("extraPodSpec") or {}).get("mainContainer") or {})
        for vm in s.get("volumeMounts") or []:
            if "name" not in vm or "mountPoint" not in vm:
                raise ValidationError(f"services.{key}.volumeMounts entries need name and mountPoint")
        for e in s.get("envs") or []:
            if "name" not in e:
                raise ValidationError(f"services.{key}.envs entries need a name")
        if not _DNS.match(f"{name}-{key.lower()}"):
            raise ValidationError(f"service key {key!r} does not form a valid DNS name")
        out.append(ServiceSpec(
            key=key, component_type=ctype, sub_component_type=sub, replicas=_int(s.get("replicas", 1), "replicas"),
            gpus=_int(lim.get("gpu", 0), f"services.{key}.resources.limits.gpu"),
            env_from_secret=s.get("envFromSecret"), envs=list(s.get("envs") or []),
            volume_mounts=list(s.get("volumeMounts") or []), image=mc.get("image"),
            working_dir=mc.get("workingDir"), command=mc.get("command"), args=mc.get("args")))
    if not any(s.component_type == "frontend" for s in out):
        raise ValidationError("a graph needs one frontend service")
    pvcs = list(spec.get("pvcs") or [])
    for p in pvcs:
        if "name" not in p:
            raise ValidationError("spec.pvcs entries need a name")
    known = {p["name"] for p in pvcs}
    for s in out:
        for vm in s.volume_mounts:
            if vm["name"] not in known:
                raise ValidationError(f"volumeMount {vm['name']!r} of {s.key} is not declared in spec.pvcs")
    return GraphSpec(name=name, namespace=namespace or meta.get("namespace") or "default", services=out,
                     pvcs=pvcs, uid=meta.get("uid"))


def image_map() -> list:
    """[(glob, image or None = the default image)] in match order."""
    env = os.environ.get("MXS_IMAGE_MAP", "")
    if env.strip().lower() == "off":
        return []
    out = []
    for part in env.split(";"):
        if "=" in part:
            pat, img = part.split("=", 1)
            if pat.strip() and img.strip():
                out.append((pat.strip(), img.strip()))
    return out + BUILTIN_IMAGE_MAP


def map_image(image: Optional[str]) -> tuple:
    """(image to run, the image it replaced or None)."""
    if not image:
        return DEFAULT_IMAGE, None
    for pat, repl in image_map():
        if fnmatch.fnmatchcase(image, pat):
            new = repl or DEFAULT_IMAGE
            return new, (image if new != image else None)
    return image, None


def image_rewrites(g: "GraphSpec") -> dict:
    """{service key: {"from": original, "to": image}} for every service whose image was mapped."""
    out = {}
    for s in g.services:
        new, old = map_image(s.image)
        if old:
            out[s.key] = {"from": old, "to": new}
    return out


def _owner(kind: str, name: str, uid: Optional[str]) -> list:
    if not uid:
        return []
    return [{"apiVersion": API_VERSION, "kind": kind, "name": name, "uid": uid, "controller": True,
             "blockOwnerDeletion": True}]


def frontend_url(g: GraphSpec) -> str:
    fe = next(s for s in g.services if s.component_type == "frontend")
    return f"http://{g.name}-{fe.dns_name}.{g.namespace}.svc.cluster.local:{FRONTEND_PORT}"


def render_dcds(g: GraphSpec) -> list[dict]:
    """DGD -> DynamoComponentDeployment objects (one per service)."""
    out = []
    for s in g.services:
        out.append({
            "apiVersion": API_VERSION, "kind": DCD_KIND,
            "metadata": {"name": f"{g.name}-{s.dns_name}", "namespace": g.namespace,
                         "labels": {NS_LABEL: f"{g.namespace}-{g.name}", COMPONENT_LABEL: s.key},
                         "ownerReferences": _owner(DGD_KIND, g.name, g.uid)},
            "spec": {"dynamoNamespace": f"{g.namespace}-{g.name}", "serviceName": s.key,
                     "componentType": s.component_type, "subComponentType": s.sub_component_type,
                     "replicas": s.replicas, "gpus": s.gpus, "image": map_image(s.image)[0]}})
    return out


def _served_model(g: GraphSpec) -> str:
    """The model a graph's workers serve, read from their flag dialects (planner sizing)."""
    for s in g.services:
        args = [str(a) for a in (s.args or [])]
        for flag in ("--served-model-name", "--model", "--model-path"):
            if flag in args and args.index(flag) + 1 < len(args):
                return args[args.index(flag) + 1]
    return "meta-llama/Llama-3.2-1B-Instruct"


def _default_command(g: GraphSpec, s: ServiceSpec) -> list:
    if s.component_type == "frontend":
        return ["python3", "-m", "dynamo.frontend"]
    if s.component_type == "planner":
        # SLA planner: reads the frontend counters from Prometheus (PROMETHEUS_ENDPOINT, handed down
        # by the operator from the installer) and scales this graph's worker replicas
        return ["python3", "-m", "mxserve.planner.planner", "--namespace", g.namespace, "--dgd", g.name,
                "--model", _served_model(g)]
    return ["python3", "-m", "mxserve.worker"]


# Streamed tokens per second one MI355X worker produces at the headline point (BENCH: ~20-24 k) and
# one frontend process forwards with headroom (scripts/frontend_load.py: 125 k tok/s over 4
# processes at a 17 ms TTFT p50, ~22-26 us of CPU per token: ~38 k/s at 100 % of a core).
TOKENS_PER_GPU = 24000
TOKENS_PER_FRONTEND_PROC = 27000


def frontend_procs(g: GraphSpec) -> int:
    """Frontend processes for a graph: enough cores for the tokens its worker GPUs stream (prefill-
    only workers stream nothing), 2..16; MXS_FRONTEND_PROCS (operator env) overrides."""
    if os.environ.get("MXS_FRONTEND_PROCS"):
        return int(os.environ["MXS_FRONTEND_PROCS"])
    gpus = sum(max(1, s.gpus) * max(0, s.replicas) for s in g.services
               if s.component_type == "worker" and s.sub_component_type != "prefill")
    return max(2, min(16, -(-gpus * TOKENS_PER_GPU // TOKENS_PER_FRONTEND_PROC)))


def _container(g: GraphSpec, s: ServiceSpec) -> dict:
    is_fe = s.component_type == "frontend"
    port = FRONTEND_PORT if is_fe else WORKER_PORT
    cmd = s.command or _default_command(g, s)
    env = [{"name": "DYN_NAMESPACE", "value": f"{g.namespace}-{g.name}"},
           {"name": "POD_IP", "valueFrom": {"fieldRef": {"fieldPath": "status.podIP"}}},
           {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}]
    if PROMETHEUS_ENDPOINT:
        env.append({"name": "PROMETHEUS_ENDPOINT", "value": PROMETHEUS_ENDPOINT})
    if is_fe:  # frontend processes on the port, sized for the graph's GPUs (frontend_procs)
        env += [{"name": "DYN_HTTP_PORT", "value": str(FRONTEND_PORT)},
                {"name": "MXS_FRONTEND_PROCS", "value": str(frontend_procs(g))}]
    else:
        env += [{"name": "MXS_FRONTEND_URL", "value": frontend_url(g)},
                {"name": "DYN_SYSTEM_PORT", "value": str(WORKER_PORT)}]
    env += [dict(e) for e in s.envs]
    c = {"name": "main", "image": map_image(s.image)[0], "command": list(cmd), "env": env,
         "ports": [{"name": "http" if is_fe else "system", "containerPort": port}],
         "readinessProbe": {"httpGet": {"path": "/health", "port": port}, "periodSeconds": 5,
                            "failureThreshold": 720},
         "livenessProbe": {"httpGet": {"path": "/live", "port": port}, "periodSeconds": 10,
                           "initialDelaySeconds": 30, "failureThreshold": 6}}
    if s.args:
        c["args"] = [str(a) for a in s.args]
    if s.working_dir:
        c["workingDir"] = s.working_dir
    if s.env_from_secret:
        c["envFrom"] = [{"secretRef": {"name": s.env_from_secret, "optional": True}}]
    if s.gpus:
        c["resources"] = {"limits": {GPU_RESOURCE: str(s.gpus)}, "requests": {GPU_RESOURCE: str(s.gpus)}}
    elif is_fe:  # one core per frontend process (the streaming work is per-process CPU)
        c["resources"] = {"requests": {"cpu": str(frontend_procs(g)), "memory": "2Gi"}}
    if s.volume_mounts:
        c["volumeMounts"] = [{"name": vm["name"], "mountPath": vm["mountPoint"]} for vm in s.volume_mounts]
    if s.gpus:  # shared memory for the TP ranks' host-side metadata and RCCL
        c.setdefault("volumeMounts", []).append({"name": "dshm", "mountPath": "/dev/shm"})
    return c


PAIR_LABEL = "mxserve.io/pd-pair"
SHAPE_LABEL = "mxserve.io/pd-group-shape"
# GPUs of one node: a P/D group pod never asks for more (single node)
NODE_GPUS = int(os.environ.get("MXS_NODE_GPUS", "8"))


def pd_pairs(g: GraphSpec) -> Optional[tuple]:
    """(decode service, prefill service) whose workers are packed into P/D group pods, or None.
    MXS_PD_POD_MODE=group (default; `pair` is accepted as its old name) renders the graph's decode
    and prefill replicas as pods that each hold several workers of both roles and all their GPUs
    (SURVEY.md §5.8 mitigation #1; mxserve/worker/pair.py); =split keeps the reference's two-pod
    form (then the KV crosses pods over hostIPC: the host's /dev/shm arena or HTTP)."""
    if os.environ.get("MXS_PD_POD_MODE", "group") not in ("group", "pair"):
        return None
    dec = [s for s in g.services if s.component_type == "worker" and s.sub_component_type == "decode"]
    pre = [s for s in g.services if s.component_type == "worker" and s.sub_component_type == "prefill"]
    if not dec or not pre or dec[0].replicas <= 0 or pre[0].replicas <= 0:
        return None
    return dec[0], pre[0]


def pd_groups(d: ServiceSpec, p: ServiceSpec, node_gpus: int = 0) -> list:
    """Pack P prefill and D decode workers (their own `gpu` limits each) into the fewest pods that
    fit one node's GPUs, spreading both roles evenly so every pod has decode workers and, where
    there are enough, prefill workers of its own.  Returns [(prefill workers, decode workers)] per
    pod: the reference's independent counts (examples/deploy/vllm/disagg.yaml:22,42) at any P:D
    ratio -- 3P+5D is one 8-GPU pod with exactly 3 prefill and 5 decode workers."""
    node = node_gpus or NODE_GPUS
    gp, gd = p.gpus or 1, d.gpus or 1
    P, D = p.replicas, d.replicas
    if gp > node or gd > node:
        raise ValidationError(f"a worker asks for more GPUs than a node has ({max(gp, gd)} > {node})")
    n = max(1, -(-(P * gp + D * gd) // node))
    while True:
        groups = [(P // n + (i < P % n), D // n + (i < D % n)) for i in range(n)]
        if all(pi * gp + di * gd <= node for pi, di in groups):
            break
        n += 1
    if D > 0 and n > D:
        # a pod without a decode worker would have a prefill worker on its readiness/system port and
        # no decode worker to hand its KV to inside the pod
        raise ValidationError(f"{P} prefill + {D} decode workers need {n} group pods of at most {node} GPUs, "
                              f"more pods than decode workers; use MXS_PD_POD_MODE=split for this layout")
    return [gr for gr in groups if gr != (0, 0)]


def group_shapes(groups: list) -> list:
    """[(prefill workers, decode workers, pod count)] per distinct group-pod shape, most pods first
    (the order of the shape Deployments: group_deployment_name)."""
    shapes: dict = {}
    for gr in groups:
        shapes[gr] = shapes.get(gr, 0) + 1
    return [(a, b, c) for (a, b), c in sorted(shapes.items(), key=lambda x: (-x[1], x[0]))]


def _full_command(g: GraphSpec, s: ServiceSpec) -> list:
    return [str(c) for c in (s.command or _default_command(g, s))] + [str(a) for a in (s.args or [])]


def _group_container(g: GraphSpec, d: ServiceSpec, p: ServiceSpec, n_pre: int, n_dec: int) -> dict:
    """One container running n_dec decode + n_pre prefill workers (mxserve/worker/pair.py assigns
    each its GPUs and port; decode workers first, so the pod's readiness port is a decode worker)."""
    c = _container(g, d)
    c["command"] = ["python3", "-m", "mxserve.worker.pair"]
    c.pop("args", None)
    have = {e["name"] for e in c["env"]}
    c["env"] += [dict(e) for e in p.envs if e["name"] not in have]
    spec = ([{"role": "decode", "cmd": _full_command(g, d), "gpus": d.gpus or 1}] * n_dec
            + [{"role": "prefill", "cmd": _full_command(g, p), "gpus": p.gpus or 1}] * n_pre)
    c["env"] += [{"name": "MXS_GROUP_SPEC", "value": json.dumps(spec)},
                 {"name": "POD_NAME", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}}]
    c["ports"] = [{"name": "system" if i == 0 else f"w{i}", "containerPort": WORKER_PORT + i}
                  for i in range(len(spec))]
    n = sum(w["gpus"] for w in spec)
    c["resources"] = {"limits": {GPU_RESOURCE: str(n)}, "requests": {GPU_RESOURCE: str(n)}}
    mounts = {m["mountPath"] for m in c.get("volumeMounts", [])}
    for vm in p.volume_mounts:
        if vm["mountPoint"] not in mounts:
            c.setdefault("volumeMounts", []).append({"name": vm["name"], "mountPath": vm["mountPoint"]})
    if not p.env_from_secret or p.env_from_secret == d.env_from_secret:
        return c
    c.setdefault("envFrom", []).append({"secretRef": {"name": p.env_from_secret, "optional": True}})
    return c


def group_deployment_name(name: str, k: int) -> str:
    """Deployment of the k-th (0-based) group-pod shape of a grouped decode service."""
    return name if k == 0 else f"{name}-g{k + 1}"


def _deployment(g: GraphSpec, name: str, labels: dict, owner: list, replicas: int, pod_spec: dict,
                extra_selector: Optional[dict] = None, dep_name: Optional[str] = None) -> dict:
    sel = {"app.kubernetes.io/name": name, **(extra_selector or {})}
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": dep_name or name,
                         "namespace": g.namespace, "labels": dict(labels, **(extra_selector or {})),
                         "ownerReferences": owner},
            "spec": {"replicas": replicas, "selector": {"matchLabels": sel},
                     "template": {"metadata": {"labels": dict(labels, **(extra_selector or {}))}, "spec": pod_spec}}}


def render_children(g: GraphSpec, dcd_uids: Optional[dict] = None) -> list[dict]:
    """Deployment + Service (+ PodMonitor) per service, owned by its DCD.  With P/D grouping the
    decode service's Deployment(s) run the group pods (pd_groups: one Deployment per distinct
    group shape) and the prefill service's Deployment keeps 0 replicas (every prefill worker runs
    inside a group pod)."""
    objs = []
    dcd_uids = dcd_uids or {}
    pair = pd_pairs(g)
    groups = pd_groups(pair[0], pair[1]) if pair is not None else []
    for s in g.services:
        name = f"{g.name}-{s.dns_name}"
        labels = {NS_LABEL: f"{g.namespace}-{g.name}", COMPONENT_LABEL: s.key, TYPE_LABEL: s.component_type,
                  "app.kubernetes.io/name": name, "app.kubernetes.io/managed-by": "mxserve-operator"}
        if s.sub_component_type:
            labels[SUBTYPE_LABEL] = s.sub_component_type
        owner = _owner(DCD_KIND, name, dcd_uids.get(name))
        grouped = pair is not None and s is pair[0]
        vms = list(s.volume_mounts) + (list(pair[1].volume_mounts) if grouped else [])
        vols = []
        for vm in vms:
            if vm["name"] not in {v["name"] for v in vols}:
                vols.append({"name": vm["name"], "persistentVolumeClaim": {"claimName": vm["name"]}})
        split_pd = pair is None and s.sub_component_type in ("prefill", "decode") and s.component_type == "worker"
        if (s.gpus or grouped) and not split_pd:
            # a pod-private /dev/shm for the TP ranks' metadata ring, RCCL and (group pods) the
            # workers' shared KV staging arena
            vols.append({"name": "dshm", "emptyDir": {"medium": "Memory"}})

        def pod(container: dict) -> dict:
            spec = {"containers": [container], "terminationGracePeriodSeconds": 30}
            if split_pd and s.gpus:
                # two-pod form: the xGMI KV transfer between prefill and decode pods opens the peer's
                # staging arena with hipIpcOpenMemHandle, and the /dev/shm arena must be the host's:
                # the pods share the host IPC namespace (SURVEY.md §5.8 mitigation #2) and mount no
                # private /dev/shm over it
                spec["hostIPC"] = True
                container.get("volumeMounts", [])[:] = [m for m in container.get("volumeMounts", [])
                                                        if m["name"] != "dshm"]
                if not container.get("volumeMounts"):
                    container.pop("volumeMounts", None)
            if vols:
                spec["volumes"] = [dict(v) for v in vols]
            return spec

        if grouped:
            labels[PAIR_LABEL] = f"{pair[0].key}+{pair[1].key}"
            for k, (n_pre, n_dec, count) in enumerate(group_shapes(groups)):
                # every shape Deployment selects on its own shape label (the first one too), so no
                # two Deployments' selectors overlap; the Service and PodMonitor select on the name
                c = _group_container(g, pair[0], pair[1], n_pre, n_dec)
                objs.append(_deployment(g, name, labels, owner, count, pod(c), {SHAPE_LABEL: f"g{k + 1}"},
                                        group_deployment_name(name, k)))
        else:
            replicas = 0 if (pair is not None and s is pair[1]) else s.replicas
            objs.append(_deployment(g, name, labels, owner, replicas, pod(_container(g, s))))
        is_fe = s.component_type == "frontend"
        svc_spec = {"selector": {"app.kubernetes.io/name": name},
                    "ports": [{"name": "http" if is_fe else "system", "port": FRONTEND_PORT if is_fe else WORKER_PORT,
                               "targetPort": FRONTEND_PORT if is_fe else WORKER_PORT}]}
        if not is_fe:
            svc_spec["clusterIP"] = "None"  # workers register themselves; deploy-incluster skips headless
        objs.append({"apiVersion": "v1", "kind": "Service",
                     "metadata": {"name": name, "namespace": g.namespace, "labels": dict(labels),
                                  "ownerReferences": owner},
                     "spec": svc_spec})
        endpoints = [{"port": "http" if is_fe else "system", "path": "/metrics", "interval": "15s"}]
        if grouped:  # every worker of a group pod serves its own /metrics
            n_max = max(a + b for a, b in groups)
            endpoints += [{"port": f"w{i}", "path": "/metrics", "interval": "15s"} for i in range(1, n_max)]
        objs.append({"apiVersion": "monitoring.coreos.com/v1", "kind": "PodMonitor",
                     "metadata": {"name": name, "namespace": g.namespace, "labels": dict(labels),
                                  "ownerReferences": owner},
                     "spec": {"selector": {"matchLabels": {"app.kubernetes.io/name": name}},
                              "podMetricsEndpoints": endpoints}})
    return objs


def graph_gpus(g: GraphSpec) -> int:
    """GPUs the rendered graph asks for (what has to fit the node)."""
    total = 0
    for o in render_children(g):
        if o["kind"] != "Deployment":
            continue
        c = o["spec"]["template"]["spec"]["containers"][0]
        total += o["spec"]["replicas"] * int((c.get("resources") or {}).get("limits", {}).get(GPU_RESOURCE, 0))
    return total


# --------------------------------------------------------------------------- DGDR
@dataclass
class RequestSpec:
    name: str
    namespace: str
    model: str
    backend: str
    config_map: Optional[str]
    config_key: Optional[str]
    isl: int
    osl: int
    ttft_ms: float
    itl_ms: float
    system: str
    workers_image: Optional[str]
    auto_apply: bool
    uid: Optional[str] = None
    profiler_image: Optional[str] = None
    measure: bool = False  # live profiling on a GPU (useAiConfigurator: false) vs the roofline model


def parse_dgdr(obj: dict, namespace: Optional[str] = None) -> RequestSpec:
    if obj.get("apiVersion") != API_VERSION or obj.get("kind") != DGDR_KIND:
        raise ValidationError(f"expected {API_VERSION} {DGDR_KIND}")
    meta = obj.get("metadata") or {}
    spec = obj.get("spec") or {}
    pc = spec.get("profilingConfig") or {}
    cfg = pc.get("config") or {}
    sla = cfg.get("sla") or {}
    sweep = cfg.get("sweep") or {}
    cm = pc.get("configMapRef") or {}
    if not spec.get("model"):
        raise ValidationError("spec.model is required")
    for k in ("isl", "osl", "ttft", "itl"):
        if k in sla and float(sla[k]) <= 0:
            raise ValidationError(f"sla.{k} must be positive")
    return RequestSpec(
        name=meta.get("name", "dgdr"), namespace=namespace or meta.get("namespace") or "default",
        model=spec["model"], backend=spec.get("backend", "vllm"), config_map=cm.get("name"), config_key=cm.get("key"),
        isl=int(sla.get("isl", 4000)), osl=int(sla.get("osl", 500)), ttft_ms=float(sla.get("ttft", 600)),
        itl_ms=float(sla.get("itl", 25)), system=str(sweep.get("aicSystem", "mi355x")),
        workers_image=(spec.get("deploymentOverrides") or {}).get("workersImage"),
        auto_apply=bool(spec.get("autoApply", False)), uid=meta.get("uid"),
        profiler_image=pc.get("profilerImage"),
        measure="useAiConfigurator" in sweep and not bool(sweep.get("useAiConfigurator")))


PROFILER_SA = "mxserve-profiler"


def render_profiler_job(r: RequestSpec, job: str, results_cm: str) -> list[dict]:
    """The DGDR profiling Job (reference: the Dynamo operator's profiling job from `profilerImage`,
    examples/dgdr/trtllm/dgdr.yaml:14-31) and the RBAC it needs to publish its results ConfigMap.
    A live (`measure`) run takes one GPU and times this engine; otherwise it runs the roofline."""
    owner = _owner(DGDR_KIND, r.name, r.uid)
    ns = r.namespace
    cmd = ["python3", "-m", "mxserve.profiler.sla", "--model", r.model, "--isl", str(r.isl), "--osl", str(r.osl),
           "--ttft", f"{r.ttft_ms:g}", "--itl", f"{r.itl_ms:g}", "--system", r.system,
           "--output-configmap", results_cm, "--namespace", ns]
    if r.measure:
        cmd.append("--measure")
    c = {"name": "profiler", "image": map_image(r.profiler_image)[0], "command": cmd,
         "env": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}]}
    if r.measure:
        c["resources"] = {"limits": {GPU_RESOURCE: "1"}, "requests": {GPU_RESOURCE: "1"}}
    labels = {"app.kubernetes.io/managed-by": "mxserve-operator", "mxserve.io/dgdr": r.name}
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": PROFILER_SA, "namespace": ns}},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
         "metadata": {"name": PROFILER_SA, "namespace": ns},
         "rules": [{"apiGroups": [""], "resources": ["configmaps"], "verbs": ["get", "create", "update", "patch"]}]},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
         "metadata": {"name": PROFILER_SA, "namespace": ns},
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": PROFILER_SA},
         "subjects": [{"kind": "ServiceAccount", "name": PROFILER_SA, "namespace": ns}]},
        {"apiVersion": "batch/v1", "kind": "Job",
         "metadata": {"name": job, "namespace": ns, "labels": labels, "ownerReferences": owner},
         "spec": {"backoffLimit": 1, "ttlSecondsAfterFinished": 3600,
                  "template": {"metadata": {"labels": labels},
                               "spec": {"restartPolicy": "Never", "serviceAccountName": PROFILER_SA,
                                        "containers": [c]}}}},
    ]


def apply_plan_to_template(template: dict, plan: dict, req: RequestSpec) -> dict:
    """Fill a DGD template (the DGDR's ConfigMap) with the profiler's plan: replica counts, TP
    degree (`gpu` limit + `--tp`), worker image override, model name."""
    dgd = copy.deepcopy(template)
    dgd.setdefault("metadata", {})["name"] = dgd["metadata"].get("name") or req.name
    dgd["metadata"]["namespace"] = req.namespace
    for key, s in (dgd.get("spec", {}).get("services") or {}).items():
        if s.get("componentType") != "worker":
            continue
        role = s.get("subComponentType") or "agg"
        p = plan.get(role) or plan.get("agg") or {}
        if "replicas" in p:
            s["replicas"] = int(p["replicas"])
        if "tp" in p:
            s.setdefault("resources", {}).setdefault("limits", {})["gpu"] = str(p["tp"])
            mc = s.setdefault("extraPodSpec", {}).setdefault("mainContainer", {})
            args = [str(a) for a in mc.get("args") or []]
            for flag in ("--tp", "--tensor-parallel-size", "--tp-size"):
                if flag in args:
                    args[args.index(flag) + 1] = str(p["tp"])
                    break
            else:
                args += ["--tensor-parallel-size", str(p["tp"])]
            mc["args"] = args
        if req.workers_image:
            s.setdefault("extraPodSpec", {}).setdefault("mainContainer", {})["image"] = req.workers_image
    return dgd
