"""SLA planner (X13) against the fake apiserver with a scripted metrics source and clock."""
import pytest

from mxserve.k8s.client import KubeClient
from mxserve.k8s.fake_apiserver import FakeApiServer
from mxserve.planner.planner import Planner, PlannerConfig, parse_prometheus
from tests.serving_utils import Server


def _dgd(kind="disagg"):
    svc = {"Frontend": {"componentType": "frontend", "replicas": 1}}
    if kind == "disagg":
        for sub in ("prefill", "decode"):
            svc[f"W{sub}"] = {"componentType": "worker", "subComponentType": sub, "replicas": 1,
                              "resources": {"limits": {"gpu": "1"}}}
    else:
        svc["W"] = {"componentType": "worker", "replicas": 1, "resources": {"limits": {"gpu": "1"}}}
    return {"apiVersion": "nvidia.com/v1alpha1", "kind": "DynamoGraphDeployment",
            "metadata": {"name": "g", "namespace": "ns"}, "spec": {"services": svc}}


class Feed:
    """Cumulative frontend counters advanced by (rps, isl, osl, ttft_s, itl_s) per window."""

    def __init__(self):
        self.c = {}
        self.t = 0.0

    def advance(self, secs, rps, isl=4000, osl=500, ttft=0.1, itl=0.01):
        n = rps * secs
        for k, v in (("dynamo_frontend_requests_total", n), ("dynamo_frontend_input_sequence_tokens_count", n),
                     ("dynamo_frontend_input_sequence_tokens_sum", n * isl),
                     ("dynamo_frontend_output_sequence_tokens_count", n),
                     ("dynamo_frontend_output_sequence_tokens_sum", n * osl),
                     ("dynamo_frontend_time_to_first_token_seconds_count", n),
                     ("dynamo_frontend_time_to_first_token_seconds_sum", n * ttft),
                     ("dynamo_frontend_inter_token_latency_seconds_count", n * osl),
                     ("dynamo_frontend_inter_token_latency_seconds_sum", n * osl * itl)):
            self.c[k] = self.c.get(k, 0.0) + v
        self.t += secs


@pytest.fixture()
def api():
    fake = FakeApiServer()
    srv = Server(fake.app).start()
    yield KubeClient(srv.url)
    srv.stop()


def test_parse_prometheus_sums_label_sets():
    text = ('# HELP x\n# TYPE x counter\ndynamo_frontend_requests_total{model="a",status="success"} 3.0\n'
            'dynamo_frontend_requests_total{model="a",status="error"} 1\nfoo 2.5e1\n')
    m = parse_prometheus(text)
    assert m["dynamo_frontend_requests_total"] == 4.0 and m["foo"] == 25.0


def test_planner_scales_up_on_load_and_sla_breach_then_down_after_cooldown(api):
    api.create(_dgd())
    feed = Feed()
    cfg = PlannerConfig(namespace="ns", dgd="g", model="meta-llama/Llama-3.2-1B-Instruct", cooldown_s=100,
                        max_gpus=8)
    p = Planner(cfg, api, lambda: dict(feed.c), clock=lambda: feed.t)
    assert p.step() is None  # first scrape only sets the baseline
    feed.advance(30, rps=60, ttft=0.9, itl=0.03)  # heavy load, both SLAs broken
    rec = p.step()
    svc = api.get("DynamoGraphDeployment", "g", "ns")["spec"]["services"]
    pre, dec = svc["Wprefill"]["replicas"], svc["Wdecode"]["replicas"]
    assert pre >= 2 and dec >= 2 and pre + dec <= 8, rec
    feed.advance(30, rps=0.2)  # idle, inside the cooldown: hold
    p.step()
    svc = api.get("DynamoGraphDeployment", "g", "ns")["spec"]["services"]
    assert (svc["Wprefill"]["replicas"], svc["Wdecode"]["replicas"]) == (pre, dec)
    for _ in range(5):  # past the cooldown: back to one replica each
        feed.advance(30, rps=0.2)
        p.step()
    svc = api.get("DynamoGraphDeployment", "g", "ns")["spec"]["services"]
    assert (svc["Wprefill"]["replicas"], svc["Wdecode"]["replicas"]) == (1, 1)


def test_planner_agg_graph_and_dry_run(api):
    api.create(_dgd("agg"))
    feed = Feed()
    cfg = PlannerConfig(namespace="ns", dgd="g", model="meta-llama/Llama-3.2-1B-Instruct", dry_run=True)
    p = Planner(cfg, api, lambda: dict(feed.c), clock=lambda: feed.t)
    p.step()
    feed.advance(30, rps=1000)
    rec = p.step()
    assert rec["changes"]["W"] == 8  # capped by the node's GPUs
    assert api.get("DynamoGraphDeployment", "g", "ns")["spec"]["services"]["W"]["replicas"] == 1  # dry run


def test_sla_plan_from_measurements():
    """--measure results replace the roofline: the measured TTFT and ITL(batch) curve decide the
    plan; a slower measured decode yields a smaller batch at the same ITL target."""
    from mxserve.profiler import sla
    fast = {"ttft_ms": 60.0, "decode_itl_ms": {"1": 2.0, "64": 4.0, "256": 10.0}}
    slow = {"ttft_ms": 60.0, "decode_itl_ms": {"1": 2.0, "64": 8.0, "256": 30.0}}
    pf = sla.plan("Qwen/Qwen3-0.6B", 4000, 500, 600, 25, measured=fast)
    ps = sla.plan("Qwen/Qwen3-0.6B", 4000, 500, 600, 25, measured=slow)
    assert pf["source"] == "measured" and pf["measurements"] == fast and pf["feasible"]
    assert pf["agg"]["ttft_ms"] == 60.0 and pf["disagg"]["prefill"]["ttft_ms"] == 60.0
    assert ps["agg"]["batch"] < pf["agg"]["batch"]
    m = sla.Measured(slow)
    assert m.itl(64) == 8.0 / 1e3 and abs(m.itl(160) - 19e-3) < 1e-9 and m.itl(512) > m.itl(256)
    # a TTFT target below the measured prefill split over 8 GPUs is infeasible
    assert not sla.plan("Qwen/Qwen3-0.6B", 4000, 500, 5, 25, measured=fast)["feasible"]


def test_one_capacity_model_for_bench_profiler_and_planner():
    """bench.py's disagg split, the DGDR profiler and the SLA planner read one
    capacity model (profiler/capacity.py): the headline workload splits 3P+5D on 8 GPUs in both
    planners, neither role is planned above 85 %, and the reference DGDR example fits one node."""
    import argparse

    import bench
    from mxserve.profiler import capacity, sla
    model = "meta-llama/Llama-3.2-1B-Instruct"
    cap = capacity.capacity(model, 4000, 500)
    assert cap["prefill_rps"] > 0 and cap["decode_rps"] > 0
    p, d, rate = capacity.pd_split(8, cap["prefill_rps"], cap["decode_rps"])
    ns = argparse.Namespace(model=model, isl=4000, osl=500, qps=-1.0, disagg_qps=-1.0, disagg_prefill_ranks=0)
    bp, bd, bq = bench.disagg_plan(ns, 8)
    plan = sla.plan(model, 4000, 500, 600, 25)
    assert (bp, bd) == (p, d) == (plan["disagg"]["prefill"]["replicas"], plan["disagg"]["decode"]["replicas"])
    assert plan["disagg"]["prefill"]["tp"] == plan["disagg"]["decode"]["tp"] == 1
    # the planned node rate loads the tighter role to 85 %, in both
    assert abs(bq * 8 - rate) < 1e-6
    assert bq * 8 <= 0.85 * min(bp * cap["prefill_rps"], bd * cap["decode_rps"]) + 1e-6
    # the SLA planner prices a TP-1 replica with the same per-GPU capacities
    from mxserve.planner.planner import Planner, PlannerConfig
    pl = Planner.__new__(Planner)
    pl.cfg = PlannerConfig(namespace="n", dgd="g", model=model)
    pl.model, pl.sys = sla.get_model_config(model), sla.SYSTEMS["mi355x"]
    assert abs(pl.capacity("prefill", 1, 4000, 500) - cap["prefill_rps"]) < 1e-6
    assert abs(pl.capacity("decode", 1, 4000, 500) - cap["decode_rps"]) < 1e-6
    # the reference DGDR example (Qwen3-0.6B, 8 GPUs) plans within the node
    q = sla.plan("Qwen/Qwen3-0.6B", 4000, 500, 600, 25)
    assert q["feasible"] and q["disagg"]["gpus_used"] <= 8


def test_measured_decode_capacity_respects_a_tighter_itl():
    """the measured decode capacity was taken at a 25 ms ITL target; a tighter target must
    not be planned with it (fewer rows fit per step), a looser one keeps the measurement."""
    from mxserve.profiler import capacity
    model = "meta-llama/Llama-3.2-1B-Instruct"
    e = capacity.lookup(model, 4000, 500)
    assert e is not None and e["decode_itl_target_ms"] == 25.0
    base = capacity.capacity(model, 4000, 500, 25.0)
    assert base["decode_rps"] == e["decode_rps"]
    assert capacity.capacity(model, 4000, 500, 40.0)["decode_rps"] == e["decode_rps"]
    tight = capacity.capacity(model, 4000, 500, 8.0)
    assert tight["decode_rps"] < e["decode_rps"] and "roofline ratio" in tight["decode_source"]
    assert tight["prefill_rps"] == e["prefill_rps"]
