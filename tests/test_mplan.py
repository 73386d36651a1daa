"""Prefill M plans (ops._mplan / ops._run_mplan): bucket lookup, the remainder shrink, and that a split
GEMM equals one F.linear (CPU tensors; the GPU path runs the same torch calls)."""
import torch

from mxserve import ops


def test_run_mplan_matches_linear():
    x = torch.randn(300, 64)
    w = torch.randn(96, 64)
    want = torch.nn.functional.linear(x, w)
    for plan in ([[44, "mm"], [256, "lin"]], [[300, "mm"]], [[100, "lin"], [200, "mm"]]):
        got = ops._run_mplan(x, w, plan)
        assert torch.allclose(got, want, atol=1e-5), plan


def test_mplan_lookup_and_shrink(monkeypatch):
    dev = torch.device("cpu")
    ops._MPLAN[dev] = {"16384x2048": {"4352": {"plan": [[256, "mm"], [4096, "lin"]]}}}
    try:
        assert ops._mplan(4352, 16384, 2048, dev) == [[256, "mm"], [4096, "lin"]]
        assert ops._mplan(4270, 16384, 2048, dev) == [[174, "mm"], [4096, "lin"]]
        assert ops._mplan(4100, 16384, 2048, dev) is None  # bucket 4224: no plan stored
        assert ops._mplan(4352, 3072, 2048, dev) is None
        monkeypatch.setenv("MXS_MPLAN", "0")
        assert ops._mplan(4352, 16384, 2048, dev) is None
    finally:
        ops._MPLAN.pop(dev, None)


def test_packaged_plan_table_parses():
    import json
    import os
    p = os.path.join(os.path.dirname(ops.__file__), "tuned", "prefill_mplan_gfx950_256cu.json")
    d = json.load(open(p))
    for k, ent in d["entries"].items():
        for m, e in ent.items():
            assert sum(r for r, _ in e["plan"]) == int(m)
            assert all(f in ("lin", "mm") for _, f in e["plan"])
