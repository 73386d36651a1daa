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
        assert ops._mplan(4100, 16384, 2048, dev) == [[4, "mm"], [4096, "lin"]]  # 128-row bucket 4224 absent: 256-row 4352
        assert ops._mplan(3900, 16384, 2048, dev) is None  # no bucket within reach
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


def test_plans_from_times_prefers_split_around_a_cliff():
    from mxserve.ops import mplan
    # F.linear: smooth except a cliff at 512 rows; mm(out=) as F.linear
    t = {128: (10.0, 10.0), 256: (12.0, 12.0), 384: (14.0, 14.0), 512: (40.0, 40.0)}
    p = mplan.plans_from_times(t, N=1024)
    assert "512" in p and sorted(r for r, _ in p["512"]["plan"]) in ([128, 384], [256, 256])
    assert "256" not in p  # no cliff: one F.linear
    # a faster call form alone
    p2 = mplan.plans_from_times({128: (10.0, 5.0), 256: (12.0, 12.0)}, N=64)
    assert p2["128"]["plan"] == [[128, "mm"]]


def test_mplan_coarse_grid_lookup():
    dev = torch.device("cpu")
    ops._MPLAN[dev] = {"4096x14336": {"4352": {"plan": [[256, "mm"], [4096, "mm"]]}}}
    try:
        assert ops._mplan(4200, 4096, 14336, dev) == [[104, "mm"], [4096, "mm"]]  # 256-row bucket 4352
        assert ops._mplan(4100, 4096, 14336, dev) == [[4, "mm"], [4096, "mm"]]
    finally:
        ops._MPLAN.pop(dev, None)


def test_mplan_lookup_stays_on_the_entry_grid():
    """a shape swept on the 128-row grid is looked up on that grid only -- a missing
    128-row bucket means 'no plan' (F.linear was best there), not the next 256-row bucket's plan
    stretched over up to 255 shaved rows; a start-up table swept every 256 rows uses its own grid."""
    dev = torch.device("cpu")
    ops._MPLAN[dev] = {
        "16384x2048": {"128": {"plan": [[128, "lin"]]}, "384": {"plan": [[128, "mm"], [256, "lin"]]},
                       "512": {"plan": [[256, "mm"], [256, "lin"]]}},
        "2048x8192": {"256": {"plan": [[256, "lin"]]}, "512": {"plan": [[256, "mm"], [256, "lin"]]}}}
    try:
        assert ops._mplan(300, 16384, 2048, dev) == [[44, "mm"], [256, "lin"]]  # 128-grid bucket 384
        assert ops._mplan(200, 16384, 2048, dev) is None  # 128-grid bucket 256 absent: no plan
        assert ops._mplan(300, 2048, 8192, dev) == [[44, "mm"], [256, "lin"]]  # 256-grid bucket 512
    finally:
        ops._MPLAN.pop(dev, None)
