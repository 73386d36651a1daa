"""prefill_hblt routing table (mxserve/ops/prefill_hblt.py) on the CPU: bucket lookup, decode-size
rows never routed, MODE gating, and the packaged table's entries name a kernel for every solution."""
import json
import os

from mxserve.ops import prefill_hblt


def test_lookup_takes_the_smallest_bucket_at_or_above(monkeypatch):
    t = prefill_hblt.HbltTable()
    t.entries[(2048, 2048, True)] = [(512, 11), (1024, None), (6592, 33)]
    monkeypatch.setattr(prefill_hblt, "MODE", "auto")
    assert t.lookup(300, 2048, 2048, True) == 11
    assert t.lookup(512, 2048, 2048, True) == 11
    assert t.lookup(513, 2048, 2048, True) is None  # bucket 1024 kept torch's call
    assert t.lookup(6000, 2048, 2048, True) == 33
    assert t.lookup(9000, 2048, 2048, True) == 33  # past the last bucket: the last
    assert t.lookup(256, 2048, 2048, True) is None  # decode-size rows: never
    assert t.lookup(600, 2048, 2048, False) is None  # the plain form has no entry
    monkeypatch.setattr(prefill_hblt, "MODE", "off")
    assert t.lookup(6000, 2048, 2048, True) is None
    monkeypatch.setattr(prefill_hblt, "MODE", "tune")
    assert t.lookup(6000, 2048, 2048, True) == 33


def test_tune_is_a_no_op_when_off(monkeypatch):
    monkeypatch.setattr(prefill_hblt, "MODE", "off")
    assert prefill_hblt.tune({}, set(), 6592, "cpu") == []


def test_packaged_table_entries():
    from mxserve.ops import tuned
    p = os.path.join(tuned.PKG_DIR, "prefill_hblt_gfx950_256cu.json")
    d = json.load(open(p))
    assert d["kind"] == "prefill_hblt" and d["entries"]
    for k, v in d["entries"].items():
        shape, m = k.split("@")
        n, rest = shape.split("x")
        kk, form = rest.split(":")
        assert int(n) % 256 == 0 and int(kk) % 64 == 0 and form in ("0", "1") and int(m) > 256, k
        assert (v["sol"] is None) == (v["kernel"] is None), k
        assert v["sol"] is None or v["us"] < v["base_us"], k  # kept only where it won
