"""Persisted kernel choices (ops/tuned.py) and the robust pick of the decode GEMM tuner
(ops/decode_gemm.py pick): stored choices are reused verbatim, MXS_RETUNE ignores them, saving is
opt-in, and a candidate wins only on a clear median margin over hipBLASLt.  CPU only."""
import json

import pytest

from mxserve.ops import decode_gemm, tuned


def test_store_roundtrip(tmp_path, monkeypatch):
    monkeypatch.setenv("MXS_TUNED_DIR", str(tmp_path))
    monkeypatch.setenv("MXS_TUNED_SAVE", "1")
    st = tuned.TunedStore("decode_gemm", "gfxtest_256cu")
    assert st.get("3072x2048x0@256") is None and st.misses == 1
    st.put("3072x2048x0@256", {"cfg": ("mt", 4, 2, 1, 2, 4, 1), "us": 9.5, "hipblaslt_us": 13.0})
    st.put("2048x2048x0@256", {"cfg": None, "us": 10.1, "hipblaslt_us": 10.1})
    path = st.save()
    assert path == str(tmp_path / "decode_gemm_gfxtest_256cu.json")
    d = json.loads(open(path).read())
    assert d["device"] == "gfxtest_256cu" and len(d["entries"]) == 2
    st2 = tuned.TunedStore("decode_gemm", "gfxtest_256cu")
    e = st2.get("3072x2048x0@256")
    assert e["cfg"] == ("mt", 4, 2, 1, 2, 4, 1)  # tuple again: hashable, comparable with candidates()
    assert st2.get("2048x2048x0@256")["cfg"] is None and st2.hits == 2
    monkeypatch.setenv("MXS_RETUNE", "1")
    assert tuned.TunedStore("decode_gemm", "gfxtest_256cu").get("3072x2048x0@256") is None


def test_save_is_opt_in(tmp_path, monkeypatch):
    monkeypatch.setenv("MXS_TUNED_DIR", str(tmp_path))
    monkeypatch.delenv("MXS_TUNED_SAVE", raising=False)
    st = tuned.TunedStore("prefill_gemm", "gfxtest_256cu")
    st.put("k", {"cfg": None})
    assert st.save() is None and not list(tmp_path.iterdir())


def test_other_device_tag_does_not_match(tmp_path, monkeypatch):
    monkeypatch.setenv("MXS_TUNED_DIR", str(tmp_path))
    monkeypatch.setenv("MXS_TUNED_SAVE", "1")
    st = tuned.TunedStore("decode_gemm", "gfxtest_256cu")
    st.put("k", {"cfg": None})
    st.save()
    assert tuned.TunedStore("decode_gemm", "gfx942_304cu").get("k") is None


def test_packaged_tables_parse():
    import glob
    import os
    for p in glob.glob(os.path.join(tuned.PKG_DIR, "*.json")):
        d = json.loads(open(p).read())
        assert d["entries"], p
        if d.get("kind") == "prefill_mplan":  # {shape: {M bucket: plan}} (ops._mplan; tests/test_mplan.py)
            continue
        for k, v in d["entries"].items():
            if d.get("kind") == "prefill_hblt":  # a hipBLASLt solution index + its kernel name (ops/prefill_hblt.py)
                assert "@" in k and "sol" in v and (v["sol"] is None) == (v.get("kernel") is None), (p, k)
                continue
            assert "@" in k and "cfg" in v, (p, k)


@pytest.fixture
def fake_clock(monkeypatch):
    """_graph_time returns scripted times per function (noise drawn from a fixed sequence)."""
    calls = {}

    def fake(fn, iters=20):
        seq = fn.times
        i = calls.get(id(fn), 0)
        calls[id(fn)] = i + 1
        return seq[i % len(seq)]

    monkeypatch.setattr(decode_gemm, "_graph_time", fake)
    return calls


def _fn(*times):
    f = lambda i: None  # noqa: E731
    f.times = list(times)
    return f


def test_pick_needs_a_clear_median_win(fake_clock):
    lib = _fn(10.0)
    # screening flatters "a" (one fast outlier); its median is no better than the library's
    cands = {"a": _fn(7.0, 10.0, 10.2, 9.9), "b": _fn(9.0, 9.5, 9.4, 9.6), "c": _fn(12.0)}
    best, t, t_lib = decode_gemm.pick(lib, cands)
    assert best == "b" and t == pytest.approx(9.5) and t_lib == 10.0


def test_pick_keeps_library_within_margin(fake_clock):
    lib = _fn(10.0)
    cands = {"a": _fn(9.8, 9.8, 9.8, 9.8)}  # 2 % faster: below the 3 % margin
    best, t, t_lib = decode_gemm.pick(lib, cands)
    assert best is None and t == t_lib == 10.0


@pytest.mark.parametrize("cfgs,want", [
    ({512: None, 1024: None}, False),             # every bucket rejects the fused form: no folded copy
    ({512: None, 1024: [256, 16]}, True),         # tune_fused()'s list form keeps gemm_pf at one bucket
    ({512: 8, 1024: None}, True),                 # earlier rounds' int form
    ({512: None}, True),                          # a bucket not measured yet
    ({512: "addmm", 1024: None}, False),          # code-2 string choices are not gemm_pf
])
def test_folded_weight_needed_reads_every_cfg_form(tmp_path, monkeypatch, cfgs, want):
    """a stored [rows, min_iters] choice must count as 'gemm_pf kept' so the norm-folded
    weight the fused kernel needs is made at start-up."""
    from mxserve.ops import prefill_pf
    monkeypatch.setenv("MXS_TUNED_DIR", str(tmp_path))
    monkeypatch.setattr(tuned, "device_tag", lambda device=None: "gfxtest_256cu")
    monkeypatch.setattr(prefill_pf, "MODE", "auto")
    monkeypatch.setattr(tuned, "PKG_DIR", str(tmp_path / "none"))
    entries = {f"2048x2048:3@{m}": {"cfg": c, "us": 1.0, "base_us": 2.0} for m, c in cfgs.items()}
    (tmp_path / "prefill_pf_gfxtest_256cu.json").write_text(json.dumps({"device": "gfxtest_256cu",
                                                                        "entries": entries}))
    assert prefill_pf.buckets_for(1024) == [512, 1024]
    assert prefill_pf.folded_weight_needed(2048, 2048, 3, 1024, None) is want
