"""Collector pause control (mxserve/utils/gcpause.py): the start-up heap is frozen, an engine torn
down after the freeze is still collectable, and PauseStats sees the collector's passes."""
import gc

from mxserve.utils import gcpause


class _Cycle:
    def __init__(self):
        self.me = self


def test_freeze_unfreeze_and_pause_stats(monkeypatch):
    monkeypatch.setenv("MXS_GC_FREEZE", "1")
    th = gc.get_threshold()
    try:
        c = _Cycle()
        gcpause.freeze_heap(gen0_threshold=5000)
        assert gc.get_freeze_count() > 0
        assert gc.get_threshold()[0] >= 5000
        # a frozen cycle is not collected until the heap is unfrozen
        import weakref
        ref = weakref.ref(c)
        del c
        gc.collect()
        assert ref() is not None
        gcpause.unfreeze_heap()
        assert gc.get_freeze_count() == 0
        gc.collect()
        assert ref() is None
        ps = gcpause.PauseStats().install()
        gc.collect()
        ps.remove()
        s = ps.summary()
        assert s["collections"][2] >= 1 and s["max_ms"][2] >= 0.0
    finally:
        gcpause.unfreeze_heap()
        gc.set_threshold(*th)


def test_freeze_disabled(monkeypatch):
    monkeypatch.setenv("MXS_GC_FREEZE", "0")
    assert gcpause.freeze_heap() is False
