"""DGDR live profiling (`python -m mxserve.profiler.sla --measure`) on the GPU: the engine's TTFT for
an ISL-token prompt and decode step times over a batch sweep, fed into the plan."""
import pytest

pytestmark = pytest.mark.gpu


def test_measure_qwen3_on_gpu(gpu):
    from mxserve.profiler import sla
    m = sla.measure("Qwen/Qwen3-0.6B", 4000, 500, batches=(1, 16, 64))
    assert 0 < m["ttft_ms"] < 600, m
    itl = [m["decode_itl_ms"][str(b)] for b in (1, 16, 64)]
    assert all(0 < t < 25 for t in itl) and itl[2] >= itl[0], m
    p = sla.plan("Qwen/Qwen3-0.6B", 4000, 500, 600, 25, measured=m)
    assert p["feasible"] and p["source"] == "measured"
