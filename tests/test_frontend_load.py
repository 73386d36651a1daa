"""Frontend under load without a GPU (scripts/frontend_load.py): synthetic
token-emitting workers behind the real multi-process frontend (httpd + push fast path), streamed
by open-loop clients.  Scaled to what a CPU test box runs next to its clients: the full node-size
point (125 k tok/s, 4 processes) is in profiles/r3/frontend_load_*.json."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_frontend_streams_without_drops_and_small_added_latency(tmp_path):
    out = tmp_path / "load.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "frontend_load.py"), "--tok-per-s", "30000",
                        "--workers", "2", "--procs", "2", "--clients", "2", "--duration", "10", "--out", str(out)],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["requests_dropped"] == 0 and d["requests_done"] > 0, d  # drop_reasons names any cause
    # rate and latency are CPU-bound here (frontend, fake workers and clients share this box): when
    # the box was saturated during the run (other tests under pytest -n 8) only looser bounds mean
    # anything (the rate then follows the CPU share this run got, and the fake workers' 10 ms step
    # cadence coalesces); zero drops is required either way
    starved = d["system_cpu_busy"] > 0.85
    if starved:  # progress only: latencies then measure the box's CPU share, not the serving path
        assert d["delivered_tok_per_s"] >= 0.25 * d["target_tok_per_s"], d
    else:
        assert d["delivered_tok_per_s"] >= 0.9 * d["target_tok_per_s"], d
        assert d["ttft_ms_p50"] < 50, d  # what the serving path adds to the first token
        assert 8.0 < d["chunk_gap_ms_p50"] < 14.0, d  # the workers' 10 ms step cadence
