"""served_phase._trace_breakdown (the served block's TTFT breakdown) against a stand-in frontend that
serves /debug/traces: steady-window filter, medians per stage, request count."""
import json
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

from mxserve.tools.served_phase import _trace_breakdown


def _serve(traces: list):
    class H(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            body = json.dumps({"traces": traces}).encode()
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass
    srv = HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv


def test_breakdown_medians_inside_the_window():
    traces = []
    for i in range(9):
        traces.append({"request_id": f"r{i}", "t_unix": 100.0 + i,
                       "spans_ms": {"received": 0.0, "tokenized": 0.1, "dispatched": 0.3, "submitted": 1.0 + i,
                                    "first_token": 40.0 + i, "done": 900.0},
                       "worker_ms": {"inbox_ms": 4.0, "queue_ms": float(i), "prefill_ms": 25.0, "delivery_ms": 2.0}})
    traces.append({"request_id": "ramp", "t_unix": 50.0, "spans_ms": {"first_token": 5.0}})  # outside the window
    srv = _serve(traces)
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}"
        out = _trace_breakdown(url, polls=3, window=(99.5, 110.0))
        assert out["requests"] == 9
        assert out["frontend_first_token"] == 44.0 and out["frontend_submitted"] == 5.0
        assert out["worker_queue"] == 4.0 and out["worker_prefill"] == 25.0 and out["worker_delivery"] == 2.0
        assert "frontend_done" not in out and "frontend_received" not in out
        assert _trace_breakdown(url, polls=1)["requests"] == 10  # no window: every trace
    finally:
        srv.shutdown()


def test_breakdown_of_an_unreachable_frontend_is_empty():
    assert _trace_breakdown("http://127.0.0.1:9", polls=2) == {}
