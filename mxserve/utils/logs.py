"""Process logging setup shared by the frontend, workers, operator and planner.

MXS_LOG_LEVEL sets the level (default INFO).  MXS_LOG_JSON=1 switches to one JSON object per line
(ts, level, logger, msg, plus request_id / worker when a record carries them) for log shippers.
"""
from __future__ import annotations

import json
import logging
import os
import time


class JsonFormatter(logging.Formatter):
    def format(self, r: logging.LogRecord) -> str:
        d = {"ts": round(r.created, 3), "time": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(r.created)),
             "level": r.levelname, "logger": r.name, "msg": r.getMessage()}
        for k in ("request_id", "worker", "model"):
            v = getattr(r, k, None)
            if v is not None:
                d[k] = v
        if r.exc_info:
            d["exc"] = self.formatException(r.exc_info)
        return json.dumps(d)


def setup_logging(default_level: str = "INFO") -> None:
    level = os.environ.get("MXS_LOG_LEVEL", default_level)
    h = logging.StreamHandler()
    if os.environ.get("MXS_LOG_JSON", "0") == "1":
        h.setFormatter(JsonFormatter())
    else:
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root = logging.getLogger()
    root.handlers[:] = [h]
    root.setLevel(level)
