"""Loader for the in-tree native host runtime (mxserve/_rt*.so).  Builds it on first use when a
compiler is available (CPU-only container), otherwise fails loudly."""
from __future__ import annotations

import importlib
import threading

_lock = threading.Lock()
_RT = None


def rt():
    global _RT
    if _RT is not None:
        return _RT
    with _lock:
        if _RT is None:
            try:
                _RT = importlib.import_module("mxserve._rt")
            except ImportError:
                import os
                import sys
                root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
                sys.path.insert(0, root)
                import setup_ext  # noqa: E402
                setup_ext.build_rt()
                _RT = importlib.import_module("mxserve._rt")
    return _RT
