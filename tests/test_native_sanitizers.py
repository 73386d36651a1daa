"""Host-side native code under AddressSanitizer + UndefinedBehaviorSanitizer.
GPU sanitizers are not available on the test pool; the block pool / hashing / indexer core that the
Python bindings wrap is built standalone with -fsanitize=address,undefined and stress-tested against
shadow models (csrc/runtime/test_kv_runtime.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_kv_runtime_asan_ubsan(tmp_path):
    exe = tmp_path / "kv_runtime_asan"
    src = os.path.join(ROOT, "csrc", "runtime", "test_kv_runtime.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "csrc", "runtime"), src, "-o", str(exe)],
                   check=True, capture_output=True, text=True)
    # verify_asan_link_order=0: the environment may preload its own library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
