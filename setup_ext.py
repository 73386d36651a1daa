#!/usr/bin/env python3
"""Build the native extensions in-tree (no JIT cache, no pip install):

  mxserve/_rt.so  host runtime (block pool, hashing, KV indexer)          g++ + pybind11
  mxserve/_C.so   gfx950 HIP kernels + KV-transfer agent, torch bindings   hipcc --offload-arch=gfx950

Incremental (mtime-based) and parallel.  `python setup_ext.py [--clean] [-j N] [--only rt|C]`.
HIP sources are written for CDNA4 directly: hipcc compiles them as-is, nothing is hipified.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shlex
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
# MXS_DEBUG_KERNELS=1: bounds-checked kernels (MXS_KCHECK, csrc/kernels/common.h), separate objects
DEBUG_KERNELS = os.environ.get("MXS_DEBUG_KERNELS", "0") == "1"
BUILD = os.path.join(ROOT, "build", "obj-debug" if DEBUG_KERNELS else "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_includes() -> list[str]:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce
    inc = [f"-I{p}" for p in ce.include_paths(device_type="cuda")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = ["-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
            "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1"]
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    libs = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            "-lc10_hip", "-ltorch_hip"]
    # hipBLASLt: the copy torch loads (one library, one set of solutions in the process)
    hblt = os.path.join(libdir, "libhipblaslt.so")
    libs.append(hblt if os.path.exists(hblt) else "-lhipblaslt")
    return inc, defs, libs


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    print("  " + " ".join(shlex.quote(c) for c in cmd[:6]) + (" ..." if len(cmd) > 6 else ""), flush=True)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[0]} ... {cmd[-1]}")


def build_rt(force: bool = False) -> str:
    out = os.path.join(ROOT, "mxserve", "_rt" + _ext_suffix())
    rdir = os.path.join(ROOT, "csrc", "runtime")
    srcs = sorted(p for p in glob.glob(os.path.join(rdir, "*.cpp")) if not os.path.basename(p).startswith("test_"))
    if force or _stale(out, srcs + glob.glob(os.path.join(rdir, "*.h"))):
        _run(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", *_pybind_includes(),
              *srcs, "-o", out])
    return out


def build_C(force: bool = False, jobs: int = 8) -> str:
    out = os.path.join(ROOT, "mxserve", "_C" + _ext_suffix())
    kdir = os.path.join(ROOT, "csrc", "kernels")
    headers = glob.glob(os.path.join(kdir, "*.h"))
    hip_srcs = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(kdir, "*.cpp")))
    os.makedirs(BUILD, exist_ok=True)
    inc, defs, libs = _torch_flags()
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *headers]):
            jobs_list.append([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
                              "-munsafe-fp-atomics", *(["-DMXS_DEBUG_KERNELS"] if DEBUG_KERNELS else []),
                              "-c", src, "-o", obj])
    for src in cpp_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, *headers]):
            jobs_list.append(["g++", "-O2", "-std=c++17", "-fPIC", f"-I{ROCM}/include", *inc, *defs,
                              *_pybind_includes(), "-c", src, "-o", obj])
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(_run, jobs_list))
    if force or jobs_list or _stale(out, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out, *libs,
              f"-L{ROCM}/lib", "-lamdhip64"])
    return out


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--only", choices=["rt", "C"], default=None)
    a = ap.parse_args(argv)
    if a.only in (None, "rt"):
        print("[mxserve] building host runtime _rt", flush=True)
        build_rt(a.clean)
    if a.only in (None, "C"):
        print(f"[mxserve] building HIP kernels _C for {ARCH}", flush=True)
        build_C(a.clean, a.j)
    print("[mxserve] build ok", flush=True)


if __name__ == "__main__":
    main()
