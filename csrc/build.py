#!/usr/bin/env python3
"""Build the native parts in-tree (no JIT cache, no hipify, no torch extension).

* ``libeia_kernels.so`` -- every ``csrc/kernels/*.hip`` compiled by hipcc for
  ``--offload-arch=gfx950`` only, exposing a plain C ABI (launchers take raw
  device pointers + a hipStream_t) that ``enterprise_inference_amd/_native.py``
  binds with ctypes.  The .so lands in ``enterprise_inference_amd/_lib`` so it
  travels with the repo snapshot to the GPU box.
* ``_eia_runtime.*.so`` -- host C++ runtime (KV block manager, batch builder,
  shm broadcast ring) as a pybind11 module, built with g++.

Usage: python csrc/build.py [--kernels] [--runtime] [--force] [-j N]
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "enterprise_inference_amd", "_lib")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("EIA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")

KERNELS_SO = os.path.join(OUT_DIR, "libeia_kernels.so")
RUNTIME_SO = os.path.join(OUT_DIR, "_eia_runtime" + sysconfig.get_config_var("EXT_SUFFIX"))

HIP_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
    "-munsafe-fp-atomics", "-fgpu-flush-denormals-to-zero",
    "-I" + os.path.join(CSRC, "include"),
    "-Wno-unused-result",
]


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _headers() -> list[str]:
    inc = os.path.join(CSRC, "include")
    return [os.path.join(inc, f) for f in os.listdir(inc)]


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def kernel_sources() -> list[str]:
    kd = os.path.join(CSRC, "kernels")
    return sorted(os.path.join(kd, f) for f in os.listdir(kd) if f.endswith(".hip"))


def build_kernels(force: bool = False, jobs: int = 8) -> str:
    if not HIPCC or not os.path.exists(HIPCC):
        raise RuntimeError("hipcc not found; ROCm toolchain required to build gfx950 kernels")
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = kernel_sources()
    hdrs = _headers()
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(OBJ_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if force or not _newer(o, [s] + hdrs):
            todo.append((s, o))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(_run, [HIPCC, *HIP_FLAGS, "-c", s, "-o", o]) for s, o in todo]
        for f in futs:
            f.result()
    # the link also re-runs when the source SET changed (a kernel file deleted or added):
    # the library must not keep symbols of sources that no longer exist
    manifest = os.path.join(OBJ_DIR, "kernels.manifest")
    want = "\n".join(os.path.basename(o) for o in objs)
    try:
        have = open(manifest).read()
    except OSError:
        have = None
    if force or todo or have != want or not _newer(KERNELS_SO, objs):
        tmp = KERNELS_SO + ".tmp"
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs])
        os.replace(tmp, KERNELS_SO)
        with open(manifest, "w") as f:
            f.write(want)
    return KERNELS_SO


def build_runtime(force: bool = False) -> str:
    import pybind11

    os.makedirs(OUT_DIR, exist_ok=True)
    rd = os.path.join(CSRC, "runtime")
    srcs = sorted(os.path.join(rd, f) for f in os.listdir(rd) if f.endswith(".cpp"))
    if not force and _newer(RUNTIME_SO, srcs):
        return RUNTIME_SO
    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    tmp = RUNTIME_SO + ".tmp"
    cmd = [cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
           "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
           *srcs, "-o", tmp, "-lrt", "-pthread"]
    if os.environ.get("EIA_SANITIZE"):
        cmd[1:1] = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"]
    _run(cmd)
    os.replace(tmp, RUNTIME_SO)
    return RUNTIME_SO


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", action="store_true")
    ap.add_argument("--runtime", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    both = not (a.kernels or a.runtime)
    if a.runtime or both:
        print("runtime ->", build_runtime(a.force))
    if a.kernels or both:
        print("kernels ->", build_kernels(a.force, a.j))
    return 0


if __name__ == "__main__":
    sys.exit(main())
