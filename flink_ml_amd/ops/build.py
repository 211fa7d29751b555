"""Builds the native libraries in-tree (no JIT cache, no hipify):

* ``flink_ml_amd/ops/_lib/libfmlx_kernels.so`` — every ``csrc/*.hip`` compiled by hipcc for
  gfx950 and linked into one shared object with a flat ``extern "C"`` launcher API.
* ``flink_ml_amd/ops/_lib/libfmlx_host.so`` — host-side C++ runtime pieces (``csrc/host/*.cpp``:
  murmur3/Java-compatible hashing, data cache, quantile sketches, ...), built with g++.

Usage: ``python -m flink_ml_amd.ops.build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
OBJDIR = os.path.join(HERE, "_build")
KERNEL_LIB = os.path.join(LIBDIR, "libfmlx_kernels.so")
HOST_LIB = os.path.join(LIBDIR, "libfmlx_host.so")
ARCH = os.environ.get("FMLX_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _run(cmd):
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        raise RuntimeError("command failed (%d): %s\n%s" % (p.returncode, " ".join(cmd), p.stdout))
    return p.stdout


# per-source compiler options. kmeans.hip: MFMA accumulators in arch VGPRs — its epilogue reads
# every accumulator with VALU ops each tile, and the AGPR form adds a v_accvgpr_read per value.
FILE_FLAGS = {"kmeans.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h")))
    hipcc = _hipcc()
    flags = ["--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-mcode-object-version=5",
             "-Wno-unused-result", "-I", CSRC]
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(OBJDIR, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or not _newer(o, [s] + headers + [__file__]):
            todo.append((s, o))

    def comp(so):
        s, o = so
        if verbose:
            print("[hipcc] %s" % os.path.basename(s), flush=True)
        _run([hipcc] + flags + FILE_FLAGS.get(os.path.basename(s), []) + ["-c", s, "-o", o])
        return o

    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(comp, todo))
    if force or todo or not _newer(KERNEL_LIB, objs):
        _run([hipcc, "--offload-arch=%s" % ARCH, "-shared", "-fPIC", "-o", KERNEL_LIB] + objs)
    return KERNEL_LIB


def build_host(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))
    if not srcs:
        return ""
    if not force and _newer(HOST_LIB, srcs + hdrs):
        return HOST_LIB
    cxx = os.environ.get("CXX", "g++")
    if verbose:
        print("[g++] host runtime (%d files)" % len(srcs), flush=True)
    _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-march=x86-64-v2", "-o", HOST_LIB] + srcs + ["-lpthread"])
    return HOST_LIB


def build_all(force: bool = False, jobs: int = 8, verbose: bool = False):
    k = build_kernels(force=force, jobs=jobs, verbose=verbose)
    h = build_host(force=force, verbose=verbose)
    return k, h


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args(argv)
    k, h = build_all(force=a.force, jobs=a.j, verbose=True)
    print("built:", k, h)


if __name__ == "__main__":
    sys.exit(main())
