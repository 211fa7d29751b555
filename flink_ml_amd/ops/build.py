"""Builds the native libraries in-tree (no JIT cache, no hipify):

* ``flink_ml_amd/ops/_lib/libfmlx_kernels.so`` — every ``csrc/*.hip`` compiled by hipcc for
  gfx950 and linked into one shared object with a flat ``extern "C"`` launcher API.
* ``flink_ml_amd/ops/_lib/libfmlx_host.so`` — host-side C++ runtime pieces (``csrc/host/*.cpp``:
  murmur3/Java-compatible hashing, data cache, quantile sketches, ...), built with g++.

Staleness is decided by CONTENT, not mtimes: ``_lib/build_manifest.json`` records the sha256
of every source, header, compile flag set and compiler version an object was built from, and
which objects the last build compiled vs reused. ``FMLX_FORCE_BUILD=1`` (or ``--force``)
recompiles everything. At load time ``native`` compares the manifest's source digest with the
tree and refuses a library built from other sources (a stale binary shipped with the tree).

``--sanitize``: the host runtime rebuilt with ``-fsanitize=address,undefined`` into
``_lib/libfmlx_host_asan.so`` (the CPU test-suite runs the host paths against it, see
``tests/test_native_build.py``); GPU code is never built with sanitizers.

Usage: ``python -m flink_ml_amd.ops.build [--force] [--sanitize] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
import os
import shutil
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
OBJDIR = os.path.join(HERE, "_build")
KERNEL_LIB = os.path.join(LIBDIR, "libfmlx_kernels.so")
HOST_LIB = os.path.join(LIBDIR, "libfmlx_host.so")
HOST_ASAN_LIB = os.path.join(LIBDIR, "libfmlx_host_asan.so")
MANIFEST = os.path.join(LIBDIR, "build_manifest.json")
ARCH = os.environ.get("FMLX_OFFLOAD_ARCH", "gfx950")
SANITIZE_FLAGS = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g"]


def _sha(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _digest(parts) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(str(p).encode())
        h.update(b"\0")
    return h.hexdigest()


def kernel_sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip"))), sorted(glob.glob(os.path.join(CSRC, "*.h")))


def host_sources():
    return sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp"))), sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))


def source_digest(which: str) -> str:
    """sha256 over the (relative name, content hash) of every source of a library."""
    srcs, hdrs = kernel_sources() if which == "kernels" else host_sources()
    return _digest([(os.path.relpath(f, CSRC), _sha(f)) for f in srcs + hdrs])


def _load_manifest() -> dict:
    try:
        with open(MANIFEST) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _save_manifest(m: dict) -> None:
    tmp = MANIFEST + ".tmp"
    with open(tmp, "w") as f:
        json.dump(m, f, indent=1, sort_keys=True)
    os.replace(tmp, MANIFEST)


def _tool_version(tool: str) -> str:
    try:
        return subprocess.run([tool, "--version"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True).stdout.strip()
    except OSError:
        return "?"


def _force(force: bool) -> bool:
    return force or os.environ.get("FMLX_FORCE_BUILD", "0") == "1"


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
FILE_FLAGS = {"kmeans.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-Wno-inline-asm"],
              # the fused round's ticket atomics: no lane-0 result fix-up (keeps counted vmcnt waits)
              "glm.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"],
              "glm_sparse.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"],
              # MFMA accumulators in arch VGPRs: the AGPR form rotated the DCT's accumulators
              # through VGPRs every k step
              "dct.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    force = _force(force)
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(OBJDIR, exist_ok=True)
    srcs, headers = kernel_sources()
    hipcc = _hipcc()
    flags = ["--offload-arch=%s" % ARCH, "-O3", "-std=c++17", "-fPIC", "-mcode-object-version=5",
             "-Wno-unused-result", "-I", CSRC]
    man = _load_manifest()
    kman = man.get("kernels", {})
    old_objs = kman.get("objects", {})
    hdr_digest = _digest([_sha(h) for h in headers])
    ver = _tool_version(hipcc)
    objs, todo, keys = [], [], {}
    for s in srcs:
        name = os.path.basename(s)
        o = os.path.join(OBJDIR, name[:-4] + ".o")
        objs.append(o)
        key = _digest([_sha(s), hdr_digest, flags, FILE_FLAGS.get(name, []), ver])
        keys[name] = key
        if force or not os.path.exists(o) or old_objs.get(name) != key:
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
    digest = source_digest("kernels")
    relink = force or bool(todo) or not os.path.exists(KERNEL_LIB) or kman.get("source_digest") != digest
    if relink:
        _run([hipcc, "--offload-arch=%s" % ARCH, "-shared", "-fPIC", "-o", KERNEL_LIB] + objs)
    man = _load_manifest()
    man["kernels"] = {"objects": keys, "source_digest": digest, "arch": ARCH, "compiler": ver.splitlines()[0] if ver else "?",
                      "compiled": sorted(os.path.basename(s) for s, _ in todo),
                      "reused": sorted(n for n in keys if n not in {os.path.basename(s) for s, _ in todo}),
                      "linked": relink, "forced": force, "time": time.strftime("%Y-%m-%dT%H:%M:%S")}
    _save_manifest(man)
    return KERNEL_LIB


def build_host(force: bool = False, verbose: bool = False, sanitize: bool = False) -> str:
    force = _force(force)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs, hdrs = host_sources()
    if not srcs:
        return ""
    target = HOST_ASAN_LIB if sanitize else HOST_LIB
    section = "host_asan" if sanitize else "host"
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O1" if sanitize else "-O3", "-std=c++17", "-fPIC", "-shared", "-march=x86-64-v2"] + (
        SANITIZE_FLAGS if sanitize else [])
    digest = source_digest("host")
    key = _digest([digest, flags, _tool_version(cxx)])
    man = _load_manifest()
    if not force and os.path.exists(target) and man.get(section, {}).get("key") == key:
        man[section]["compiled"] = False
        _save_manifest(man)
        return target
    if verbose:
        print("[g++] host runtime%s (%d files)" % (" (ASan+UBSan)" if sanitize else "", len(srcs)), flush=True)
    _run([cxx] + flags + ["-o", target] + srcs + ["-lpthread"])
    man = _load_manifest()
    man[section] = {"key": key, "source_digest": digest, "compiled": True, "flags": flags,
                    "time": time.strftime("%Y-%m-%dT%H:%M:%S")}
    _save_manifest(man)
    return target


def build_all(force: bool = False, jobs: int = 8, verbose: bool = False):
    k = build_kernels(force=force, jobs=jobs, verbose=verbose)
    h = build_host(force=force, verbose=verbose)
    return k, h


def check_fresh(which: str) -> None:
    """Raises if the library ``which`` ("kernels" / "host") was built from other sources than the
    tree holds (sources present but digest differs), i.e. a stale prebuilt binary."""
    srcs, _ = kernel_sources() if which == "kernels" else host_sources()
    if not srcs or os.environ.get("FMLX_SKIP_FRESHNESS", "0") == "1":
        return
    rec = _load_manifest().get(which, {})
    if not rec:
        return  # library built by hand / older tree: nothing to compare against
    if rec.get("source_digest") != source_digest(which):
        raise RuntimeError("native %s library is stale: built from other sources than this tree "
                           "(run python -m flink_ml_amd.ops.build)" % which)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--sanitize", action="store_true", help="also build the ASan/UBSan host runtime")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args(argv)
    k, h = build_all(force=a.force, jobs=a.j, verbose=True)
    print("built:", k, h)
    if a.sanitize:
        print("built:", build_host(force=a.force, verbose=True, sanitize=True))


if __name__ == "__main__":
    sys.exit(main())
