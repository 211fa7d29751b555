"""Native build hygiene: content-hash manifest (what the last build compiled vs reused), refusal
of a library built from other sources, and the host C++ runtime under ASan + UBSan (SURVEY §5
"Race detection / sanitizers": sanitizers on host code; GPU code is never built with them)."""
import json
import os
import subprocess
import sys

import pytest

from flink_ml_amd.ops import build as b

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_manifest_records_sources_and_build_outcome():
    b.build_all()
    man = json.load(open(b.MANIFEST))
    k = man["kernels"]
    assert k["source_digest"] == b.source_digest("kernels")
    assert set(k["compiled"]) | set(k["reused"]) == {os.path.basename(s) for s in b.kernel_sources()[0]}
    assert man["host"]["source_digest"] == b.source_digest("host")
    b.check_fresh("kernels")
    b.check_fresh("host")


def test_stale_library_is_refused(monkeypatch):
    monkeypatch.setattr(b, "source_digest", lambda which: "0" * 64)
    with pytest.raises(RuntimeError, match="stale"):
        b.check_fresh("kernels")


def test_force_build_env(monkeypatch):
    monkeypatch.setenv("FMLX_FORCE_BUILD", "1")
    assert b._force(False)
    monkeypatch.setenv("FMLX_FORCE_BUILD", "0")
    assert not b._force(False)


def _asan_runtime():
    try:
        p = subprocess.run(["g++", "-print-file-name=libasan.so"], stdout=subprocess.PIPE, text=True)
    except OSError:
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_host_runtime_under_asan_ubsan():
    """The host paths (data cache spill/replay, GK sketches, NN-chain, Java-compatible string
    hashing, reservoir sampling) run their CPU tests against the ASan+UBSan build of the host
    runtime; any report fails the run (UBSan is non-recoverable, ASan aborts on error)."""
    asan = _asan_runtime()
    if asan is None:
        pytest.skip("no libasan")
    lib = b.build_host(sanitize=True)
    env = dict(os.environ, LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", FMLX_DEVICE="cpu",
               FMLX_HOST_LIB=lib, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:xdist", "-m", "not gpu",
           "tests/test_datacache.py", "tests/test_quantile_summary.py", "tests/test_agglomerative.py",
           "tests/test_feature_text.py", "tests/test_kmeans.py", "tests/test_feature_lsh.py"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    out = p.stdout
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert p.returncode == 0, out[-4000:]
    assert " passed" in out
