"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer.

Builds oracle/librvz_oracle_san.so (oracle/Makefile, host-only sanitizers) and re-runs the
oracle's fixture tests — every board vector and every recorded reference game replayed through
the literal search — in a child interpreter with the ASan runtime preloaded and the oracle
loader pointed at the sanitized build (RVZ_ORACLE_LIB). Any out-of-bounds access, use after
free, signed overflow or undefined shift in the oracle aborts the child. CPU only.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


def _runtime(name):
    out = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True)
    path = out.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_oracle_fixtures_clean_under_asan_ubsan():
    asan = _runtime("libasan.so")
    if asan is None:
        pytest.skip("no libasan runtime for gcc")
    subprocess.run(["make", "-s", "-C", ORACLE, "librvz_oracle_san.so"], check=True)
    san = os.path.join(ORACLE, "librvz_oracle_san.so")
    env = dict(os.environ)
    # the ASan runtime must come first in the preload list; keep whatever else is preloaded
    env["LD_PRELOAD"] = ":".join(p for p in (asan, os.environ.get("LD_PRELOAD", "")) if p)
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"   # CPython's own allocations leak
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["RVZ_ORACLE_LIB"] = san
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
           os.path.join(ROOT, "tests", "test_oracle_board.py"),
           os.path.join(ROOT, "tests", "test_oracle_search.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    log = r.stdout[-3000:] + r.stderr[-3000:]
    assert r.returncode == 0, log
    assert "passed" in r.stdout and "runtime error" not in r.stderr, log
    assert "AddressSanitizer" not in r.stderr, log
