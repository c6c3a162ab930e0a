"""roctx ranges of the C-ABI (csrc/rvz_trace.h; SURVEY §5 tracing): with RVZ_ROCTX=1 a
rocprofv3 --marker-trace run of eager self-play plies records the search / eval / act / env
ranges; without it, none."""
import csv
import glob
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ranges(tmp_path, env_on):
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        pytest.skip("rocprofv3 not installed")
    out = tmp_path / ("on" if env_on else "off")
    env = dict(os.environ, TMPDIR="/tmp")
    env.pop("RVZ_ROCTX", None)
    if env_on:
        env["RVZ_ROCTX"] = "1"
    cmd = [prof, "--marker-trace", "--output-format", "csv", "-d", str(out), "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "tools", "trace_plies.py"), "1", "256"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    names = set()
    for f in glob.glob(os.path.join(str(out), "**", "*marker_api_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            names.add(row["Function"])
    return names


def test_roctx_ranges_present_only_when_enabled(tmp_path):
    on = _ranges(tmp_path, True)
    for want in ("rvz.search.step (expand/backup + select)", "rvz.eval.trunk (k_resnet_h2)",
                 "rvz.eval.heads (k_heads_mfma)", "rvz.search.submit",
                 "rvz.act (expand/backup + action + move)", "rvz.env.autoreset"):
        assert want in on, (want, sorted(on))
    off = _ranges(tmp_path, False)
    assert not any(n.startswith("rvz.") for n in off), sorted(off)
