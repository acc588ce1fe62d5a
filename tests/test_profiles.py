"""CPU: every committed round-6 profile summary is what scripts/prof_summary.py computes from
the committed raw files beside it (no field of a summary may come from a
file that a later stage overwrote).  A summary records its inputs in `source` (paths on the
GPU box); the test maps them onto the committed directory, re-runs the script and compares
every field."""
import glob
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUMMARIES = sorted(glob.glob(os.path.join(ROOT, "profiles", "r06_*", "summary_*.json")))


@pytest.mark.parametrize("path", SUMMARIES, ids=[os.path.relpath(p, ROOT) for p in SUMMARIES])
def test_summary_reproduces_from_committed_files(path, tmp_path):
    d = os.path.dirname(path)
    want = json.load(open(path))
    src = want["source"]
    name = os.path.basename(path)[len("summary_"):-len(".json")]
    args = [sys.executable, os.path.join(ROOT, "scripts", "prof_summary.py"), "--last", str(src["last"]),
            "--out", str(tmp_path / "s.json")]
    for opt, base in (("trace", "kernel_trace.csv"), ("fetch", "pmc_fetch.csv"), ("write", "pmc_write.csv")):
        if opt in src:
            local = os.path.join(d, "raw_" + name, base)
            assert os.path.exists(local), local
            args += ["--" + opt, local]
    if "bench" in src:
        local = os.path.join(d, os.path.basename(src["bench"]))
        assert os.path.basename(local) == "pbench_%s.json" % name, "the summary's bench line is the profile's own"
        args += ["--bench", local]
    subprocess.run(args, check=True, capture_output=True, cwd=ROOT)
    got = json.load(open(tmp_path / "s.json"))
    got.pop("source")
    want.pop("source")
    assert got == want
