import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)
# the age-index build compares the device's membership counts with the host's on every build
os.environ.setdefault("ESC_CHECK_INDEX", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def golden():
    import json
    out = {}
    gdir = os.path.join(ROOT, "tests", "golden")
    for f in sorted(os.listdir(gdir)):
        if f.endswith(".json"):
            with open(os.path.join(gdir, f)) as fh:
                out[f[:-5]] = json.load(fh)
    return out
