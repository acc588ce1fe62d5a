"""Host AddressSanitizer + UBSan run of the native host code: the packer,
the generator, the runtime's host paths (device = -1), the C oracle (incl. its OpenMP
pass) and the shim harness, through the CPU tests of scripts/asan_check.sh."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_clean_under_asan_ubsan():
    if not os.path.exists(os.path.join(ROOT, "build", "csrc", "esc_kernels.o")):
        pytest.skip("device object not built here (run __graft_entry__.build() first)")
    env = {k: v for k, v in os.environ.items() if not k.startswith(("ESC_", "LD_PRELOAD", "ASAN", "UBSAN"))}
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "asan_check.sh")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "asan/ubsan: clean" in r.stdout
