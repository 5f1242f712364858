"""Host sanitizer run (CPU, no GPU): tests/asan/Makefile builds the drop-in's
host layout code (sfm_amd/csrc/ba_host_layout.h, what sfm_ba_set_problem runs
on the host), the compat header's gather / scatter-back and the oracle under
AddressSanitizer + UBSan and runs them on the C1, shuffled-duplicate,
empty-camera, bad-index and empty scenes."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_and_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "asan"), "asan"], capture_output=True,
                       text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "asan: all checks passed" in out, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
