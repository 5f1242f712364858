"""include/sfm_ctracker_compat.hpp: the C++ drop-in for CTracker's hot-path
signatures compiles against the C ABI, deduplicates the reference's
pointer-identified point blocks in first-seen order, and leaves the caller's
parameters untouched on an ABI error (no GPU here)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sfm_amd", "libsfm_amd.so")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_compat_header_packs_and_errors(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("libsfm_amd.so not built")
    exe = tmp_path / "compat_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "compat", "compat_check.cpp"), "-L", os.path.dirname(LIB),
                    "-lsfm_amd", "-Wl,-rpath," + os.path.dirname(LIB), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "compat ok" in out.stdout
