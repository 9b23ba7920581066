"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer: every entry
point of oracle/mqr_oracle.c runs once on a procedural scene (oracle/asan_driver.c); any memory
error, leak or undefined behaviour fails the build's run.  Host code only (no GPU sanitizers)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_clean_under_asan_ubsan():
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "asan driver ok" in r.stdout
