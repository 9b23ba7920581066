"""The A/B integrate kernels (vbg_ab.hpp: LDS-tiled k_integrate_lt, the round-1 plate map, the
XCD-grouped order) are not in the shipped library; they are built into tools/_ab/libmqr_ab.so
(`make -C metaquest-3d-reconstruction_amd/csrc ab`, part of __graft_entry__.build()).  This runs
test_gpu_numerics.py's integrate tests against that library in a child process (one library per
process) with the A/B variants added: each must equal the generic kernel bit for bit."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB_LIB = os.path.join(ROOT, "tools", "_ab", "libmqr_ab.so")


def test_ab_integrate_variants_equal_generic():
    assert os.path.exists(AB_LIB), f"{AB_LIB} missing: run __graft_entry__.build()"
    env = dict(os.environ, MQR_HIP_LIB=AB_LIB, MQR_AB_TEST="1")
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_numerics.py"), "-k", "integrate",
                        "--timeout", "240", "--timeout-method", "thread"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " passed" in r.stdout and "failed" not in r.stdout, r.stdout[-2000:]
