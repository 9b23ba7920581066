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


def test_ab_extraction_modes_bit_identical():
    """The A/B library's extraction configurations (tools/ab_extract.py modes: per-cube triangle
    counts from the count pass, LDS row maps, the scan's totals written straight to pinned memory; all
    three = the shipped default 7) emit the same mesh bit for bit on the C2 volume."""
    import json
    assert os.path.exists(AB_LIB), f"{AB_LIB} missing: run __graft_entry__.build()"
    env = dict(os.environ, MQR_HIP_LIB=AB_LIB)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "ab_extract.py"), "--modes", "0,1,2,3,4,7",
                        "--reps", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])["modes"]
    assert set(res) == {"0", "1", "2", "3", "4", "7"}
    assert all(m["bit_identical_to_first"] for m in res.values()), res
    assert res["0"]["triangles"] > 1_000_000
