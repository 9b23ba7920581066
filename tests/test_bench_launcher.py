"""bench.py --gpus N self-launch (no torchrun around it): the parent starts N fresh rank processes
with the torch.distributed env contract, relays rank 0's JSON line and returns the worst exit code;
a failing rank takes the others down.  A stub child stands in for the rank (no torch, no GPU)."""
import io
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (stdlib-only at import time)

STUB = r'''
import json, os, sys, time
mode = sys.argv[1]
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                      "MASTER_ADDR", "MASTER_PORT")}
assert env["LOCAL_RANK"] == env["RANK"] and env["LOCAL_WORLD_SIZE"] == env["WORLD_SIZE"], env
assert env["MASTER_ADDR"] == "127.0.0.1" and int(env["MASTER_PORT"]) > 0, env
if mode == "ok":
    if r == 0:
        print("not json noise")
        print(json.dumps({"n_gpus": w, "env": env, "argv": sys.argv[2:]}), flush=True)
    sys.exit(0)
if mode == "fail1":           # rank 1 fails at once, the others would hang
    if r == 1:
        sys.exit(3)
    time.sleep(600)
if mode == "hang":
    time.sleep(600)
if mode == "gloo":            # a real gloo rendezvous through the env the launcher set
    import torch.distributed as dist
    import torch
    dist.init_process_group("gloo")
    t = torch.tensor([r + 1.0])
    dist.all_reduce(t)
    if r == 0:
        print(json.dumps({"sum": float(t.item()), "n_gpus": w}), flush=True)
    dist.destroy_process_group()
'''


@pytest.fixture()
def stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return p


def _launch(stub, mode, n, timeout=60.0, extra=()):
    out = io.StringIO()
    rc = bench.launch_ranks(n, [mode, *extra], child=[sys.executable, str(stub)], timeout=timeout, out=out,
                            grace=2.0)
    lines = [ln for ln in out.getvalue().splitlines() if ln.startswith("{")]
    return rc, lines


def test_launcher_sets_the_rank_env_and_relays_rank0(stub):
    rc, lines = _launch(stub, "ok", 4, extra=("--gpus", "4", "--steps", "3"))
    assert rc == 0 and len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 4 and rec["env"]["RANK"] == "0" and rec["env"]["WORLD_SIZE"] == "4"
    assert rec["argv"] == ["--gpus", "4", "--steps", "3"]


def test_launcher_kills_the_siblings_of_a_failed_rank(stub):
    t = time.monotonic()
    rc, lines = _launch(stub, "fail1", 3)
    assert time.monotonic() - t < 30, "siblings not terminated"
    assert rc in (3, 137, 143), rc  # the worst of rank 1's 3 and its SIGTERM'd (or killed) siblings
    rec = json.loads(lines[-1])
    assert rec["value"] is None and "exited" in rec["error"]


def test_launcher_time_limit(stub):
    t = time.monotonic()
    rc, lines = _launch(stub, "hang", 2, timeout=2.0)
    assert time.monotonic() - t < 20
    assert rc >= 124 and json.loads(lines[-1])["value"] is None


def test_launcher_gloo_rendezvous(stub):
    rc, lines = _launch(stub, "gloo", 2, timeout=120.0)
    assert rc == 0 and json.loads(lines[0]) == {"sum": 3.0, "n_gpus": 2}


def test_bench_rejects_a_world_size_other_than_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 1
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["value"] is None and "WORLD_SIZE=2" in rec["error"]


def test_rank_stdout_carries_only_the_json_line():
    """Native libraries write to fd 1 behind Python's back (gloo's connection log): in a rank process
    bench._json_stdout points fd 1 at stderr, so stdout holds the JSON line alone."""
    code = ("import os, sys, json; sys.path.insert(0, %r); import bench\n"
            "out = bench._json_stdout()\n"
            "os.write(1, b'[Gloo] Rank 0 is connected to 1 peer ranks\\n')\n"
            "print('python log line')\n"
            "print(json.dumps({'value': 1.0}), file=out, flush=True)\n") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert p.stdout.splitlines() == ['{"value": 1.0}'], p.stdout
    assert "[Gloo]" in p.stderr and "python log line" in p.stderr
