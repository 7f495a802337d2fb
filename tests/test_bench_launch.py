"""bench.py --gpus N started directly (as the driver does) must run N ranks, not one process on one
GPU.  --launch-dry-run makes every rank join a gloo group and report its
rank / LOCAL_RANK without touching a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_starts_n_ranks(n):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-dry-run"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    got = json.loads(line)
    assert got["world"] == n
    assert sorted(got["ranks"]) == list(range(n))
    assert sorted(got["local_ranks"]) == list(range(n))


def test_bench_world_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--launch-dry-run"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
