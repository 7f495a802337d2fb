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


def test_camera_phase_bytes_scale_with_owned_pixels():
    """bench.py's library roofline at N > 1: rank 0's timed raster phase is priced
    at the 32 B of each pixel it owns, not the whole frame's, so `frac` does not grow with N."""
    import bench
    from shs_gpu import shard
    W, H, S = 3840, 2160, 2048
    full = bench.camera_phase_bytes(W, H, W * H)
    assert full == W * H * 32
    assert bench.camera_phase_bytes(W, H, W * H, S) == W * H * 32 + S * S * 4
    for n in (2, 4, 8):
        shares = [bench.camera_phase_bytes(W, H, shard.owned_pixels(W, H, 32, r, n)) for r in range(n)]
        assert sum(shares) == full
        assert max(shares) <= full // n + 120 * 32 * 32 * 32    # within one tile row of an even split
        with_shadow = [bench.camera_phase_bytes(W, H, shard.owned_pixels(W, H, 32, r, n), S) for r in range(n)]
        assert abs(sum(with_shadow) - (full + S * S * 4)) < n   # the shadow reads apportioned, floor per rank
