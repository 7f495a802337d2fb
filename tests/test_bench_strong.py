"""bench.py's strong-scaling legs: the keys the driver's `--gpus N` line carries for the
4K tile-sharded C4 / C5 frames, computed from per-rank measurements (CPU: the arithmetic only)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_strong_summary_arithmetic():
    s = bench.strong_summary("c4", 1_000_000, 60, 0.0125, [0.110, 0.131, 0.098], [0.020, 0.004, 0.005],
                             [3_000_000, 2_500_000, 2_794_400], "regions", 3)
    assert s["n_gpus"] == 3 and s["frames"] == 60
    assert abs(s["ms_per_frame"] - 0.0125 / 60 * 1e3) < 1e-5
    assert abs(s["mtri_s"] - 1_000_000 * 60 / 0.0125 / 1e6) < 1e-3
    assert s["worst_rank"] == 1 and s["worst_rank_kernels_ms"] == 0.131
    assert s["gather_ms"] == [0.02, 0.004, 0.005]
    assert sum(s["owned_pixels"]) == 3840 * 2160
    assert s["layout"] == "regions" and s["frames_in_flight"] == 3
    assert s["workload"] == bench.WORKLOADS["c4"]


def test_strong_summary_single_gpu_is_whole_frame():
    s = bench.strong_summary("c5", 63_000, 60, 0.024, np.array([0.39]), np.array([0.0]), np.array([3840 * 2160.0]),
                             "regions", 3)
    assert s["n_gpus"] == 1 and s["worst_rank"] == 0 and s["layout"] == "whole frame"
    assert s["owned_pixels"] == [3840 * 2160]


def test_strong_legs_default_on():
    """The driver's plain `bench.py --gpus N` runs both legs (argparse default)."""
    import argparse
    old = sys.argv
    try:
        sys.argv = ["bench.py"]
        ap_args = None

        def fake_parse(self, *a, **k):
            nonlocal ap_args
            ap_args = argparse.ArgumentParser.parse_known_args(self, [])[0]
            raise SystemExit(0)
        orig = argparse.ArgumentParser.parse_args
        argparse.ArgumentParser.parse_args = fake_parse
        try:
            bench.main()
        except SystemExit:
            pass
        finally:
            argparse.ArgumentParser.parse_args = orig
    finally:
        sys.argv = old
    assert ap_args.strong == ["c4", "c5"] and ap_args.strong_frames > 0


def test_strong_legs_failure_keeps_the_headline(monkeypatch):
    """A sharded leg that raises on every rank leaves strong_error in the line instead of ending the bench."""
    def boom(*a, **k):
        raise RuntimeError("sharded leg failed")
    monkeypatch.setattr(bench, "strong_legs", boom)
    out = bench.strong_legs_guarded(None, 0, 0, 1, None)
    assert set(out) == {"strong_error"} and "sharded leg failed" in out["strong_error"]
