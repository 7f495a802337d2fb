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


def test_strong_roofline_arithmetic():
    """each strong leg carries its HBM roofline -- the whole frame's algorithmic bytes per
    ms_per_frame against N x 8 TB/s, and every rank's camera phase (owned pixels x 32 B / its raster +
    resolve event time) against one GPU's 8 TB/s."""
    fb = 140_000_000
    s = bench.strong_summary("c4", 1_000_000, 200, 0.030, [0.110, 0.131], [0.020, 0.004], [4_000_000, 4_294_400],
                             "regions", 3, frame_bytes=fb, rank_cam_bytes=[128_000_000, 137_420_800],
                             rank_cam_ms=[0.080, 0.100], ramp={"ms": 61.0, "frames": 96})
    r = s["roofline"]
    ach = fb * 200 / 0.030 / 1e9
    assert abs(r["achieved"] - ach) < 0.01 and r["peak"] == 2 * bench.HBM_PEAK_GBS
    assert abs(r["frac"] - ach / (2 * bench.HBM_PEAK_GBS)) < 1e-4
    assert abs(r["rank_camera_phase_frac"][0] - 128_000_000 / 0.080e-3 / 1e9 / 8000) < 1e-4
    assert abs(r["rank_camera_phase_frac"][1] - 137_420_800 / 0.100e-3 / 1e9 / 8000) < 1e-4
    assert r["rank0_camera_phase_frac"] == r["rank_camera_phase_frac"][0]
    assert s["clock_ramp"]["frames"] == 96
    # N = 1: the leg's whole-frame fraction against one GPU
    s1 = bench.strong_summary("c5", 63_000, 100, 0.038, [0.39], [0.0], [8_294_400], "regions", 3,
                              frame_bytes=300_000_000, rank_cam_bytes=[282_000_000], rank_cam_ms=[0.35])
    assert s1["roofline"]["peak"] == bench.HBM_PEAK_GBS
    assert abs(s1["roofline"]["frac"] - 300_000_000 * 100 / 0.038 / 1e9 / 8000) < 1e-4


def test_strong_leg_failure_on_one_rank_fails_the_leg(monkeypatch):
    """a leg that raises on this rank reaches the common status point and raises there (the
    guarded caller turns it into strong_error) -- single process: no collective, same path."""
    import types

    def boom(*a, **k):
        raise ValueError("rank-local failure")
    monkeypatch.setattr(bench, "run_gpu_c4", boom)
    args = types.SimpleNamespace(strong=["c4"], strong_frames=10, reduce_device="cpu")
    out = bench.strong_legs_guarded(args, 0, 0, 1, None)
    assert set(out) == {"strong_error"} and "rank-local failure" in out["strong_error"]
