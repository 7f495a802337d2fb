"""Shared test helpers: parity assertions between the HIP path and the oracle."""
import numpy as np

FLT_MAX = np.finfo(np.float32).max
TOL = 1e-5  # per-channel tolerance on shaded floats in [0,1] (BASELINE.json north_star)


def assert_depth_bitexact(gpu_d, ref_d):
    g = gpu_d.view(np.uint32)
    r = ref_d.view(np.uint32)
    bad = np.argwhere(g != r)
    assert bad.size == 0, f"{len(bad)} depth words differ, first at {bad[:5].tolist()}: gpu={gpu_d[tuple(bad[0])]!r} ref={ref_d[tuple(bad[0])]!r}"


def assert_color_parity(gpu_c, ref_c, gpu_pq=None, ref_pq=None):
    """Coverage (alpha + which pixels were written) must match exactly.  A shaded byte may differ only
    by 1 and only where both shaders' pre-truncation floats agree within TOL*255 -- i.e. a uint8
    truncation boundary split by an ulp-level libm difference (powf)."""
    assert np.array_equal(gpu_c[..., 3], ref_c[..., 3])
    diff = gpu_c != ref_c
    n = int(diff.sum())
    if n == 0:
        return 0
    assert gpu_pq is not None and ref_pq is not None, f"{n} colour bytes differ and no prequant to explain them"
    idx = np.argwhere(diff)
    d8 = np.abs(gpu_c.astype(np.int16) - ref_c.astype(np.int16))[diff]
    assert d8.max() <= 1, f"colour byte differs by {d8.max()}"
    dp = np.abs(gpu_pq[..., :3] - ref_pq[..., :3])[diff[..., :3]] if diff[..., :3].any() else np.zeros(0)
    assert (dp <= TOL * 255.0).all(), f"pre-truncation floats differ by {dp.max()} (> {TOL * 255})"
    return n


def assert_float_close(gpu, ref, tol=TOL, what="hdr"):
    """Shaded floats (library path: HDR colour, motion): |gpu - ref| <= tol per channel, absolute
    (north_star: within 1e-5 per channel), whatever the magnitude.  Returns the number of channels
    that are not bit-identical (libm powf ulp differences)."""
    assert gpu.shape == ref.shape
    assert np.array_equal(np.isfinite(gpu), np.isfinite(ref)), f"{what}: non-finite values differ"
    fin = np.isfinite(ref)
    err = np.zeros(ref.shape, np.float64)
    err[fin] = np.abs(gpu[fin].astype(np.float64) - ref[fin].astype(np.float64))
    bad = np.argwhere(err > tol)
    assert bad.size == 0, (f"{what}: {len(bad)} channels off by > {tol} (max {err.max():.3g}), first at "
                           f"{bad[:3].tolist()}: gpu={gpu[tuple(bad[0])]!r} ref={ref[tuple(bad[0])]!r}")
    return int((gpu.view(np.uint32) != ref.view(np.uint32)).sum())
