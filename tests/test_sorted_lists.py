"""Depth-sorted bin lists (round 6, k_lib_hsort): a camera-pass bin list longer than one deep candidate
round (> 1024 entries, up to LIB_HSORT_MAX = 8192) is sorted whole by depth bound before the raster, and
k_lib_raster stops a tile's candidate rounds once the tile's largest key z lies below the bucket of the
next round's first entry.  The sort changes only the order inside a tile's list; the results must stay
the oracle's bit for bit, z ties (decided by submission order alone) included.

Scenes: thousands of small NDC-space triangles (identity viewproj) packed into a small screen area, on a
few exact depth planes (every overlap of one plane a z tie) plus scattered depths, so the bin tiles hold
from ~1,000 to past 8,192 entries (the sorted and the unsorted paths, either side of both limits)."""
import numpy as np
import pytest

from helpers import assert_depth_bitexact, assert_float_close


def _dense_soup(rng, n, box=0.3, levels=(0.0, 0.5, -0.25), scattered=0.3):
    """n triangles of ~2-6 px at 256x192 inside [-box, box]^2 of NDC; a fraction at random depths."""
    c = rng.uniform(-box, box, size=(n, 1, 2))
    xy = c + rng.normal(scale=0.02, size=(n, 3, 2))
    z = np.asarray(levels, np.float32)[rng.integers(0, len(levels), n)]
    rnd = rng.random(n) < scattered
    z = np.where(rnd, rng.uniform(-0.9, 0.9, n).astype(np.float32), z)
    zc = np.repeat(z[:, None, None], 3, axis=1)
    if scattered:   # some tilted triangles (distinct z per corner)
        tilt = rng.random(n) < 0.5 * scattered
        zc = zc + np.where(tilt[:, None, None], rng.normal(scale=0.05, size=(n, 3, 1)), 0.0)
    pos = np.concatenate([xy, zc], axis=2).reshape(-1, 3).astype(np.float32)
    nrm = rng.normal(size=pos.shape).astype(np.float32)   # distinct shading per triangle: the winner shows
    return pos, nrm


def _render_check(ctx, oracle_mod, frame, draws):
    ctx.render_pbr_forward(frame, draws)
    gh, gd, gm = ctx.resolve_lib()
    rh, rd, rm, rst = oracle_mod.pbr_forward(frame, draws, None)
    assert_depth_bitexact(gd, rd)
    assert_float_close(gm, rm, what="motion")
    assert_float_close(gh, rh, what="hdr")
    st = ctx.lib_stats()
    for k in ("tri_input", "tri_after_clip", "tri_raster"):
        assert st[k] == rst[k], (k, st[k], rst[k])
    return st, rd


@pytest.mark.gpu
@pytest.mark.parametrize("n,box,lo,hi", [(9000, 0.30, 1025, 8192), (30000, 0.22, 8193, 1 << 30)])
def test_sorted_bin_lists_exact(gpu_ctx, oracle_mod, n, box, lo, hi):
    from shs_gpu.lib_path import LibDraw, LibFrame, LibMesh
    rng = np.random.default_rng(n)
    W, H = 256, 192
    pos, nrm = _dense_soup(rng, n, box)
    frame = LibFrame(W, H, depth_motion=True, zn=1.0, zf=1.0, bg_gradient=False, clear_hdr=(0.1, 0.2, 0.3, 1.0))
    d = LibDraw(mesh=LibMesh(pos, nrm), program=2, cull_mode=0)
    for _ in range(2):   # the first pass (no statistics yet) and a pass after one with long lists
        st, rd = _render_check(gpu_ctx, oracle_mod, frame, [d])
        assert lo <= st["max_tile_bin"] <= hi, st["max_tile_bin"]
    cov = rd != np.float32(1.0)
    assert cov.sum() > 2000 and np.isin(rd[cov], np.float32([0.5, 0.75, 0.375])).mean() > 0.02   # tie planes win pixels


@pytest.mark.gpu
def test_sorted_lists_with_a_second_draw_and_painters_order(gpu_ctx, oracle_mod):
    """Two draws (submission bases) over the same dense area, then the same without a depth target (every
    fragment writes, the last submitted wins: no depth bound may stop a round there)."""
    from shs_gpu.lib_path import LibDraw, LibFrame, LibMesh
    rng = np.random.default_rng(5)
    W, H = 256, 192
    p0, n0 = _dense_soup(rng, 5000, 0.25)
    p1, n1 = _dense_soup(rng, 4000, 0.25, levels=(0.5, 0.1))
    d0 = LibDraw(mesh=LibMesh(p0, n0), program=2, cull_mode=0)
    d1 = LibDraw(mesh=LibMesh(p1, n1), program=3, cull_mode=0, base_color=(0.9, 0.3, 0.2))
    frame = LibFrame(W, H, depth_motion=True, zn=1.0, zf=1.0, bg_gradient=False, clear_hdr=(0.1, 0.2, 0.3, 1.0))
    for _ in range(2):
        st, _ = _render_check(gpu_ctx, oracle_mod, frame, [d0, d1])
        assert st["max_tile_bin"] > 1024
    nodepth = LibFrame(W, H, depth_motion=False, zn=1.0, zf=1.0, bg_gradient=False, clear_hdr=(0.1, 0.2, 0.3, 1.0))
    gpu_ctx.render_pbr_forward(nodepth, [d0, d1])
    gh, _, _ = gpu_ctx.resolve_lib()
    rh, _, _, _ = oracle_mod.pbr_forward(nodepth, [d0, d1], None)
    assert_float_close(gh, rh, what="hdr")
