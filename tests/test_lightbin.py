"""The software library's CPU light binning: build_light_bin_culling
(light_culling_runtime.hpp:266-371) -> cull_lights_tiled / _tiled_view_depth_range / _clustered
(jolt_light_culling.hpp:135-412) with classify_vs_cell (jolt_culling.hpp:129-257).

CPU: the oracle restatement (oracle/shs_oracle_lightbin.c) against analytic cases -- a light enclosing
the camera is in every bin, a light behind the camera in none, mode None / no lights give no bins,
lists ascend, the depth-range cells only narrow the tiled lists, the clusters of a tile union to
(a subset of) the tile's list.  GPU: shs_light_bin_culling bit-exact against the oracle (counts and
every index) at C4's 3840x2160 / 16-px tiles / 256 lights in all three modes, with truncated lists
and the depth-range fallback.  Parity unpinned: Jolt v5.2.0 (the SceneShape bounds) and GLM are
absent here; both are restated."""
import numpy as np
import pytest

from shs_gpu import lib_path, scene_lib


def _camera(width=3840, height=2160, zn=0.1, zf=200.0, yaw=0.0):
    ang = np.deg2rad(yaw)
    eye = (np.float32(12.0 * np.sin(ang)), np.float32(8.0), np.float32(-12.0 * np.cos(ang)))
    view = lib_path.look_at_lh(eye, (0.0, 4.0, 40.0))
    proj = lib_path.perspective_lh_no(np.float32(np.deg2rad(60.0)), np.float32(width) / np.float32(height), zn, zf)
    return lib_path.mat_mul(proj, view), eye


def _lb(mode, w=3840, h=2160, **kw):
    vp, _ = _camera(w, h)
    return lib_path.LightBin(w, h, vp, mode=mode, z_near=0.1, z_far=200.0, **kw)


def _depth_ranges(w, h, ts=16, seed=3):
    tx, ty = (w + ts - 1) // ts, (h + ts - 1) // ts
    rng = np.random.default_rng(seed)
    mn = rng.uniform(0.5, 40.0, tx * ty).astype(np.float32)
    mx = (mn + rng.uniform(0.0, 60.0, tx * ty)).astype(np.float32)
    return mn, mx


def test_oracle_enclosing_and_behind(oracle_mod):
    vp, eye = _camera(640, 360)
    lb = lib_path.LightBin(640, 360, vp, mode=1, z_near=0.1, z_far=200.0)
    big = np.array([[eye[0] - 500, eye[1] - 500, eye[2] - 500, eye[0] + 500, eye[1] + 500, eye[2] + 500]], np.float32)
    behind = np.array([[eye[0] - 1, eye[1] - 1, eye[2] - 30, eye[0] + 1, eye[1] + 1, eye[2] - 28]], np.float32)
    bins, counts, idx = oracle_mod.light_bin_culling(lb, np.concatenate([behind, big]))
    assert bins == (40, 23, 1)
    assert (counts == 1).all() and (idx[:, 0] == 1).all()      # the enclosing light everywhere, never the other
    bins, counts, _ = oracle_mod.light_bin_culling(lib_path.LightBin(640, 360, vp, mode=0), big)
    assert bins == (0, 0, 0)
    bins, counts, _ = oracle_mod.light_bin_culling(lb, np.zeros((0, 6), np.float32))
    assert bins == (0, 0, 0)


def test_oracle_lists_ascend_and_modes_nest(oracle_mod):
    aabbs = lib_path.light_aabbs(scene_lib.c4_lights(256))
    w, h = 960, 540
    b1, c1, i1 = oracle_mod.light_bin_culling(_lb(1, w, h), aabbs)
    assert c1.sum() > 0
    for l in np.nonzero(c1)[0]:
        assert np.all(np.diff(i1[l, :c1[l]].astype(np.int64)) > 0)
    mn, mx = _depth_ranges(w, h)
    b2, c2, i2 = oracle_mod.light_bin_culling(_lb(2, w, h, tile_min_view_depth=mn, tile_max_view_depth=mx), aabbs)
    assert b2 == b1 and (c2 <= c1).all() and c2.sum() < c1.sum()
    for l in np.nonzero(c2)[0]:
        assert set(i2[l, :c2[l]]) <= set(i1[l, :c1[l]])
    b3, c3, i3 = oracle_mod.light_bin_culling(_lb(3, w, h), aabbs)
    assert b3 == (b1[0], b1[1], 16)
    per = b1[0] * b1[1]
    for t in range(0, per, 97):
        u = set()
        for z in range(16):
            u |= set(i3[z * per + t, :c3[z * per + t]])
        assert u <= set(i1[t, :c1[t]])
    # depth ranges of the wrong size: the reference falls back to plain tiles (:341-352)
    b4, c4, _ = oracle_mod.light_bin_culling(_lb(2, w, h, tile_min_view_depth=mn[:-1], tile_max_view_depth=mx[:-1]), aabbs)
    assert np.array_equal(c4, c1)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_light_bin_gpu_exact(gpu_ctx, oracle_mod, mode):
    aabbs = lib_path.light_aabbs(scene_lib.c4_lights(256))
    kw = {}
    if mode == 2:
        kw = dict(zip(("tile_min_view_depth", "tile_max_view_depth"), _depth_ranges(3840, 2160)))
    lb = _lb(mode, **kw)
    gb, gc, gi = gpu_ctx.light_bin_culling(lb, aabbs)
    rb, rc, ri = oracle_mod.light_bin_culling(lb, aabbs)
    assert gb == rb
    assert np.array_equal(gc, rc)
    assert rc.sum() > 1000
    for l in np.nonzero(rc)[0]:
        assert np.array_equal(gi[l, :rc[l]], ri[l, :rc[l]]), l


@pytest.mark.gpu
def test_light_bin_gpu_truncated_and_edges(gpu_ctx, oracle_mod):
    """Lists capped at 4 (counts keep every match), a ragged viewport, 1-px tiles on a tiny frame,
    clustered with 5 slices, and an empty light set."""
    aabbs = lib_path.light_aabbs(scene_lib.c4_lights(300, seed=7))
    for lb in (_lb(1, 1000, 563, max_per_bin=4), _lb(3, 333, 211, z_slices=5, max_per_bin=8),
               lib_path.LightBin(37, 23, _camera(37, 23)[0], mode=1, tile_size=1, z_far=200.0)):
        gb, gc, gi = gpu_ctx.light_bin_culling(lb, aabbs)
        rb, rc, ri = oracle_mod.light_bin_culling(lb, aabbs)
        assert gb == rb and np.array_equal(gc, rc)
        cap = gi.shape[1]
        for l in np.nonzero(rc)[0]:
            n = min(int(rc[l]), cap)
            assert np.array_equal(gi[l, :n], ri[l, :n])
    gb, gc, _ = gpu_ctx.light_bin_culling(_lb(1, 640, 360), np.zeros((0, 6), np.float32))
    assert gb == (0, 0, 0)
