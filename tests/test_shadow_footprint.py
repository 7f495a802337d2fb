"""SHS_OPT_SHADOW_FOOTPRINT's bound (csrc/shs_footprint.hpp, host-only shs_shadow_footprint): the texels a
camera pass's PCF can read (lighting/shadow_sample.hpp:65-104) from points of a draw's world box that
project onto the rank's pixel rectangle.  Checked here without a GPU against brute force: random world
points of the box, kept where their camera projection lands on a pixel centre of the rectangle and
inside the clip volume, projected with the light camera exactly as shadow_visibility_dir does (round
to a texel, +- the PCF reach, clamped) -- every such texel must lie in the footprint."""
import numpy as np
import pytest

import shs_gpu
from shs_gpu import scene_lib


def _mat(m):
    return np.asarray(m, np.float64).reshape(4, 4).T    # column-major float[16] -> row-major matrix


def _world_box(draw):
    p = np.asarray(draw.mesh.positions, np.float64).reshape(-1, 3)
    M = _mat(draw.model)
    w = p @ M[:3, :3].T + M[:3, 3]
    return w.min(axis=0), w.max(axis=0)


def _light_vp(S=2048):
    """The C5 light camera (shs_render_shadow_map's build_dir_light_camera_aabb) from the oracle, which
    restates it (oracle/shs_oracle_lib.c); the footprint only needs the matrix."""
    from oracle import oracle
    frame, draws, casters, sun, S = scene_lib.c5_scene(384, 216, S)
    _, lvp = oracle.shadow_map(S, sun, casters)
    return lvp


def _brute(lvp, S, cvp, W, H, px, bmin, bmax, reach, n=400_000, seed=1):
    rng = np.random.default_rng(seed)
    pts = rng.uniform(bmin, bmax, size=(n, 3))
    ph = np.concatenate([pts, np.ones((n, 1))], axis=1)
    c = ph @ _mat(cvp).T
    w = c[:, 3]
    ok = (w > 0) & (np.abs(c[:, 0]) <= w) & (np.abs(c[:, 1]) <= w) & (np.abs(c[:, 2]) <= w)
    sx = (c[:, 0] / w * 0.5 + 0.5) * (W - 1)
    sy = (c[:, 1] / w * 0.5 + 0.5) * (H - 1)
    ok &= (sx >= px[0] + 0.5) & (sx <= px[2] + 0.5) & (sy >= px[1] + 0.5) & (sy <= px[3] + 0.5)
    lp = ph[ok] @ _mat(lvp).T
    u = (lp[:, 0] / lp[:, 3]) * 0.5 + 0.5
    v = (lp[:, 1] / lp[:, 3]) * 0.5 + 0.5
    inside = (u >= 0) & (u <= 1) & (v >= 0) & (v <= 1)   # outside the map: lit, nothing read
    cx = np.round(u[inside] * (S - 1)).astype(np.int64)
    cy = np.round(v[inside] * (S - 1)).astype(np.int64)
    if cx.size == 0:
        return None
    return (int(np.clip(cx.min() - reach, 0, S - 1)), int(np.clip(cy.min() - reach, 0, S - 1)),
            int(np.clip(cx.max() + reach, 0, S - 1)), int(np.clip(cy.max() + reach, 0, S - 1)))


@pytest.mark.parametrize("rect", [(0, 0, 3839, 2159), (0, 0, 959, 1079), (1920, 1080, 3839, 2159), (2880, 0, 3839, 2159),
                                  (1600, 900, 1663, 931)])
@pytest.mark.parametrize("which", [0, 1])   # floor, Suzanne
def test_footprint_holds_every_read_texel(rect, which):
    S, W, H = 2048, 3840, 2160
    lvp = _light_vp(S)
    frame, draws, _, _, _ = scene_lib.c5_scene(W, H, S)
    d = draws[which]
    bmin, bmax = _world_box(d)
    reach = 2
    fp = shs_gpu.Context.shadow_footprint(lvp, S, d.viewproj, W, H, rect, bmin, bmax, reach)
    got = _brute(lvp, S, d.viewproj, W, H, rect, bmin, bmax, reach)
    if got is None:
        return
    assert fp[2] >= fp[0] and fp[3] >= fp[1], f"empty footprint but texels {got} are read"
    assert fp[0] <= got[0] and fp[1] <= got[1] and fp[2] >= got[2] and fp[3] >= got[3], (fp, got)
    # and not the whole map for a partial view (the bound is useful, not just safe)
    if rect == (2880, 0, 3839, 2159):
        assert (fp[2] - fp[0] + 1) * (fp[3] - fp[1] + 1) < 0.6 * S * S, fp


def test_footprint_of_a_box_off_the_rectangle_is_empty():
    S, W, H = 2048, 3840, 2160
    lvp = _light_vp(S)
    frame, draws, _, _, _ = scene_lib.c5_scene(W, H, S)
    d = draws[1]                           # Suzanne sits near the screen centre
    bmin, bmax = _world_box(d)
    fp = shs_gpu.Context.shadow_footprint(lvp, S, d.viewproj, W, H, (0, 0, 127, 127), bmin, bmax, 2)
    assert fp[2] < fp[0] or fp[3] < fp[1], fp
    assert _brute(lvp, S, d.viewproj, W, H, (0, 0, 127, 127), bmin, bmax, 2) is None
    # an empty pixel rectangle reads nothing
    fp = shs_gpu.Context.shadow_footprint(lvp, S, d.viewproj, W, H, (5, 5, 4, 4), bmin, bmax, 2)
    assert fp[2] < fp[0]


def test_footprint_degenerate_inputs_fall_back_to_the_whole_map():
    S = 512
    eye = np.eye(4, dtype=np.float32).reshape(16)
    nan = eye.copy()
    nan[0] = np.nan
    fp = shs_gpu.Context.shadow_footprint(eye, S, nan, 64, 64, (0, 0, 63, 63), (-1, -1, -1), (1, 1, 1), 1)
    assert fp == (0, 0, S - 1, S - 1)
    # a light projection with w <= 0 somewhere on the polytope: no bound, the whole map
    flip = np.diag([1.0, 1.0, 1.0, -1.0]).astype(np.float32).reshape(16)
    fp = shs_gpu.Context.shadow_footprint(flip, S, eye, 64, 64, (0, 0, 63, 63), (-0.5, -0.5, -0.5), (0.5, 0.5, 0.5), 1)
    assert fp == (0, 0, S - 1, S - 1)


@pytest.mark.gpu
@pytest.mark.parametrize("count", [1, 3])
def test_footprint_frames_match_oracle(oracle_mod, count):
    """SHS_OPT_SHADOW_FOOTPRINT on: the shadow pass is recorded and enqueued by the camera pass over only
    its footprint's tiles (for count > 1: region-sharded ranks, two frames each); the composed HDR /
    depth / motion equal the oracle frame (whole shadow map) as without the option, every rank's shadow
    region is a strict part of the map, and resolving a recorded pass renders the whole map exactly."""
    from helpers import assert_depth_bitexact, assert_float_close
    W, H, S = 960, 540, 1024
    frame, draws, casters, sun, _ = scene_lib.c5_scene(W, H, S)
    sm_ref, lvp_ref = oracle_mod.shadow_map(S, sun, casters)
    scene_lib.wire_shadow(draws, lvp_ref)
    rh, rd, rm, _ = oracle_mod.pbr_forward(frame, draws, sm_ref)
    ctxs = [shs_gpu.Context(0) for _ in range(count)]
    tiles = (S + 31) // 32
    try:
        for it in range(2):
            gh, gd, gm = np.zeros_like(rh), np.zeros_like(rd), np.zeros_like(rm)
            for r, c in enumerate(ctxs):
                c.set_shadow_footprint(True)
                if count > 1:
                    c.set_shard_layout(True)
                frame.shard_rank, frame.shard_count = r, count
                lvp = c.render_shadow_map(S, sun, casters)
                assert np.array_equal(lvp.view(np.uint32), lvp_ref.view(np.uint32))
                assert c.shadow_region()[2] < c.shadow_region()[0], "a recorded pass is not enqueued yet"
                c.render_pbr_forward(frame, draws)
                x0, y0, x1, y1 = c.shadow_region()
                assert (x1 - x0 + 1) * (y1 - y0 + 1) < tiles * tiles, "the footprint is the whole map"
                h, d, m = c.resolve_lib()
                if count > 1:
                    rx0, ry0, rx1, ry1 = c.shard_regions(count)[r]
                    own = np.zeros((H, W), bool)
                    own[ry0 * 32:(ry1 + 1) * 32, rx0 * 32:(rx1 + 1) * 32] = True
                else:
                    own = np.ones((H, W), bool)
                gh[own], gd[own], gm[own] = h[own], d[own], m[own]
            assert_depth_bitexact(gd, rd)
            assert_float_close(gm, rm, what="motion")
            assert_float_close(gh, rh, what="hdr")
        # a recorded pass read back: rendered whole, equal to the oracle's map
        c = ctxs[0]
        frame.shard_rank, frame.shard_count = 0, 1
        c.render_shadow_map(S, sun, casters)
        assert_depth_bitexact(c.resolve_shadow_map(), sm_ref)
        assert c.shadow_region() == (0, 0, tiles - 1, tiles - 1)
    finally:
        for c in ctxs:
            c.close()
        frame.shard_rank, frame.shard_count = 0, 1


def _own_mask(c, count, rank, W, H):
    if count == 1:
        return np.ones((H, W), bool)
    rx0, ry0, rx1, ry1 = c.shard_regions(count)[rank]
    own = np.zeros((H, W), bool)
    own[ry0 * 32:(ry1 + 1) * 32, rx0 * 32:(rx1 + 1) * 32] = True
    return own


@pytest.mark.gpu
def test_footprint_map_reused_by_later_passes(oracle_mod):
    """one footprint-restricted shadow map sampled by several camera passes (a static sun
    reused over frames): another region of the same view, then another view.  Each pass whose footprint
    leaves what was rendered re-renders the map over the union; every pass matches the oracle."""
    from helpers import assert_depth_bitexact, assert_float_close
    W, H, S, count = 960, 540, 1024, 3
    frame, draws, casters, sun, _ = scene_lib.c5_scene(W, H, S)
    sm_ref, lvp_ref = oracle_mod.shadow_map(S, sun, casters)
    c = shs_gpu.Context(0)
    try:
        c.set_shadow_footprint(True)
        c.set_shard_layout(True)
        lvp = c.render_shadow_map(S, sun, casters)
        assert np.array_equal(lvp.view(np.uint32), lvp_ref.view(np.uint32))
        regions = []
        for yaw, rank in [(0.0, 0), (0.0, 2), (55.0, 1), (-70.0, 0)]:
            frame, draws, _, _, _ = scene_lib.c5_scene(W, H, S, yaw=yaw)
            scene_lib.wire_shadow(draws, lvp_ref)
            rh, rd, rm, _ = oracle_mod.pbr_forward(frame, draws, sm_ref)
            frame.shard_rank, frame.shard_count = rank, count
            c.render_pbr_forward(frame, draws)
            regions.append(c.shadow_region())
            h, d, m = c.resolve_lib()
            own = _own_mask(c, count, rank, W, H)
            assert_depth_bitexact(np.where(own, d, rd), rd)
            assert_float_close(np.where(own[..., None], m, rm), rm, what="motion")
            assert_float_close(np.where(own[..., None], h, rh), rh, what="hdr")
        for a, b in zip(regions, regions[1:]):   # the rendered rectangle only grows
            assert b[0] <= a[0] and b[1] <= a[1] and b[2] >= a[2] and b[3] >= a[3], regions
        assert regions[-1] != regions[0], "no later pass read beyond the first footprint"
    finally:
        c.close()


@pytest.mark.gpu
def test_footprint_empty_for_a_rank(oracle_mod):
    """a rank whose rectangle no shadowed draw reaches (only Suzanne samples the map) records
    an empty footprint: its shadow pass renders nothing, the region reads as empty and its pixels still
    match the oracle."""
    from helpers import assert_depth_bitexact, assert_float_close
    W, H, S, count = 960, 540, 1024, 8
    frame, draws, casters, sun, _ = scene_lib.c5_scene(W, H, S)
    sm_ref, lvp_ref = oracle_mod.shadow_map(S, sun, casters)
    scene_lib.wire_shadow(draws, lvp_ref)
    draws[0].shadow = False                     # the floor does not sample the map
    rh, rd, rm, _ = oracle_mod.pbr_forward(frame, draws, sm_ref)
    n_empty = 0
    for rank in range(count):
        c = shs_gpu.Context(0)
        try:
            c.set_shadow_footprint(True)
            c.set_shard_layout(True)
            for _ in range(2):                      # the second pass balances on the first one's bounds
                c.render_shadow_map(S, sun, casters)
                frame.shard_rank, frame.shard_count = rank, count
                c.render_pbr_forward(frame, draws)
                h, d, m = c.resolve_lib()
            reg = c.shadow_region()
            n_empty += reg[2] < reg[0] or reg[3] < reg[1]
            own = _own_mask(c, count, rank, W, H)
            assert_depth_bitexact(np.where(own, d, rd), rd)
            assert_float_close(np.where(own[..., None], m, rm), rm, what="motion")
            assert_float_close(np.where(own[..., None], h, rh), rh, what="hdr")
        finally:
            c.close()
            frame.shard_rank, frame.shard_count = 0, 1
    assert n_empty >= 1, "every rank's rectangle reached Suzanne's shadow reads"


def _brute_texels(lvp, S, cvp, W, H, px, bmin, bmax, reach, n=400_000, seed=1):
    """The brute force's read texels themselves: (cx, cy) of every kept point, before the +- reach."""
    rng = np.random.default_rng(seed)
    pts = rng.uniform(bmin, bmax, size=(n, 3))
    ph = np.concatenate([pts, np.ones((n, 1))], axis=1)
    c = ph @ _mat(cvp).T
    w = c[:, 3]
    ok = (w > 0) & (np.abs(c[:, 0]) <= w) & (np.abs(c[:, 1]) <= w) & (np.abs(c[:, 2]) <= w)
    sx = (c[:, 0] / w * 0.5 + 0.5) * (W - 1)
    sy = (c[:, 1] / w * 0.5 + 0.5) * (H - 1)
    ok &= (sx >= px[0] + 0.5) & (sx <= px[2] + 0.5) & (sy >= px[1] + 0.5) & (sy <= px[3] + 0.5)
    lp = ph[ok] @ _mat(lvp).T
    u = (lp[:, 0] / lp[:, 3]) * 0.5 + 0.5
    v = (lp[:, 1] / lp[:, 3]) * 0.5 + 0.5
    inside = (u >= 0) & (u <= 1) & (v >= 0) & (v <= 1)
    return np.round(u[inside] * (S - 1)).astype(np.int64), np.round(v[inside] * (S - 1)).astype(np.int64)


@pytest.mark.parametrize("rect", [(0, 0, 3839, 2159), (1920, 1080, 3839, 2159), (960, 1080, 1919, 2159),
                                  (1600, 900, 1663, 931)])
@pytest.mark.parametrize("which", [0, 1])   # floor, Suzanne
def test_footprint_rows_hold_every_read_texel(rect, which):
    """Round 6: the per-row spans of the footprint (the convex hull of the polytope's light-space image,
    what a footprint shadow pass renders of its rectangle) hold every texel the brute force reads,
    PCF taps included, and for a partial view are much smaller than the rectangle."""
    S, W, H, reach = 2048, 3840, 2160, 2
    lvp = _light_vp(S)
    frame, draws, _, _, _ = scene_lib.c5_scene(W, H, S)
    d = draws[which]
    bmin, bmax = _world_box(d)
    x0, x1 = shs_gpu.Context.shadow_footprint_rows(lvp, S, d.viewproj, W, H, rect, bmin, bmax, reach)
    cx, cy = _brute_texels(lvp, S, d.viewproj, W, H, rect, bmin, bmax, reach)
    for ox in (-reach, reach):                         # the PCF taps' extreme columns and rows
        for oy in (-reach, 0, reach):
            tx, ty = np.clip(cx + ox, 0, S - 1), np.clip(cy + oy, 0, S - 1)
            r = ty // 32
            assert (x0[r] <= x1[r]).all(), "a read texel in a row with no span"
            assert ((tx >= x0[r]) & (tx <= x1[r])).all(), (rect, which, ox, oy)
    fp = shs_gpu.Context.shadow_footprint(lvp, S, d.viewproj, W, H, rect, bmin, bmax, reach)
    if fp[2] >= fp[0]:
        span = np.where(x1 >= x0, x1 - x0 + 1, 0).sum() * 32
        assert span <= (fp[2] - fp[0] + 1) * (fp[3] // 32 - fp[1] // 32 + 1) * 32, (span, fp)   # within the rectangle's rows
        if rect == (960, 1080, 1919, 2159) and which == 0:   # the far floor of a partial view: much smaller
            assert span < 0.7 * (fp[2] - fp[0] + 1) * (fp[3] - fp[1] + 1), (span, fp)
