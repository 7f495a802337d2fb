"""GPU parity of the library path (rasterize_mesh + builtin programs, PassShadowMap, PassPBRForward)
against the CPU oracle (oracle/shs_oracle_lib.c), through the C ABI.

Coverage, depth (z01) and the shadow map: bit-exact.  HDR colour and motion vectors: within 1e-5 per
channel, absolute (helpers.assert_float_close)."""
import numpy as np
import pytest

from helpers import assert_depth_bitexact, assert_float_close

pytestmark = pytest.mark.gpu


def _both(ctx, oracle_mod, frame, draws, shadow=None):
    """shadow = (size, sun_dir, casters) -> shadow pass on both sides first."""
    sm_ref = None
    if shadow is not None:
        size, sun, casters = shadow
        lvp = ctx.render_shadow_map(size, sun, casters)
        sm_ref, lvp_ref = oracle_mod.shadow_map(size, sun, casters)
        assert np.array_equal(lvp.view(np.uint32), lvp_ref.view(np.uint32)), "light camera differs"
        sm_gpu = ctx.resolve_shadow_map()
        assert_depth_bitexact(sm_gpu, sm_ref)
        for d in draws:
            if d.shadow:
                d.light_viewproj = lvp
    ctx.render_pbr_forward(frame, draws)
    g = ctx.resolve_lib()
    st = ctx.lib_stats()
    r = oracle_mod.pbr_forward(frame, draws, sm_ref)
    return g, r, st


def _check(ctx, oracle_mod, frame, draws, shadow=None):
    (gh, gd, gm), (rh, rd, rm, rst), st = _both(ctx, oracle_mod, frame, draws, shadow)
    for k in ("tri_input", "tri_after_clip", "tri_raster"):
        assert st[k] == rst[k], (k, st[k], rst[k])
    if gd is not None:
        assert_depth_bitexact(gd, rd)
        assert st["covered_pixels"] == int((rd < 1.0).sum())
        assert_float_close(gm, rm, what="motion")
    assert_float_close(gh, rh, what="hdr")
    return st


@pytest.mark.parametrize("program", [0, 1, 2, 3, 4])
def test_c5_small_all_programs(gpu_ctx, oracle_mod, program):
    from shs_gpu import scene_lib
    frame, draws, casters, sun, _ = scene_lib.c5_scene(480, 270, program=program)
    scene_lib.wire_shadow(draws, np.eye(4, dtype=np.float32).reshape(16))
    st = _check(gpu_ctx, oracle_mod, frame, draws, shadow=(256, sun, casters))
    assert st["covered_pixels"] > 20000
    assert st["tri_after_clip"] > 0


def test_c5_no_shadow_no_motion(gpu_ctx, oracle_mod):
    from shs_gpu import scene_lib
    frame, draws, _, _, _ = scene_lib.c5_scene(400, 300, motion=False, yaw=25.0)
    _check(gpu_ctx, oracle_mod, frame, draws)


def test_c5_shadow_map_sizes(gpu_ctx, oracle_mod):
    """Non-square shadow map and a second frame re-using the context's buffers."""
    from shs_gpu import scene_lib
    frame, draws, casters, sun, _ = scene_lib.c5_scene(320, 200, yaw=-40.0)
    scene_lib.wire_shadow(draws, np.eye(4, dtype=np.float32).reshape(16))
    for d in draws:
        d.shadow_pcf_radius = 1
    _check(gpu_ctx, oracle_mod, frame, draws, shadow=((300, 170), sun, casters))
    for d in draws:
        d.shadow_pcf_radius, d.shadow_pcf_step = 0, 2.0
    _check(gpu_ctx, oracle_mod, frame, draws, shadow=(128, sun, casters))


@pytest.mark.parametrize("W,H", [(1, 1), (1, 29), (37, 1), (16, 4), (65, 33)])
def test_tiny_frames(gpu_ctx, oracle_mod, W, H):
    """Frames below one 16x16 raster tile / one 16x4 resolve block, single rows and columns: the
    edge masks of the raster, the per-block coverage words and the resolve's pixel guard."""
    from shs_gpu import scene_lib
    frame, draws, casters, sun, _ = scene_lib.c5_scene(W, H, program=(W + H) % 5)
    scene_lib.wire_shadow(draws, np.eye(4, dtype=np.float32).reshape(16))
    _check(gpu_ctx, oracle_mod, frame, draws, shadow=(64, sun, casters))


def test_resize_sequence(gpu_ctx, oracle_mod):
    """One context through heights / widths that keep or change the bin-tile grid and the raster-tile
    rows, with the shadow map resized between frames: every frame vs the oracle."""
    from shs_gpu import scene_lib
    for (W, H), sm in zip([(96, 64), (96, 56), (96, 64), (90, 60), (33, 17), (96, 64)], [64, 64, 64, 48, 80, 64]):
        frame, draws, casters, sun, _ = scene_lib.c5_scene(W, H, program=W % 5)
        scene_lib.wire_shadow(draws, np.eye(4, dtype=np.float32).reshape(16))
        _check(gpu_ctx, oracle_mod, frame, draws, shadow=(sm, sun, casters))


def _clip_soup(rng, n):
    """Random world-space triangles around a perspective camera: many cross the near / far / side
    planes (Sutherland-Hodgman + fan), some lie behind the eye, some are degenerate."""
    c = rng.uniform([-12, -8, -2], [12, 8, 40], size=(n, 1, 3))
    tris = c + rng.normal(scale=rng.choice([0.3, 2.0, 9.0], size=(n, 1, 1)), size=(n, 3, 3))
    tris[: n // 20, 2] = tris[: n // 20, 0] + 1e-4 * rng.normal(size=(n // 20, 3))   # near-degenerate
    pos = tris.reshape(-1, 3).astype(np.float32)
    nrm = rng.normal(size=pos.shape).astype(np.float32)
    uv = rng.uniform(-2, 2, size=(pos.shape[0], 2)).astype(np.float32)
    return pos, nrm, uv


def _camera(width, height, zn=0.5, zf=30.0):
    from shs_gpu.lib_path import look_at_lh, mat_mul, perspective_lh_no
    view = look_at_lh((0.3, 0.7, -3.0), (0.0, 0.0, 10.0))
    proj = perspective_lh_no(np.float32(np.deg2rad(60.0)), np.float32(width) / np.float32(height), zn, zf)
    return mat_mul(proj, view)


@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("cull", [0, 1, 2])
def test_clip_soup_exact(gpu_ctx, oracle_mod, seed, cull):
    from shs_gpu.lib_path import LibDraw, LibFrame, LibMesh, model_euler
    rng = np.random.default_rng(seed)
    W, H = 331, 227
    pos, nrm, uv = _clip_soup(rng, 1200)
    mesh = LibMesh(pos, nrm[: len(nrm) - 7], uv)          # short normal array -> (0,1,0) defaults
    vp = _camera(W, H)
    d = LibDraw(mesh=mesh, program=seed % 2, viewproj=vp, model=model_euler((0.1, -0.2, 0.3), (0.2, 0.4, -0.1), (1.0, 1.2, 0.9)),
                prev_model=model_euler((0.0, -0.2, 0.3), (0.2, 0.45, -0.1), (1.0, 1.2, 0.9)), camera_pos=(0.3, 0.7, -3.0),
                cull_mode=cull, front_face_ccw=bool(seed % 2), enable_motion_vectors=True, light_intensity=3.0)
    st = _check(gpu_ctx, oracle_mod, LibFrame(W, H, zn=0.5, zf=30.0), [d])
    assert st["clipped_extra"] > 0 and st["tri_after_clip"] > st["tri_raster"] // 2


def test_painter_mode_without_depth_target(gpu_ctx, oracle_mod):
    """No RT_ColorDepthMotion: every fragment writes colour, the last in submission order wins."""
    from shs_gpu.lib_path import LibDraw, LibFrame, LibMesh
    rng = np.random.default_rng(5)
    W, H = 200, 150
    pos, nrm, uv = _clip_soup(rng, 600)
    vp = _camera(W, H)
    draws = [LibDraw(mesh=LibMesh(pos[:900], nrm[:900], uv[:900]), program=3, viewproj=vp, cull_mode=0),
             LibDraw(mesh=LibMesh(pos[900:], nrm[900:], uv[900:]), program=2, viewproj=vp, cull_mode=0,
                     base_color=(0.2, 0.9, 0.1))]
    frame = LibFrame(W, H, depth_motion=False, bg_gradient=False, clear_hdr=(0.1, 0.2, 0.3, 1.0))
    _check(gpu_ctx, oracle_mod, frame, draws)


def test_linear_depth_off(gpu_ctx, oracle_mod):
    """zf <= zn + 1e-6: the NDC depth (z_ndc * 0.5 + 0.5) is kept (rasterizer.hpp:354)."""
    from shs_gpu.lib_path import LibDraw, LibFrame, LibMesh
    rng = np.random.default_rng(9)
    pos, nrm, uv = _clip_soup(rng, 500)
    vp = _camera(160, 120)
    _check(gpu_ctx, oracle_mod, LibFrame(160, 120, zn=1.0, zf=1.0), [LibDraw(mesh=LibMesh(pos, nrm, uv), viewproj=vp, cull_mode=0)])


def test_indexed_grid_bins_mode(gpu_ctx, oracle_mod):
    """> 4096 primitives (per-tile bins), 16 indexed monkeys + floor, several draws, 2 programs."""
    from shs_gpu import scene_lib
    from shs_gpu.lib_path import LibDraw, model_euler
    frame, draws, casters, sun, _ = scene_lib.c5_scene(512, 288)
    base = draws[1]
    for i in range(16):
        m = model_euler(((i % 4) * 3.0 - 4.5, 1.0 + (i // 4) * 0.4, (i // 4) * 3.0 - 2.0), (0.0, 0.3 * i, 0.0), (1.0, 1.0, 1.0))
        draws.append(LibDraw(mesh=base.mesh, program=i % 2, model=m, viewproj=base.viewproj,
                             prev_viewproj=base.prev_viewproj, light_dir_ws=base.light_dir_ws, light_intensity=5.0,
                             camera_pos=base.camera_pos, base_color=(0.2 + 0.05 * i, 0.5, 0.7), roughness=0.3,
                             cull_mode=i % 3, enable_motion_vectors=True))
    st = _check(gpu_ctx, oracle_mod, frame, draws)
    assert st["tri_input"] > 4096


def test_lib_shards_compose(gpu_ctx):
    """Library pass with tile ownership (tile % count == rank) composes to the full frame."""
    from shs_gpu import scene_lib
    frame, draws, _, _, _ = scene_lib.c5_scene(320, 180)
    gpu_ctx.render_pbr_forward(frame, draws)
    fh, fd, fm = gpu_ctx.resolve_lib()
    T = 32
    oh, od = np.zeros_like(fh), np.zeros_like(fd)
    for rank in range(3):
        frame.shard_rank, frame.shard_count = rank, 3
        gpu_ctx.render_pbr_forward(frame, draws)
        h, d, m = gpu_ctx.resolve_lib()
        for ty in range((180 + T - 1) // T):
            for tx in range((320 + T - 1) // T):
                if (ty * ((320 + T - 1) // T) + tx) % 3 == rank:
                    sl = (slice(ty * T, ty * T + T), slice(tx * T, tx * T + T))
                    oh[sl], od[sl] = h[sl], d[sl]
    assert np.array_equal(oh.view(np.uint32), fh.view(np.uint32))
    assert np.array_equal(od.view(np.uint32), fd.view(np.uint32))


def test_back_to_back_frames_no_host_sync(gpu_ctx, oracle_mod):
    """Two shadow + camera frames enqueued without a host sync between them: the second camera pass's
    setup / raster run on the side stream beside its shadow pass and must wait only for the first
    frame's resolve; the resolved targets are the second frame's, exactly."""
    from shs_gpu import scene_lib
    frames = [scene_lib.c5_scene(352, 200, 256, yaw=y) for y in (0.0, 23.0)]
    for frame, draws, casters, sun, S in frames:        # no resolve in between
        lvp = gpu_ctx.render_shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)
        gpu_ctx.render_pbr_forward(frame, draws)
    gh, gd, gm = gpu_ctx.resolve_lib()
    frame, draws, casters, sun, S = frames[1]
    sm_ref, _ = oracle_mod.shadow_map(S, sun, casters)
    rh, rd, rm, _ = oracle_mod.pbr_forward(frame, draws, sm_ref)
    assert_depth_bitexact(gd, rd)
    assert_float_close(gm, rm, what="motion")
    assert_float_close(gh, rh, what="hdr")


def test_shallow_raster_after_first_frame(oracle_mod):
    """The first camera pass of a context runs the deep raster (1024-candidate rounds); once a pass's
    fullest bin tile is known to fit 256, the next uses the shallow one (more workgroups per CU).
    Both frames must equal the oracle, in a fresh context so the order is known."""
    import shs_gpu
    from shs_gpu import scene_lib
    frame, draws, casters, sun, S = scene_lib.c5_scene(2560, 1440, 512)   # fullest bin tile ~140
    sm_ref, _ = oracle_mod.shadow_map(S, sun, casters)
    with shs_gpu.Context(0) as ctx:
        lvp = ctx.render_shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)
        rh, rd, rm, _ = oracle_mod.pbr_forward(frame, draws, sm_ref)
        for _ in range(2):
            ctx.render_pbr_forward(frame, draws)
            gh, gd, gm = ctx.resolve_lib()
            assert ctx.lib_stats()["max_tile_bin"] <= 256
            assert_depth_bitexact(gd, rd)
            assert_float_close(gm, rm, what="motion")
            assert_float_close(gh, rh, what="hdr")


@pytest.mark.gpu
@pytest.mark.parametrize("part", [16, 64, 512])
def test_split_raster_items_exact(oracle_mod, part):
    """SHS_OPT_LIB_PART: busy tiles with more bin entries than `part` are rendered as spatial parts
    (32x4 halves / 16x4 blocks) on different workgroups -- the C4-like Forward+ frame (deep bins) must
    stay bit-identical to the oracle (depth) / within 1e-5 (HDR)."""
    import shs_gpu
    from shs_gpu import scene_lib
    from helpers import assert_depth_bitexact, assert_float_close
    frame, draws, lights, cull = scene_lib.c4_scene(640, 360, n_objects=80, tris_per_object=600)
    rc, ri = oracle_mod.light_cull(cull, lights)[:2]
    rh, rd, rm, _ = oracle_mod.forward_plus(frame, draws, lights, cull, (rc, ri))
    ctx = shs_gpu.Context(0)
    try:
        ctx.set_lib_part(part)
        ctx.upload_lights(lights)
        ctx.light_cull(cull)
        ctx.render_pbr_forward(frame, draws)
        gh, gd, gm = ctx.resolve_lib()
        assert_depth_bitexact(gd, rd)
        assert_float_close(gh, rh, what="split hdr")
        assert ctx.lib_stats()["covered_pixels"] == int((rd < 1.0).sum())
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("count", [2, 5, 8])
def test_shard_cull_prepass_identical(count):
    """SHS_OPT_SHARD_CULL: a tile-sharded camera pass with the positions-only pre-pass (the rank's
    triangles only) renders the same tiles and counts the same statistics as without it."""
    import shs_gpu
    from shs_gpu import scene_lib
    frame, draws, lights, cull = scene_lib.c4_scene(800, 450, n_objects=120, tris_per_object=400)
    res = {}
    for on in (True, False):
        ctx = shs_gpu.Context(0)
        try:
            ctx.set_shard_cull(on)
            ctx.upload_lights(lights)
            outs = []
            for r in range(count):
                frame.shard_rank, frame.shard_count = r, count
                cull.shard_rank, cull.shard_count = r, count
                ctx.light_cull(cull)
                ctx.render_pbr_forward(frame, draws)
                h, d, m = ctx.resolve_lib()
                ty, tx = np.mgrid[0:450, 0:800] // 32
                own = ((ty * 25 + tx) % count) == r
                outs.append((h[own].copy(), d[own].copy(), m[own].copy(), ctx.lib_stats()))
            res[on] = outs
        finally:
            ctx.close()
    frame.shard_rank, frame.shard_count = 0, 1
    for a, b in zip(res[True], res[False]):
        for x, y in zip(a[:3], b[:3]):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
        for k in ("tri_input", "tri_after_clip", "tri_raster", "covered_pixels"):
            assert a[3][k] == b[3][k], (k, a[3][k], b[3][k])


@pytest.mark.gpu
@pytest.mark.parametrize("part", [8, 300])
def test_split_parts_painter_and_regions(oracle_mod, part):
    """Candidate-range parts (k_lib_plan): without a depth target (the merge's min is over the inverted
    submission order: the last submitted fragment still wins), and under the region layout with two
    passes (the split tiles' key slots and counters are reset by each tile's last part)."""
    import shs_gpu
    from shs_gpu import scene_lib
    from shs_gpu.lib_path import LibFrame
    frame, draws, lights, cull = scene_lib.c4_scene(512, 288, n_objects=60, tris_per_object=500)
    rc, ri = oracle_mod.light_cull(cull, lights)[:2]
    ctx = shs_gpu.Context(0)
    try:
        ctx.set_lib_part(part)
        ctx.upload_lights(lights)
        ctx.light_cull(cull)
        pf = LibFrame(512, 288, depth_motion=False, bg_gradient=False, clear_hdr=(0.1, 0.2, 0.3, 1.0))
        rh, _, _, _ = oracle_mod.forward_plus(pf, draws, lights, cull, (rc, ri))
        ctx.render_pbr_forward(pf, draws)
        gh, _, _ = ctx.resolve_lib()
        assert_float_close(gh, rh, what="painter split hdr")
        rh, rd, rm, _ = oracle_mod.forward_plus(frame, draws, lights, cull, (rc, ri))
        ctx.set_shard_layout(True)
        for rank in (1, 2, 1):
            frame.shard_rank, frame.shard_count = rank, 3
            cull.shard_rank, cull.shard_count = rank, 3
            ctx.light_cull(cull)
            ctx.render_pbr_forward(frame, draws)
            h, d, m = ctx.resolve_lib()
            x0, y0, x1, y1 = ctx.shard_regions(3)[rank]
            own = np.zeros(d.shape, bool)
            own[y0 * 32:(y1 + 1) * 32, x0 * 32:(x1 + 1) * 32] = True
            assert_depth_bitexact(np.where(own, d, rd), rd)
            assert_float_close(np.where(own[..., None], h, rh), rh, what="region split hdr")
    finally:
        frame.shard_rank, frame.shard_count = 0, 1
        cull.shard_rank, cull.shard_count = 0, 1
        ctx.close()
