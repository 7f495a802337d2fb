"""GPU parity: the HIP path through the C ABI vs the CPU oracle, on the same seeded inputs.

Coverage and depth: bit-exact.  Colour: exact, except a byte may differ by 1 where both shaders'
pre-truncation floats agree within 1e-5 (per channel, [0,1] scale).
"""
import numpy as np
import pytest

from helpers import FLT_MAX, assert_color_parity, assert_depth_bitexact

pytestmark = pytest.mark.gpu

SHADINGS = [0, 1, 2, 3]


def _render_both(ctx, oracle_mod, frame, draws, threads=8):
    frame.prequant = True
    ctx.render(frame, draws)
    gc, gd = ctx.resolve()
    gpq = ctx.resolve_prequant()
    stats = ctx.stats()
    rc, rd, rpq = oracle_mod.render_legacy(frame.width, frame.height, draws, tile=frame.ref_tile,
                                           threads=threads, prequant=True)
    return gc, gd, gpq, rc, rd, rpq, stats


def _check(ctx, oracle_mod, frame, draws):
    gc, gd, gpq, rc, rd, rpq, stats = _render_both(ctx, oracle_mod, frame, draws)
    assert_depth_bitexact(gd, rd)
    nbad = assert_color_parity(gc, rc, gpq, rpq)
    assert stats["covered_pixels"] == int((rd < FLT_MAX).sum())
    return stats, nbad


@pytest.mark.parametrize("cfg", ["c1", "c2"])
def test_config_blinn_phong(gpu_ctx, oracle_mod, cfg):
    from shs_gpu import scene
    frame, draws = scene.config(cfg)
    stats, nbad = _check(gpu_ctx, oracle_mod, frame, draws)
    assert stats["tri_input"] == 967
    assert stats["covered_pixels"] > 10000


@pytest.mark.parametrize("shading", SHADINGS)
@pytest.mark.parametrize("yaw,pitch", [(0.0, 0.0), (17.0, -9.0), (-33.0, 12.5)])
def test_shading_models_camera_sweep(gpu_ctx, oracle_mod, shading, yaw, pitch):
    from shs_gpu import scene
    frame, draws = scene.monkey_scene(640, 480, shading, yaw=yaw, pitch=pitch, rotation=23.0 * shading,
                                      cam_pos=(0.0, 5.0, -12.0))
    _check(gpu_ctx, oracle_mod, frame, draws)


def test_config3_grid_phong(gpu_ctx, oracle_mod):
    from shs_gpu import scene
    frame, draws = scene.config("c3")
    stats, _ = _check(gpu_ctx, oracle_mod, frame, draws)
    assert stats["tri_input"] == 64 * 967


def _ndc_soup(rng, W, H, n, kind="mixed", zq=None):
    """Random triangle soup given in pixel space, returned as NDC positions for an identity MVP."""
    tris = []
    for _ in range(n):
        t = rng.choice(["small", "sliver", "big", "off", "degen"], p=[0.55, 0.2, 0.1, 0.1, 0.05]) if kind == "mixed" else kind
        c = rng.uniform([-20, -20], [W + 20, H + 20])
        if t == "small":
            p = c + rng.uniform(-25, 25, size=(3, 2))
        elif t == "sliver":
            d = rng.normal(size=2); d /= np.linalg.norm(d)
            L = rng.uniform(10, 300)
            nrm = np.array([-d[1], d[0]])
            p = np.stack([c, c + d * L, c + d * L * rng.uniform(0.2, 0.8) + nrm * rng.uniform(-0.3, 0.3)])
        elif t == "big":
            p = c + rng.uniform(-400, 400, size=(3, 2))
        elif t == "off":
            p = c + np.array([rng.choice([-1, 1]) * (W + 200), 0]) + rng.uniform(-30, 30, size=(3, 2))
        else:
            d = rng.normal(size=2)
            p = np.stack([c, c + d * 5, c + d * 11])
        if zq is not None:
            z = np.full(3, rng.choice(zq))
        else:
            z = rng.uniform(-0.9, 0.9, size=3)
        x = p[:, 0] / (0.5 * (W - 1)) - 1.0
        y = 1.0 - p[:, 1] / (0.5 * (H - 1))
        tris.append(np.stack([x, y, z], axis=1).reshape(9))
    pos = np.asarray(tris, dtype=np.float32)
    nrm = rng.normal(size=pos.shape).astype(np.float32)
    return pos, nrm


def _identity_draw(mesh, shading=3, color=(200, 120, 40, 255)):
    import shs_gpu
    eye = np.eye(4, dtype=np.float32).reshape(16)
    return shs_gpu.Draw(mesh, shading, eye, eye, np.array([-0.3, -0.5, 0.8], np.float32),
                        np.array([0.0, 0.0, -3.0], np.float32), color)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_soup_exact(gpu_ctx, oracle_mod, seed):
    """Slivers, huge, off-screen, degenerate and overlapping triangles; 80x80 reference tiles that
    32x32 GPU tiles straddle; ragged frame size."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    rng = np.random.default_rng(seed)
    W, H = 333, 241
    pos, nrm = _ndc_soup(rng, W, H, 1500)
    mesh = Mesh(pos, nrm)
    frame = shs_gpu.Frame(W, H)
    stats, _ = _check(gpu_ctx, oracle_mod, frame, [_identity_draw(mesh, shading=seed % 4)])
    assert stats["tri_setup"] > 100


def test_z_ties_first_wins(gpu_ctx, oracle_mod):
    """Quantised z -> many exact ties; the reference keeps the first triangle in submission order
    (strict '<', shs_renderer.hpp:664), across two draws."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    rng = np.random.default_rng(7)
    W, H = 256, 192
    pos, nrm = _ndc_soup(rng, W, H, 800, kind="small", zq=[0.25, 0.5, -0.0, 0.0])
    m1, m2 = Mesh(pos[:400], nrm[:400]), Mesh(pos[400:], nrm[400:])
    frame = shs_gpu.Frame(W, H)
    _check(gpu_ctx, oracle_mod, frame, [_identity_draw(m1, 3, (255, 0, 0, 255)), _identity_draw(m2, 3, (0, 255, 0, 255))])


def test_slivers_ghost_path(gpu_ctx, oracle_mod):
    """Only slivers: exercises the exact tile-clamp ("ghost") visited-set pass."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    rng = np.random.default_rng(11)
    W, H = 400, 300
    pos, nrm = _ndc_soup(rng, W, H, 600, kind="sliver")
    frame = shs_gpu.Frame(W, H)
    stats, _ = _check(gpu_ctx, oracle_mod, frame, [_identity_draw(Mesh(pos, nrm), 0)])
    assert stats["tri_ghost"] > 0


def test_odd_reference_tiles(gpu_ctx, oracle_mod):
    import shs_gpu
    from shs_gpu.scene import Mesh
    rng = np.random.default_rng(5)
    W, H = 301, 207
    pos, nrm = _ndc_soup(rng, W, H, 700)
    frame = shs_gpu.Frame(W, H, ref_tile=(37, 53))
    _check(gpu_ctx, oracle_mod, frame, [_identity_draw(Mesh(pos, nrm), 2)])


@pytest.mark.parametrize("W,H", [(1, 1), (1, 37), (45, 1), (2, 2), (31, 33), (81, 79)])
def test_tiny_and_ragged_frames(gpu_ctx, oracle_mod, W, H):
    """Frames smaller than one 32x32 GPU tile / one 80x80 reference tile, single rows and columns,
    and sizes one pixel either side of a tile edge: the edge clamps of both tilings."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    rng = np.random.default_rng(W * 131 + H)
    pos, nrm = _ndc_soup(rng, max(W, 8), max(H, 8), 300)
    frame = shs_gpu.Frame(W, H)
    _check(gpu_ctx, oracle_mod, frame, [_identity_draw(Mesh(pos, nrm), (W + H) % 4)])


def test_resize_sequence(gpu_ctx, oracle_mod):
    """One context through sizes that keep or change the 32x32 bin-tile grid and the raster-tile
    rows (the busy flags and per-slot workspaces are cached per geometry): every frame vs the oracle."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    rng = np.random.default_rng(23)
    for W, H in [(160, 96), (160, 90), (150, 90), (33, 17), (160, 96), (160, 96)]:
        pos, nrm = _ndc_soup(rng, W, H, 250)
        _check(gpu_ctx, oracle_mod, shs_gpu.Frame(W, H), [_identity_draw(Mesh(pos, nrm), H % 4)])


@pytest.mark.parametrize("cam_z", [6.5, 8.0, 9.5])
def test_vertices_behind_camera(gpu_ctx, oracle_mod, cam_z):
    """Camera inside / just in front of the Suzanne: vertices with clip w < 0 and triangles straddling
    the camera plane.  The legacy pipelines divide by w without clipping (Canvas::clip_to_screen,
    shs_renderer.hpp:823-831) and clamp the bbox to the tile in float (draw_triangle_tile): the GPU
    must reproduce the same flipped, huge-coordinate triangles."""
    from shs_gpu import scene
    frame, draws = scene.monkey_scene(320, 240, 3, rotation=31.0, cam_pos=(0.3, 0.4, cam_z))
    stats, _ = _check(gpu_ctx, oracle_mod, frame, draws)
    assert stats["covered_pixels"] > 0


def test_empty_frame_clears(gpu_ctx):
    import shs_gpu
    frame = shs_gpu.Frame(100, 70, clear_color=(1, 2, 3, 255))
    gpu_ctx.render(frame, [])
    c, d = gpu_ctx.resolve()
    assert (c == np.array([1, 2, 3, 255], np.uint8)).all()
    assert (d == FLT_MAX).all()


def test_shards_compose_to_full_frame(gpu_ctx):
    """Tile ownership (tile % count == rank): the union of the shards' owned tiles is the full frame."""
    import shs_gpu
    from shs_gpu import scene
    frame, draws = scene.monkey_scene(640, 480, 3, cam_pos=(0.0, 5.0, -12.0))
    gpu_ctx.render(frame, draws)
    full_c, full_d = gpu_ctx.resolve()
    out_c = np.zeros_like(full_c)
    out_d = np.zeros_like(full_d)
    T = shs_gpu.lib().shs_gpu_tile_size()
    tx = (frame.width + T - 1) // T
    for rank in range(3):
        f = shs_gpu.Frame(640, 480, shard_rank=rank, shard_count=3)
        gpu_ctx.render(f, draws)
        c, d = gpu_ctx.resolve()
        for ty in range((480 + T - 1) // T):
            for txi in range(tx):
                if (ty * tx + txi) % 3 != rank:
                    continue
                ys, xs = slice(ty * T, min(ty * T + T, 480)), slice(txi * T, min(txi * T + T, 640))
                out_d[ys, xs] = d[ys, xs]
                cys = slice(480 - min(ty * T + T, 480), 480 - ty * T)
                out_c[cys, xs] = c[cys, xs]
    assert np.array_equal(out_c, full_c)
    assert np.array_equal(out_d.view(np.uint32), full_d.view(np.uint32))


def test_4k_full_frame_properties(gpu_ctx):
    """At 3840x2160 (beyond what the oracle is run at in this suite): every pixel is either the clear
    value or a finite depth and opaque colour, and the frame hash is deterministic across runs."""
    from shs_gpu import scene
    frame, draws = scene.grid_scene(3840, 2160)
    gpu_ctx.render(frame, draws)
    c1, d1 = gpu_ctx.resolve()
    gpu_ctx.render(frame, draws)
    c2, d2 = gpu_ctx.resolve()
    assert np.array_equal(c1, c2) and np.array_equal(d1.view(np.uint32), d2.view(np.uint32))
    cov = d1 < FLT_MAX
    assert cov.sum() > 100000
    assert np.isfinite(d1[cov]).all()
    assert (c1[..., 3] == 255).all()


def test_bin_spill_path_exact(gpu_ctx, oracle_mod):
    """Tiny per-tile bin capacity: most entries spill to the global list; results stay exact."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    rng = np.random.default_rng(23)
    W, H = 200, 160
    pos, nrm = _ndc_soup(rng, W, H, 600)
    ctx = shs_gpu.Context(0)
    try:
        ctx.set_raster_mode(2)      # bins (this scene would auto-select scan mode)
        ctx.set_bin_capacity(2)
        frame = shs_gpu.Frame(W, H)
        stats, _ = _check(ctx, oracle_mod, frame, [_identity_draw(Mesh(pos, nrm), 3)])
        assert stats["spilled"] > 0
    finally:
        ctx.close()


def test_many_draws_device_table(gpu_ctx, oracle_mod):
    """More draws than fit in kernel arguments -> the uniform table is uploaded to HBM."""
    from shs_gpu import scene
    frame, draws = scene.grid_scene(480, 360, n=3, shading=3)
    assert len(draws) > 6
    _check(gpu_ctx, oracle_mod, frame, draws)


def _hair_soup(rng, W, H, n):
    """Extremely thin slivers (third vertex within 0.02 px of the long edge): their float
    barycentrics can pass at pixels outside their own bbox, which the reference only tests where its
    80x80 tile clamp visits them."""
    tris = []
    for _ in range(n):
        c = rng.uniform([0, 0], [W, H])
        d = rng.normal(size=2); d /= np.linalg.norm(d)
        L = rng.uniform(20, 400)
        nrm = np.array([-d[1], d[0]])
        p = np.stack([c, c + d * L, c + d * L * rng.uniform(0.05, 0.95) + nrm * rng.uniform(-0.02, 0.02)])
        z = rng.uniform(-0.9, 0.9, size=3)
        x = p[:, 0] / (0.5 * (W - 1)) - 1.0
        y = 1.0 - p[:, 1] / (0.5 * (H - 1))
        tris.append(np.stack([x, y, z], axis=1).reshape(9))
    pos = np.asarray(tris, dtype=np.float32)
    return pos, rng.normal(size=pos.shape).astype(np.float32)


def test_hair_slivers_tile_clamp_ghosts(gpu_ctx, oracle_mod):
    """The reference's tile clamp changes the image for these slivers (ghost pixels exist: the oracle's
    80x80-tile render differs from its single-tile render); the GPU matches both bit-exactly."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    rng = np.random.default_rng(99)
    W, H = 400, 300
    pos, nrm = _hair_soup(rng, W, H, 3000)
    draw = _identity_draw(Mesh(pos, nrm), 3)
    c80, d80, _ = oracle_mod.render_legacy(W, H, [draw], tile=(80, 80), threads=8)
    c1, d1, _ = oracle_mod.render_legacy(W, H, [draw], tile=(W, H), threads=8)
    assert not np.array_equal(d80.view(np.uint32), d1.view(np.uint32)), "scene has no tile-clamp ghost pixels"
    stats, _ = _check(gpu_ctx, oracle_mod, shs_gpu.Frame(W, H, ref_tile=(80, 80)), [draw])
    assert stats["tri_ghost_unbounded"] > 0
    _check(gpu_ctx, oracle_mod, shs_gpu.Frame(W, H, ref_tile=(W, H)), [draw])


@pytest.fixture(scope="module", params=[(1, 0), (2, 0), (1, 1), (2, 1)],
                ids=["scan-pixel", "bins-pixel", "scan-pairs", "bins-pairs"])
def mode_ctx(request):
    import shs_gpu
    ctx = shs_gpu.Context(0)
    ctx.set_raster_mode(request.param[0])
    ctx.set_raster_loop(request.param[1])
    yield ctx
    ctx.close()


@pytest.mark.parametrize("what", ["c1", "c3", "soup", "hair", "ties"])
def test_both_raster_modes_exact(mode_ctx, oracle_mod, what):
    """Scan mode (every tile scans all bin boxes) and bin mode (per-tile bins, spill, unbounded list)
    give identical, oracle-exact frames."""
    import shs_gpu
    from shs_gpu import scene
    from shs_gpu.scene import Mesh
    if what in ("c1", "c3"):
        frame, draws = scene.config(what)
    elif what == "soup":
        rng = np.random.default_rng(31)
        pos, nrm = _ndc_soup(rng, 333, 241, 1500)
        frame, draws = shs_gpu.Frame(333, 241), [_identity_draw(Mesh(pos, nrm), 2)]
    elif what == "hair":
        rng = np.random.default_rng(99)
        pos, nrm = _hair_soup(rng, 400, 300, 3000)
        frame, draws = shs_gpu.Frame(400, 300), [_identity_draw(Mesh(pos, nrm), 3)]
    else:
        rng = np.random.default_rng(8)
        pos, nrm = _ndc_soup(rng, 256, 192, 800, kind="small", zq=[0.25, 0.5, -0.0, 0.0])
        frame, draws = shs_gpu.Frame(256, 192), [_identity_draw(Mesh(pos, nrm), 1)]
    _check(mode_ctx, oracle_mod, frame, draws)


def test_counters_reset_across_empty_frame(gpu_ctx, oracle_mod):
    """Per-frame counters (ghost fragments, spill, overflow) are zeroed even when a frame has no
    triangles: hair-sliver frame (ghost fragments emitted) -> empty frame -> C1 must match the oracle."""
    import shs_gpu
    from shs_gpu import scene
    from shs_gpu.scene import Mesh
    rng = np.random.default_rng(99)
    pos, nrm = _hair_soup(rng, 400, 300, 3000)
    gpu_ctx.render(shs_gpu.Frame(400, 300), [_identity_draw(Mesh(pos, nrm), 3)])
    gpu_ctx.resolve()
    assert gpu_ctx.stats()["tri_ghost_unbounded"] > 0
    gpu_ctx.render(shs_gpu.Frame(64, 64), [])
    gpu_ctx.resolve()
    frame, draws = scene.config("c1")
    _check(gpu_ctx, oracle_mod, frame, draws)
