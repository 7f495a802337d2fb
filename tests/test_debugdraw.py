"""the software library's debug_draw colour + depth raster
(shs-renderer-lib/include/shs/sw_render/debug_draw.hpp:60-109 draw_filled_triangle, :147-203
draw_mesh_blinn_phong_transformed), GPU (shs_debug_fill_triangles / shs_debug_draw_meshes) against the
oracle restatement (oracle/shs_oracle_debugdraw.c).  Parity unpinned beyond the analytic cases here:
the reference ships no fixture for these functions and cannot be built (glm is absent).

Bar: depth bit-exact and the written pixels identical; draw_filled_triangle's colours exact (they are
the caller's); draw_mesh's colours exact except a byte may differ by 1 where the triangle's lit float
(before the byte conversion) agrees with the oracle's within 1e-5 (the specular pow(x, 32) is taken by
double squaring on the GPU, powf on the host)."""
import numpy as np
import pytest

from oracle import oracle
from helpers import TOL


def _u8(lit):
    return np.clip(lit.astype(np.float32) * np.float32(255.0), 0, 255).astype(np.uint8)


# ---- oracle known-answer tests (CPU) -------------------------------------------------------------

def test_fill_triangle_kat_coverage_and_depth():
    # right triangle (0,0) (8,0) (0,8): pixel centres with x + y + 1 <= 8 are inside (edges included)
    scr = np.array([[[0, 0], [8, 0], [0, 8]]], np.float32)
    rgba, depth = oracle.draw_filled_triangles(10, 10, scr, [[0.5, 0.5, 0.5]], [[10, 20, 30, 255]])
    ys, xs = np.mgrid[0:10, 0:10]
    inside = (xs + 0.5) + (ys + 0.5) <= 8.0
    assert np.array_equal(depth < 1.0, inside)
    assert np.all(depth[inside] == np.float32(0.5))
    assert np.all(rgba[inside] == [10, 20, 30, 255]) and np.all(rgba[~inside] == 0)
    # the opposite winding covers the same pixels (draw_filled_triangle accepts both, :91-92)
    rgba2, depth2 = oracle.draw_filled_triangles(10, 10, scr[:, ::-1], [[0.5, 0.5, 0.5]], [[10, 20, 30, 255]])
    assert np.array_equal(depth2, depth) and np.array_equal(rgba2, rgba)


def test_fill_triangle_kat_order_range_and_degenerate():
    scr = np.array([[[0, 0], [8, 0], [0, 8]]] * 2, np.float32)
    # equal depth: the first triangle keeps the pixel (strict <, :102)
    rgba, _ = oracle.draw_filled_triangles(10, 10, scr, [[0.25] * 3, [0.25] * 3], [[1, 1, 1, 255], [2, 2, 2, 255]])
    assert rgba[0, 0, 0] == 1
    # nearer second triangle wins; depth outside [0, 1] is skipped (:99)
    rgba, depth = oracle.draw_filled_triangles(10, 10, scr, [[0.25] * 3, [0.125] * 3], [[1, 1, 1, 255], [2, 2, 2, 255]])
    assert rgba[0, 0, 0] == 2 and depth[0, 0] == np.float32(0.125)
    rgba, depth = oracle.draw_filled_triangles(10, 10, scr[:1], [[-0.5] * 3], [[1, 1, 1, 255]])
    assert np.all(depth == 1.0) and not rgba.any()
    # |area| <= 1e-6: nothing
    deg = np.array([[[0, 0], [4, 4], [8, 8]]], np.float32)
    rgba, depth = oracle.draw_filled_triangles(10, 10, deg, [[0.1] * 3], [[1, 1, 1, 255]])
    assert np.all(depth == 1.0)


def test_draw_mesh_kat_flat_blinn_phong():
    """One triangle facing the camera at z = 5 under a head-on light: n = (0, 0, -1), L = V = H ~ -z, so
    ndotl ~ ndoth ~ 1 and lit = base * (0.18 + 0.72) + 0.35 (clamped)."""
    from shs_gpu.lib_path import LibMesh
    from shs_gpu.scene_lib import look_at_lh, perspective_lh_no, mat_mul
    # clockwise front face seen from -z (LH): the reference's cross(p2 - p0, p1 - p0) points at the camera
    mesh = LibMesh(positions=np.array([[-1, -1, 0], [-1, 1, 0], [1, -1, 0]], np.float32),
                   indices=np.array([0, 2, 1], np.uint32))
    model = np.eye(4, dtype=np.float32).reshape(-1)
    model[14] = 5.0
    view = look_at_lh((0.0, 0.0, -5.0), (0.0, 0.0, 5.0))
    proj = perspective_lh_no(np.float32(np.deg2rad(60.0)), np.float32(1.0), np.float32(0.1), np.float32(100.0))
    vp = mat_mul(proj, view)
    base = (0.25, 0.5, 0.0)
    rgba, depth, lit = oracle.debug_draw_meshes(64, 64, vp, (0.0, 0.0, -5.0), (0.0, 0.0, 1.0), [(mesh, model, base)])
    assert lit[0, 3] == 1.0
    # n = L = (0, 0, -1): n.L = 1; the centroid (-1/3, -1/3, 5) is off axis, so n.H is just below 1
    v = np.array([0.0, 0.0, -5.0]) - np.array([-1 / 3, -1 / 3, 5.0])
    h = np.array([0.0, 0.0, -1.0]) + v / np.linalg.norm(v)
    spec = 0.35 * (-h[2] / np.linalg.norm(h)) ** 32
    want = np.minimum(np.array(base) * 0.9 + spec, 1.0)
    assert np.allclose(lit[0, :3], want, atol=1e-5)
    assert (depth < 1.0).sum() > 40
    assert np.all(rgba[depth < 1.0][:, :3] == _u8(lit[0, :3]))


# ---- GPU parity ----------------------------------------------------------------------------------

def _random_triangles(rng, n, W, H):
    c = rng.uniform([-0.2 * W, -0.2 * H], [1.2 * W, 1.2 * H], size=(n, 1, 2))
    r = rng.uniform(2, 0.25 * min(W, H), size=(n, 1, 1))
    scr = (c + r * rng.uniform(-1, 1, size=(n, 3, 2))).astype(np.float32)
    z = rng.uniform(-0.1, 1.1, size=(n, 3)).astype(np.float32)
    z[::7] = z[::7, :1]                                  # flat triangles: exact depth ties across triangles
    z[::11] = np.float32(0.5)
    z[5::13, :] = np.float32(-0.0)                       # depth -0 (kept, stored with its sign)
    scr[3::17, 2] = scr[3::17, 0]                        # degenerate (area 0)
    scr[4::19] = np.round(scr[4::19])                    # pixel-aligned edges: exact edge-function zeros
    col = rng.integers(0, 256, size=(n, 4), dtype=np.uint8)
    return scr, z, col


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,n,seed", [(64, 48, 40, 1), (300, 225, 600, 2), (1200, 900, 3000, 3)])
def test_fill_triangles_bitexact(W, H, n, seed):
    import shs_gpu
    rng = np.random.default_rng(seed)
    scr, z, col = _random_triangles(rng, n, W, H)
    rgba0 = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    depth0 = rng.uniform(0.0, 1.2, size=(H, W)).astype(np.float32)
    depth0[::5, ::3] = 1.0
    want_c, want_d = oracle.draw_filled_triangles(W, H, scr, z, col, rgba0, depth0)
    ctx = shs_gpu.Context(0)
    try:
        got_c, got_d = ctx.debug_fill_triangles(W, H, scr, z, col, rgba0.copy(), depth0.copy())
        assert np.array_equal(got_d.view(np.uint32), want_d.view(np.uint32))
        assert np.array_equal(got_c, want_c)
        # empty list: the buffers come back untouched
        c2, d2 = ctx.debug_fill_triangles(W, H, np.zeros((0, 3, 2), np.float32), np.zeros((0, 3), np.float32),
                                          np.zeros((0, 4), np.uint8), rgba0.copy(), depth0.copy())
        assert np.array_equal(c2, rgba0) and np.array_equal(d2.view(np.uint32), depth0.view(np.uint32))
    finally:
        ctx.close()


def _check_meshes(ctx, W, H, vp, cam, light, meshes, rgba0=None, depth0=None):
    want_c, want_d, want_l = oracle.debug_draw_meshes(W, H, vp, cam, light, meshes, rgba0, depth0)
    got_c, got_d, got_l = ctx.debug_draw_meshes(W, H, vp, cam, light, meshes,
                                                None if rgba0 is None else rgba0.copy(),
                                                None if depth0 is None else depth0.copy(), tri_lit=True)
    bad = np.flatnonzero(got_l[:, 3] != want_l[:, 3])
    assert bad.size == 0, (f"{bad.size} area flags differ, first {bad[:8].tolist()} of {len(got_l)}: "
                           f"gpu {got_l[bad[:4]].tolist()} oracle {want_l[bad[:4]].tolist()}")
    assert np.abs(got_l[:, :3] - want_l[:, :3]).max(initial=0.0) <= TOL
    assert np.array_equal(got_d.view(np.uint32), want_d.view(np.uint32))
    diff = got_c.astype(np.int16) - want_c.astype(np.int16)
    if diff.any():
        assert np.abs(diff).max() <= 1
        assert (_u8(got_l[:, :3]) != _u8(want_l[:, :3])).any(), "byte differences without a lit-float split"
    return int((diff != 0).sum()), int((got_d < 1.0).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("n_objects,W,H", [(60, 300, 225), (300, 300, 225), (2000, 1200, 900)])
def test_draw_meshes_parity(n_objects, W, H):
    """The lit-surface draw of hello_occlusion_culling_sw.cpp:387-407 over random boxes and spheres,
    walls and objects behind the camera (skipped per triangle by project_world_to_screen)."""
    import shs_gpu
    from shs_gpu import scene_lib
    objs, view, vp, W, H = scene_lib.occlusion_scene(n_objects=n_objects, width=W, height=H)
    rng = np.random.default_rng(n_objects)
    meshes = [(o[0], o[1], rng.uniform(0.0, 1.2, 3).astype(np.float32)) for o in objs]
    ctx = shs_gpu.Context(0)
    try:
        n_diff, n_cov = _check_meshes(ctx, W, H, vp, (0.0, 3.0, -4.0), (-0.4, -1.0, 0.3), meshes)
        assert n_cov > W * H // 10
    finally:
        ctx.close()


@pytest.mark.gpu
def test_draw_meshes_into_existing_buffers():
    """In place: a second draw over the canvas and depth a first one left (the demo clears once per
    frame and then draws every visible instance into the same buffers)."""
    import shs_gpu
    from shs_gpu import scene_lib
    objs, view, vp, W, H = scene_lib.occlusion_scene(n_objects=120, width=320, height=240, seed=11)
    meshes = [(o[0], o[1], (0.8, 0.4, 0.2)) for o in objs]
    rgba0 = np.zeros((H, W, 4), np.uint8)
    rgba0[...] = (12, 13, 18, 255)
    rng = np.random.default_rng(5)
    depth0 = rng.uniform(0.9, 1.0, size=(H, W)).astype(np.float32)
    ctx = shs_gpu.Context(0)
    try:
        _check_meshes(ctx, W, H, vp, (0.0, 3.0, -4.0), (0.3, -1.0, 0.2), meshes[:60], rgba0, depth0)
        c1, d1, _ = oracle.debug_draw_meshes(W, H, vp, (0.0, 3.0, -4.0), (0.3, -1.0, 0.2), meshes[:60], rgba0, depth0)
        _check_meshes(ctx, W, H, vp, (0.0, 3.0, -4.0), (0.3, -1.0, 0.2), meshes[60:], c1, d1)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_fill_and_draw_resize_sequence():
    """One context through canvas sizes down to 1x1 and single rows / columns: the filled-triangle
    raster and the lit mesh draw, each vs the oracle."""
    import shs_gpu
    from shs_gpu import scene_lib
    ctx = shs_gpu.Context(0)
    try:
        for seed, (W, H) in enumerate([(64, 48), (64, 40), (1, 1), (1, 29), (45, 1), (64, 48)]):
            rng = np.random.default_rng(100 + seed)
            scr, z, col = _random_triangles(rng, 60, max(W, 16), max(H, 16))
            rgba0 = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
            depth0 = rng.uniform(0.0, 1.2, size=(H, W)).astype(np.float32)
            want_c, want_d = oracle.draw_filled_triangles(W, H, scr, z, col, rgba0, depth0)
            got_c, got_d = ctx.debug_fill_triangles(W, H, scr, z, col, rgba0.copy(), depth0.copy())
            assert np.array_equal(got_d.view(np.uint32), want_d.view(np.uint32)), (W, H)
            assert np.array_equal(got_c, want_c), (W, H)
            objs, view, vp, _, _ = scene_lib.occlusion_scene(n_objects=40, width=W, height=H, seed=seed)
            meshes = [(o[0], o[1], (0.7, 0.5, 0.3)) for o in objs]
            _check_meshes(ctx, W, H, vp, (0.0, 3.0, -4.0), (-0.4, -1.0, 0.3), meshes)
    finally:
        ctx.close()
