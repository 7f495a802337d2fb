"""CPU known-answer tests of the library-path oracle (oracle/shs_oracle_lib.c) and of the host GLM
helpers the C ABI uses for it.  The reference ships no golden vectors for this path:
these analytic cases follow rasterizer.hpp / builtin_shaders.hpp / pass_shadow_map.hpp line by line,
and tests/golden/lib_golden.json pins the oracle's own output on the C5-small scene."""
import ctypes
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lib_golden.json")
f32 = np.float32


def _tri_mesh(ndc_tris):
    from shs_gpu.lib_path import LibMesh
    pos = np.asarray(ndc_tris, np.float32).reshape(-1, 3)
    return LibMesh(pos, np.tile(np.array([0, 0, -1], np.float32), (pos.shape[0], 1)))


def _draw(mesh, **kw):
    from shs_gpu.lib_path import LibDraw
    kw.setdefault("cull_mode", 0)
    kw.setdefault("program", 2)
    return LibDraw(mesh=mesh, **kw)


def test_identity_triangle_coverage_and_ndc_depth(oracle_mod):
    """Identity viewproj: clip = world, w = 1.  No depth target -> z01 is NDC-based but unused; with a
    target and zf <= zn + 1e-6 the NDC depth z*0.5+0.5 is stored (rasterizer.hpp:347-356)."""
    from shs_gpu.lib_path import LibFrame
    tri = [(-0.5, -0.5, 0.2), (0.5, -0.5, 0.2), (0.0, 0.5, 0.2)]
    W, H = 65, 49
    hdr, d, m, st = oracle_mod.pbr_forward(LibFrame(W, H, zn=1.0, zf=1.0), [_draw(_tri_mesh(tri))])
    assert st == {"tri_input": 1, "tri_after_clip": 1, "tri_raster": 1}
    cov = d < 1.0
    assert np.all(d[cov] == f32(0.2) * f32(0.5) + f32(0.5))
    # NDC area 0.5 (base 1, height 1) scaled by (W-1)/2 x (H-1)/2 pixels per NDC unit
    expect = 0.5 * (0.5 * (W - 1)) * (0.5 * (H - 1))
    assert abs(int(cov.sum()) - expect) < 0.15 * expect
    # rows are y-up: the apex (ndc y = +0.5) is near the top row index
    ys = np.nonzero(cov.any(axis=1))[0]
    assert ys.min() < H // 2 < ys.max()
    assert np.all(hdr[cov][:, :3] == np.array([1.0, 1.0, 1.0], np.float32))   # debug albedo = base_color


def test_linear_view_depth():
    """w = 4 everywhere -> view_z = 1/denom = 4 (up to the rounding of u + v + w), z01 = (4 - zn) / (zf - zn)."""
    from oracle import oracle
    from shs_gpu.lib_path import LibFrame
    w = 4.0
    tri = [(-0.5 * w, -0.5 * w, 0.0), (0.5 * w, -0.5 * w, 0.0), (0.0, 0.5 * w, 0.0)]
    P = np.zeros(16, np.float32)   # x, y, z passthrough, w = 4 (constant)
    P[0] = P[5] = P[10] = 1.0
    P[15] = w
    _, d, _, _ = oracle.pbr_forward(LibFrame(40, 30, zn=0.5, zf=10.0), [_draw(_tri_mesh(tri), viewproj=P)])
    cov = d < 1.0
    assert cov.sum() > 50
    assert np.allclose(d[cov], (4.0 - 0.5) / (10.0 - 0.5), rtol=1e-6, atol=0)


@pytest.mark.parametrize("cull,ccw,flip,visible", [(1, True, False, True), (1, True, True, False), (2, True, False, False),
                                                    (2, True, True, True), (1, False, False, False), (0, True, True, True)])
def test_cull_modes(oracle_mod, cull, ccw, flip, visible):
    """RasterizerCullMode + front_face_ccw on the screen-space signed area (rasterizer.hpp:271-278);
    screen rows are y-up, so NDC winding is screen winding."""
    from shs_gpu.lib_path import LibFrame
    tri = [(-0.5, -0.5, 0.0), (0.5, -0.5, 0.0), (0.0, 0.5, 0.0)]   # CCW
    if flip:
        tri = [tri[0], tri[2], tri[1]]
    _, d, _, st = oracle_mod.pbr_forward(LibFrame(32, 32), [_draw(_tri_mesh(tri), cull_mode=cull, front_face_ccw=ccw)])
    assert st["tri_raster"] == (1 if visible else 0)
    assert bool((d < 1).any()) == visible


def test_near_plane_clip_fans(oracle_mod):
    """One corner behind the near plane (z < -w): Sutherland-Hodgman yields a quad -> 2 fan triangles."""
    from shs_gpu.lib_path import LibFrame
    tri = [(-0.5, -0.5, 0.0), (0.5, -0.5, 0.0), (0.0, 0.5, -3.0)]
    _, d, _, st = oracle_mod.pbr_forward(LibFrame(48, 48, zn=1.0, zf=1.0), [_draw(_tri_mesh(tri))])
    assert st["tri_after_clip"] == 2 and st["tri_raster"] == 2
    cov = d < 1.0
    assert cov.sum() > 0 and np.all(d[cov] >= 0.0)


def test_fully_outside_is_dropped(oracle_mod):
    from shs_gpu.lib_path import LibFrame
    tri = [(2.0, 2.0, 0.0), (3.0, 2.0, 0.0), (2.5, 3.0, 0.0)]
    _, d, _, st = oracle_mod.pbr_forward(LibFrame(16, 16), [_draw(_tri_mesh(tri))])
    assert st == {"tri_input": 1, "tri_after_clip": 0, "tri_raster": 0}
    assert (d == 1.0).all()


def test_depth_first_wins_and_painter_last_wins(oracle_mod):
    """Equal depth: strict '<' keeps the first triangle; without a depth target the last one is painted."""
    from shs_gpu.lib_path import LibFrame
    tri = [(-0.8, -0.8, 0.1), (0.8, -0.8, 0.1), (0.0, 0.8, 0.1)]
    a = _draw(_tri_mesh(tri), base_color=(1.0, 0.0, 0.0))
    b = _draw(_tri_mesh(tri), base_color=(0.0, 1.0, 0.0))
    hdr, d, _, _ = oracle_mod.pbr_forward(LibFrame(32, 32), [a, b])
    cov = d < 1
    assert np.all(hdr[cov][:, 0] == 1.0) and np.all(hdr[cov][:, 1] == 0.0)
    hdr2, _, _, _ = oracle_mod.pbr_forward(LibFrame(32, 32, depth_motion=False), [a, b])
    assert np.all(hdr2[cov][:, 1] == 1.0) and np.all(hdr2[cov][:, 0] == 0.0)


def test_background_gradient(oracle_mod):
    """PassPBRForward's no-sky background (pass_pbr_forward.hpp:71-84), row y = bottom-up index."""
    from shs_gpu.lib_path import LibFrame
    hdr, _, _, _ = oracle_mod.pbr_forward(LibFrame(8, 5), [])
    for y in range(5):
        t = f32(y) / f32(4)
        assert hdr[y, 3, 0] == f32(0.06) + f32(0.08) * t and hdr[y, 3, 2] == f32(0.12) + f32(0.12) * t


def test_shadow_map_flat_quad(oracle_mod):
    """Sun straight down (|dir.y| > 0.95 -> up = +z): an orthographic light camera sees the quad at one
    constant depth; everything else stays at the clear value 1."""
    from shs_gpu.lib_path import LibMesh, ShadowCaster
    pos = np.array([[-1, 0, -1], [1, 0, -1], [1, 0, 1], [-1, 0, -1], [1, 0, 1], [-1, 0, 1]], np.float32)
    caster = ShadowCaster(LibMesh(pos), np.eye(4, dtype=np.float32).reshape(16))
    sm, vp = oracle_mod.shadow_map(64, (0.0, -1.0, 0.0), [caster])
    inside = sm < 1.0
    assert 0 < inside.sum() < 64 * 64
    assert len(np.unique(sm[inside])) <= 2   # a plane at constant light depth (up to one rounding)


def test_light_camera_host_matches_oracle(oracle_mod):
    """build_dir_light_camera_aabb: the C-ABI host helper (product) and the oracle's independent
    restatement agree bit-for-bit."""
    from shs_gpu.lib_path import dir_light_camera_aabb
    rng = np.random.default_rng(4)
    for _ in range(50):
        sun = rng.normal(size=3).astype(np.float32)
        if rng.random() < 0.2:
            sun = np.array([0.01, -1.0, 0.02], np.float32)
        mn = rng.uniform(-50, 0, size=3).astype(np.float32)
        mx = mn + rng.uniform(0.1, 80, size=3).astype(np.float32)
        res = int(rng.choice([256, 1024, 2048]))
        a = dir_light_camera_aabb(sun, mn, mx, 10.0, res)
        b = oracle_mod.dir_light_camera_aabb(sun, mn, mx, 10.0, res)
        for x, y in zip(a, b):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_lib_struct_layouts():
    from shs_gpu import _abi
    assert ctypes.sizeof(_abi.LibDrawC) == 4 * 4 + 4 * 64 + 4 * (3 + 3 + 1 + 3 + 3 + 3) + 4 + 64 + 4 * 6 + 4   # + base_color_tex
    assert ctypes.sizeof(_abi.LibFrameC) == 5 * 4 + 2 * 4 + 16
    assert ctypes.sizeof(_abi.LibStats) == 7 * 8
    assert ctypes.sizeof(_abi.ShadowCasterC) == 4 + 64


def _c5_small_outputs(oracle_mod):
    from shs_gpu import scene_lib
    frame, draws, casters, sun, _ = scene_lib.c5_scene(320, 180)
    sm, lvp = oracle_mod.shadow_map(128, sun, casters)
    scene_lib.wire_shadow(draws, lvp)
    hdr, d, m, st = oracle_mod.pbr_forward(frame, draws, sm)
    return sm, hdr, d, m, st


def test_lib_golden_fixture(oracle_mod):
    """Regression pin of the oracle on C5-small (tests/golden/make_golden.py --lib writes it)."""
    g = json.load(open(GOLDEN))
    sm, hdr, d, m, st = _c5_small_outputs(oracle_mod)
    assert st == g["stats"]
    assert oracle_mod.fnv1a64(sm) == int(g["shadow_fnv"], 16)
    assert oracle_mod.fnv1a64(d) == int(g["depth_fnv"], 16)
    assert int((d < 1).sum()) == g["covered"]
    # shaded floats: pinned to 1e-5 (libm powf may differ by an ulp across hosts)
    for (y, x), v in zip(g["probe_px"], g["probe_hdr"]):
        assert np.allclose(hdr[y, x], v, rtol=1e-5, atol=1e-5)


def test_row_parallel_split_matches_sequential():
    """The oracle's row-parallel split of big bboxes (the reference's parallel_for_1d over rows,
    rasterizer.hpp:424-436) leaves the same targets as the sequential loop."""
    from oracle import oracle
    from shs_gpu import scene_lib
    frame, draws, casters, sun, S = scene_lib.c5_scene(640, 360, floor_seg=1)   # 2 floor triangles: big bboxes
    sm, lvp = oracle.shadow_map(256, sun, casters)
    scene_lib.wire_shadow(draws, lvp)
    a = oracle.pbr_forward(frame, draws, sm)
    try:
        oracle.set_lib_threads(6)
        b = oracle.pbr_forward(frame, draws, sm)
    finally:
        oracle.set_lib_threads(1)
    for x, y in zip(a, b):
        if isinstance(x, np.ndarray):
            assert np.array_equal(x.view(np.uint8), y.view(np.uint8))
