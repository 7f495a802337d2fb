"""CPU tests of the oracle (CPU restatement of the reference path).

PARITY UNPINNED: the reference ships no golden vectors for this path and cannot be built here
(SURVEY.md 8c), so these are analytic known-answer tests derived directly from the reference lines
(cited per test) plus regression fixtures the oracle itself produced (tests/golden/, made by
tests/golden/make_golden.py)."""
import json
import os

import numpy as np
import pytest

FLT_MAX = np.finfo(np.float32).max
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "legacy_golden.json")


class _Mesh:
    def __init__(self, pos, nrm):
        self.positions = np.asarray(pos, np.float32).reshape(-1, 9)
        self.normals = np.asarray(nrm, np.float32).reshape(-1, 9)


class _Draw:
    def __init__(self, mesh, shading=3, color=(200, 100, 50, 255), mvp=None, model=None):
        eye = np.eye(4, dtype=np.float32).reshape(16)
        self.mesh = mesh
        self.shading = shading
        self.mvp = eye if mvp is None else mvp
        self.model = eye if model is None else model
        self.light_dir = np.array([0.0, 0.0, 1.0], np.float32)
        self.camera_pos = np.array([0.0, 0.0, -5.0], np.float32)
        self.color = color


def _ndc(px, py, z, W, H):
    """Pixel-space corner -> NDC position that clip_to_screen maps back (identity MVP)."""
    return [px / (0.5 * (W - 1)) - 1.0, 1.0 - py / (0.5 * (H - 1)), z]


def _tri(W, H, pts, z=0.5):
    return np.array([c for p in pts for c in _ndc(p[0], p[1], z, W, H)], np.float32)


# ---- Canvas::barycentric_coordinate (shs_renderer.hpp:802-821) --------------------------------
def test_barycentric_known_answers(oracle_mod):
    bc = oracle_mod.barycentric([0, 0, 8, 0, 0, 8], 2.0, 2.0)
    assert bc.tolist() == [0.5, 0.25, 0.25]
    bc = oracle_mod.barycentric([0, 0, 8, 0, 0, 8], 8.0, 8.0)
    assert bc.tolist() == [-1.0, 1.0, 1.0]


def test_barycentric_degenerate_double_compare(oracle_mod):
    """`std::abs(denom) < 1e-5` compares a float against the DOUBLE literal: a denominator equal to
    1e-5f (9.99999974738e-06 < 1e-5) is rejected; the next float up is not."""
    # v0 = (a, 0), v1 = (0, b): denom = a^2 b^2 -> choose a*b = sqrt(denom)
    den_f = np.float32(1e-5)
    assert float(den_f) < 1e-5
    # a = 1, b = sqrt(den): denom = b^2 rounded; search b so that fl(b*b) == den_f
    b = np.float32(np.sqrt(np.float64(den_f)))
    while np.float32(b * b) < den_f:
        b = np.nextafter(b, np.float32(1))
    while np.float32(b * b) > den_f:
        b = np.nextafter(b, np.float32(0))
    if np.float32(b * b) == den_f:
        assert (oracle_mod.barycentric([0, 0, 1, 0, 0, float(b)], 0.1, 0.001) == -1.0).all()
    b2 = np.float32(0.01)   # denom 1e-4: accepted
    assert not (oracle_mod.barycentric([0, 0, 1, 0, 0, float(b2)], 0.1, 0.001) == -1.0).all()


# ---- draw_triangle_tile (hello_pipeline_blinn_phong_shading.cpp:189-242) -----------------------
def test_area_cull_winding(oracle_mod):
    """`if (area <= 0) return` with screen y down: only one winding of a triangle renders."""
    W, H = 64, 48
    a = _tri(W, H, [(10, 10), (40, 12), (20, 35)])
    b = _tri(W, H, [(10, 10), (20, 35), (40, 12)])
    n = np.zeros(9, np.float32) + np.float32(0.577)
    ca, da, _ = oracle_mod.render_legacy(W, H, [_Draw(_Mesh(a, n))])
    cb, db, _ = oracle_mod.render_legacy(W, H, [_Draw(_Mesh(b, n))])
    cov_a, cov_b = (da < FLT_MAX).sum(), (db < FLT_MAX).sum()
    assert (cov_a == 0) != (cov_b == 0)
    assert max(cov_a, cov_b) > 200


def test_clear_values_and_row_flip(oracle_mod):
    """Canvas clear = black opaque, ZBuffer clear = FLT_MAX; colour lands in canvas rows
    (H-1-y), depth in screen rows (blinn_phong_shading.cpp:231, 238)."""
    W, H = 64, 48
    t = _tri(W, H, [(2, 2), (20, 2), (2, 12)])
    t2 = _tri(W, H, [(2, 2), (2, 12), (20, 2)])
    n = np.zeros(9, np.float32) + np.float32(0.577)
    c, d, _ = oracle_mod.render_legacy(W, H, [_Draw(_Mesh(np.concatenate([t, t2]), np.concatenate([n, n])))])
    ys, xs = np.nonzero(d < FLT_MAX)
    assert ys.max() < 14                       # depth: near the top (screen rows)
    written = np.nonzero(c[..., 0] | c[..., 1] | c[..., 2])[0]
    assert written.min() > H - 15              # colour: flipped to the bottom canvas rows
    assert (c[d.shape[0] - 1 - ys, xs, 3] == 255).all()
    assert (c[0, W - 1] == [0, 0, 0, 255]).all() and d[H - 1, W - 1] == FLT_MAX


def test_strict_less_first_wins(oracle_mod):
    """ZBuffer::test_and_set_depth is strict '<' (shs_renderer.hpp:664): of two identical triangles
    at equal z the FIRST submitted one keeps the pixel."""
    W, H = 64, 48
    t = _tri(W, H, [(5, 5), (50, 8), (10, 40)])
    if oracle_mod.render_legacy(W, H, [_Draw(_Mesh(t, np.ones(9, np.float32)))])[1].min() == FLT_MAX:
        t = _tri(W, H, [(5, 5), (10, 40), (50, 8)])
    n = np.ones(9, np.float32)
    first = _Draw(_Mesh(t, n), color=(255, 0, 0, 255))
    second = _Draw(_Mesh(t, n), color=(0, 255, 0, 255))
    c, d, _ = oracle_mod.render_legacy(W, H, [first, second])
    cov = d < FLT_MAX
    assert cov.sum() > 100
    rows = H - 1 - np.nonzero(cov)[0]
    assert (c[rows, np.nonzero(cov)[1], 1] == 0).all()     # no green anywhere


def test_threads_and_tiles_deterministic(oracle_mod):
    """Disjoint tile jobs: results do not depend on the worker count."""
    from shs_gpu import scene
    frame, draws = scene.config("c1")
    a = oracle_mod.render_legacy(frame.width, frame.height, draws, threads=1)
    b = oracle_mod.render_legacy(frame.width, frame.height, draws, threads=7)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))


def test_tile_clamp_visits_outside_bbox(oracle_mod):
    """The tile clamp (blinn_phong_shading.cpp:208-215) makes the reference test pixels outside a
    triangle's bbox; for hair-thin slivers some of those pass: the 80x80-tile image differs from
    the single-tile image."""
    rng = np.random.default_rng(99)
    W, H = 400, 300
    tris = []
    for _ in range(3000):
        c = rng.uniform([0, 0], [W, H])
        dv = rng.normal(size=2); dv /= np.linalg.norm(dv)
        L = rng.uniform(20, 400)
        nv = np.array([-dv[1], dv[0]])
        p = np.stack([c, c + dv * L, c + dv * L * rng.uniform(0.05, 0.95) + nv * rng.uniform(-0.02, 0.02)])
        z = rng.uniform(-0.9, 0.9, size=3)
        tris.append(np.stack([p[:, 0] / (0.5 * (W - 1)) - 1.0, 1.0 - p[:, 1] / (0.5 * (H - 1)), z], axis=1).reshape(9))
    pos = np.asarray(tris, np.float32)
    d = _Draw(_Mesh(pos, rng.normal(size=pos.shape)))
    _, d80, _ = oracle_mod.render_legacy(W, H, [d], tile=(80, 80), threads=8)
    _, d1, _ = oracle_mod.render_legacy(W, H, [d], tile=(W, H), threads=8)
    assert (d80.view(np.uint32) != d1.view(np.uint32)).sum() > 0


# ---- regression fixtures ------------------------------------------------------------------
def _load_golden():
    with open(GOLDEN) as fh:
        return json.load(fh)


def _draws_from_fixture(entry):
    from shs_gpu import scene
    mesh = scene.monkey()
    draws = []
    for d in entry["draws"]:
        dd = _Draw(mesh, d["shading"], tuple(d["color"]),
                   np.array(d["mvp"], np.uint32).view(np.float32), np.array(d["model"], np.uint32).view(np.float32))
        dd.light_dir = np.array(d["light_dir"], np.uint32).view(np.float32)
        dd.camera_pos = np.array(d["camera_pos"], np.uint32).view(np.float32)
        draws.append(dd)
    return draws


@pytest.mark.parametrize("name", [e["name"] for e in json.load(open(GOLDEN))["frames"]] if os.path.exists(GOLDEN) else [])
def test_golden_frames(oracle_mod, name):
    """Oracle output hashes for the committed scenes (uniforms stored as float bits)."""
    entry = next(e for e in _load_golden()["frames"] if e["name"] == name)
    draws = _draws_from_fixture(entry)
    c, d, _ = oracle_mod.render_legacy(entry["width"], entry["height"], draws, tile=tuple(entry["tile"]), threads=8)
    assert oracle_mod.fnv1a64(d) == int(entry["depth_fnv1a64"], 16)
    assert oracle_mod.fnv1a64(c) == int(entry["color_fnv1a64"], 16)
    assert int((d < FLT_MAX).sum()) == entry["covered"]


@pytest.mark.parametrize("name", [e["name"] for e in json.load(open(GOLDEN))["frames"]] if os.path.exists(GOLDEN) else [])
def test_golden_uniforms_from_host_helpers(name):
    """The product's host GLM helpers rebuild exactly the fixture's uniforms (bit-exact)."""
    from shs_gpu import scene
    entry = next(e for e in _load_golden()["frames"] if e["name"] == name)
    frame, draws = scene.build_named(entry["scene"])
    assert (frame.width, frame.height) == (entry["width"], entry["height"])
    for got, want in zip(draws, entry["draws"]):
        assert got.mvp.view(np.uint32).tolist() == want["mvp"]
        assert got.model.view(np.uint32).tolist() == want["model"]
        assert np.asarray(got.light_dir, np.float32).view(np.uint32).tolist() == want["light_dir"]
