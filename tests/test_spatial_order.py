"""Spatially ordered library meshes: shs_mesh_upload stores a mesh of more than one
256-triangle chunk sorted by the Morton code of each triangle's centroid, so a setup block's chunk box is
tight; the submission order stays the MeshData order (LibDrawGPU::orig, the per-pass s2s map).

The order-sensitive cases, against the oracle (which draws in MeshData order):
- exact z ties everywhere: NDC-space triangles (identity viewproj) on a few exact depth planes, so every
  overlap is decided by the submission order alone (strict `<`: the first submitted wins,
  rasterizer.hpp:355-363);
- no depth target: every fragment writes, the last submitted wins;
- the same through an indexed mesh and with a second draw after the first (per-draw bases).
The numpy restatement of the stored order (`stored_order`) checks the upload really reorders these
meshes, so the tests are not vacuous."""
import numpy as np
import pytest

from helpers import assert_depth_bitexact, assert_float_close


def stored_order(pos, idx=None):
    """csrc/shs_abi_lib.cpp spatial_order: MeshData indices by (30-bit Morton code of the float32
    centroid sum in the mesh's centroid bounds, index)."""
    p = np.asarray(pos, np.float32).reshape(-1, 3)
    tri = (np.asarray(idx, np.int64).reshape(-1, 3) if idx is not None else np.arange(p.shape[0]).reshape(-1, 3))
    c = ((np.float32(0) + p[tri[:, 0]]) + p[tri[:, 1]]) + p[tri[:, 2]]
    lo, hi = c.min(0), c.max(0)
    ext = hi - lo
    u = np.where(ext > 0, (c - lo) / np.where(ext > 0, ext, 1), np.float32(0)).astype(np.float32)
    b = np.clip(u * np.float32(1024.0), 0, 1023).astype(np.uint32)

    def spread(x):
        x = x.astype(np.uint64) & 0x3FF
        out = np.zeros_like(x)
        for i in range(10):
            out |= ((x >> i) & 1) << (3 * i)
        return out
    code = spread(b[:, 0]) | (spread(b[:, 1]) << 1) | (spread(b[:, 2]) << 2)
    return np.lexsort((np.arange(len(code)), code))


def _ndc_tie_soup(rng, n, levels=(0.0, 0.5, -0.25)):
    """n triangles in NDC (identity viewproj: clip = position, w = 1), each on one of a few exact depth
    planes: z01 = z * 0.5 + 0.5 exactly, so overlapping triangles of one plane tie at every pixel."""
    c = rng.uniform(-0.9, 0.9, size=(n, 1, 2))
    xy = c + rng.normal(scale=rng.choice([0.04, 0.15, 0.4], size=(n, 1, 1)), size=(n, 3, 2))
    z = np.repeat(np.asarray(levels, np.float32)[rng.integers(0, len(levels), n)][:, None, None], 3, axis=1)
    pos = np.concatenate([xy, z], axis=2).reshape(-1, 3).astype(np.float32)
    nrm = rng.normal(size=pos.shape).astype(np.float32)   # distinct shading per triangle: the winner shows
    return pos, nrm


def _check(ctx, oracle_mod, frame, draws):
    ctx.render_pbr_forward(frame, draws)
    gh, gd, gm = ctx.resolve_lib()
    rh, rd, rm, rst = oracle_mod.pbr_forward(frame, draws, None)
    if gd is not None:
        assert_depth_bitexact(gd, rd)
        assert_float_close(gm, rm, what="motion")
    assert_float_close(gh, rh, what="hdr")
    st = ctx.lib_stats()
    for k in ("tri_input", "tri_after_clip", "tri_raster"):
        assert st[k] == rst[k], (k, st[k], rst[k])
    return rd


def test_stored_order_reorders_the_test_meshes():
    rng = np.random.default_rng(3)
    pos, _ = _ndc_tie_soup(rng, 3000)
    order = stored_order(pos)
    assert sorted(order.tolist()) == list(range(3000))
    assert (order != np.arange(3000)).mean() > 0.9


@pytest.mark.gpu
@pytest.mark.parametrize("indexed", [False, True])
@pytest.mark.parametrize("depth", [True, False])
def test_submission_order_survives_spatial_order(gpu_ctx, oracle_mod, indexed, depth):
    from shs_gpu.lib_path import LibDraw, LibFrame, LibMesh
    rng = np.random.default_rng(11 + indexed)
    W, H = 256, 192
    pos, nrm = _ndc_tie_soup(rng, 3000)
    if indexed:   # shared vertices through a shuffled index buffer
        perm = rng.permutation(pos.shape[0])
        vpos, vnrm = pos[perm], nrm[perm]
        inv = np.empty_like(perm)
        inv[perm] = np.arange(perm.size)
        mesh = LibMesh(vpos, vnrm, None, inv.astype(np.uint32))
        assert (stored_order(vpos, inv) != np.arange(3000)).mean() > 0.9
    else:
        mesh = LibMesh(pos, nrm)
    frame = LibFrame(W, H, depth_motion=depth, zn=1.0, zf=1.0, bg_gradient=False, clear_hdr=(0.1, 0.2, 0.3, 1.0))
    d0 = LibDraw(mesh=mesh, program=2, cull_mode=0, light_intensity=2.0)
    rd = _check(gpu_ctx, oracle_mod, frame, [d0])
    if depth:   # the tie planes really cover pixels
        assert np.isin(rd, np.float32([0.5, 0.75, 0.375])).mean() > 0.5
    # a second draw of another reordered mesh after the first: its submission indices start at 3000
    pos2, nrm2 = _ndc_tie_soup(np.random.default_rng(99), 1500)
    d1 = LibDraw(mesh=LibMesh(pos2, nrm2), program=3, cull_mode=0, base_color=(0.9, 0.3, 0.2))
    _check(gpu_ctx, oracle_mod, frame, [d0, d1])


@pytest.mark.gpu
def test_spatial_order_with_clipping_and_motion(gpu_ctx, oracle_mod):
    """Perspective soup crossing the clip planes (fans >= 1 in extra slots: the s2s -> xbase path) with
    motion vectors, in a reordered mesh."""
    from test_lib_parity import _camera, _clip_soup
    from shs_gpu.lib_path import LibDraw, LibFrame, LibMesh, model_euler
    rng = np.random.default_rng(21)
    W, H = 320, 200
    pos, nrm, uv = _clip_soup(rng, 2500)
    assert (stored_order(pos) != np.arange(2500)).mean() > 0.9
    d = LibDraw(mesh=LibMesh(pos, nrm, uv), program=1, viewproj=_camera(W, H),
                model=model_euler((0.1, -0.2, 0.3), (0.2, 0.4, -0.1), (1.0, 1.2, 0.9)),
                prev_model=model_euler((0.0, -0.2, 0.3), (0.2, 0.45, -0.1), (1.0, 1.2, 0.9)), camera_pos=(0.3, 0.7, -3.0),
                cull_mode=0, enable_motion_vectors=True, light_intensity=3.0)
    _check(gpu_ctx, oracle_mod, LibFrame(W, H, zn=0.5, zf=30.0), [d])
    assert gpu_ctx.lib_stats()["clipped_extra"] > 0
