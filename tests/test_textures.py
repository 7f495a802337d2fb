"""SURVEY 8(a) row a13, the texture half: base_color_tex sampled by the builtin PBR and Blinn-Phong
programs (shader/builtin_shaders.hpp:25-55, read at :113 and :162) at the perspective-correct UV0
varying (sw_render/rasterizer.hpp:383-387), through clipping (lerp_rv, :69-79).

CPU: the oracle's sampler against a float32 numpy restatement (repeat wrap, the four texels, the
glm::mix order), including 1x1 / 1xN textures and UVs outside [0, 1].  GPU: textured C5 frames
(non-power-of-two, 1x1 and single-row textures, negative UVs, the floor clipped at the frustum) against
the oracle -- depth bit-exact, HDR within 1e-5 -- at 640x360 for both programs and at the full 4K
size with the 2048^2 shadow pass."""
import numpy as np
import pytest

from helpers import assert_depth_bitexact, assert_float_close

f32 = np.float32


def _srgb(c):
    # std::pow((float)c / 255.0f, 2.2f): glibc powf, within an ulp of the double-rounded value
    return f32((float(c) / 255.0) ** 2.2)


def _mix(a, b, t):
    return a * (f32(1.0) - t) + b * t


def _sample_ref(rgba, u, v):
    h, w = rgba.shape[:2]
    u, v = f32(u), f32(v)
    uu = u - f32(np.floor(u))
    vv = v - f32(np.floor(v))
    fx = uu * f32(w - 1)
    fy = vv * f32(h - 1)
    x0, y0 = int(np.floor(fx)), int(np.floor(fy))
    x1, y1 = min(x0 + 1, w - 1), min(y0 + 1, h - 1)
    tx, ty = fx - f32(x0), fy - f32(y0)
    lin = lambda x, y: np.array([_srgb(c) for c in rgba[y, x, :3]], f32)
    return _mix(_mix(lin(x0, y0), lin(x1, y0), tx), _mix(lin(x0, y1), lin(x1, y1), tx), ty)


@pytest.mark.parametrize("w,h", [(2, 2), (1, 1), (1, 7), (5, 1), (37, 23)])
def test_oracle_sampler_known_answers(oracle_mod, w, h):
    rng = np.random.default_rng(w * 100 + h)
    rgba = rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    uvs = [(0.0, 0.0), (1.0, 1.0), (0.5, 0.5), (-0.25, 0.75), (3.3, -2.7), (0.999, 0.001), (-1e-9, 2.0), (17.125, -4.5)]
    uvs += [tuple(x) for x in rng.uniform(-5, 5, size=(40, 2))]
    for u, v in uvs:
        got = oracle_mod.sample_texture(rgba, u, v)
        want = _sample_ref(rgba, u, v)
        assert np.allclose(got, want, rtol=0, atol=2e-7), (u, v, got, want)
    # a 1x1 texture is its texel's linear colour everywhere
    one = rgba[:1, :1]
    assert np.allclose(oracle_mod.sample_texture(one, 0.3, -7.1), [_srgb(c) for c in one[0, 0, :3]], atol=2e-7)


def test_oracle_untextured_equals_white_texture(oracle_mod):
    """albedo_tex = vec3(1) without a texture (:35): a 1x1 texel of 255 gives the same frame."""
    from shs_gpu import scene_lib
    from shs_gpu.lib_path import Texture2D
    frame, draws, _, _, _ = scene_lib.c5_scene(96, 64, textured=False)
    h0, d0, _, _ = oracle_mod.pbr_forward(frame, draws)
    for d in draws:
        d.base_color_tex = Texture2D(rgba=np.full((1, 1, 4), 255, np.uint8))
    h1, d1, _, _ = oracle_mod.pbr_forward(frame, draws)
    assert np.array_equal(d0.view(np.uint32), d1.view(np.uint32))
    assert np.array_equal(h0.view(np.uint32), h1.view(np.uint32))


def _render_both(ctx, oracle_mod, frame, draws, casters, sun, S):
    from shs_gpu import scene_lib
    lvp = ctx.render_shadow_map(S, sun, casters)
    sm_ref, lvp_ref = oracle_mod.shadow_map(S, sun, casters)
    assert np.array_equal(lvp.view(np.uint32), lvp_ref.view(np.uint32))
    scene_lib.wire_shadow(draws, lvp)
    ctx.render_pbr_forward(frame, draws)
    gh, gd, gm = ctx.resolve_lib()
    rh, rd, rm, rst = oracle_mod.pbr_forward(frame, draws, sm_ref)
    st = ctx.lib_stats()
    for k in ("tri_input", "tri_after_clip", "tri_raster"):
        assert st[k] == rst[k], (k, st[k], rst[k])
    assert_depth_bitexact(gd, rd)
    assert_float_close(gm, rm, what="motion")
    return assert_float_close(gh, rh, what="textured hdr"), gh, rh


@pytest.mark.gpu
@pytest.mark.parametrize("program", [0, 1], ids=["pbr", "blinn_phong"])
@pytest.mark.parametrize("floor_tex,monkey_tex", [((37, 23), (1, 1)), ((1, 1), (5, 3)), ((1, 17), (64, 64)),
                                                  ((64, 64), (13, 1))])
def test_textured_frames_vs_oracle(gpu_ctx, oracle_mod, program, floor_tex, monkey_tex):
    from shs_gpu import scene_lib
    frame, draws, casters, sun, S = scene_lib.c5_scene(640, 360, 512, program=program, textured=True,
                                                       floor_tex=floor_tex, monkey_tex=monkey_tex)
    n, gh, rh = _render_both(gpu_ctx, oracle_mod, frame, draws, casters, sun, S)
    # the texture changes the image: the same frame untextured differs
    frame0, draws0, casters0, _, _ = scene_lib.c5_scene(640, 360, 512, program=program, textured=False)
    scene_lib.wire_shadow(draws0, draws[0].light_viewproj)
    gpu_ctx.render_pbr_forward(frame0, draws0)
    h0, _, _ = gpu_ctx.resolve_lib()
    if floor_tex != (1, 1) or monkey_tex != (1, 1):
        assert not np.array_equal(h0, gh)
    print(f"program {program} floor {floor_tex} monkey {monkey_tex}: {n} HDR channels not bit-identical")


@pytest.mark.gpu
def test_textured_c5_full_size(gpu_ctx, oracle_mod):
    """The textured C5 variant at the stated size: 3840x2160 PBR + PCF over the 2048^2 shadow map."""
    from shs_gpu import scene_lib
    frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160, 2048, textured=True)
    n, gh, _ = _render_both(gpu_ctx, oracle_mod, frame, draws, casters, sun, S)
    print(f"textured c5 4K: {n} HDR channels not bit-identical (within 1e-5)")


@pytest.mark.gpu
def test_texture_ids_and_release(gpu_ctx):
    import ctypes
    import shs_gpu
    L = gpu_ctx._lib
    rgba = np.zeros((3, 5, 4), np.uint8)
    tid = ctypes.c_int32()
    assert L.shs_texture_upload(gpu_ctx._h, rgba.ctypes.data_as(ctypes.c_void_p), 5, 3, ctypes.byref(tid)) == 0
    assert tid.value >= 1
    assert L.shs_texture_upload(gpu_ctx._h, rgba.ctypes.data_as(ctypes.c_void_p), 0, 3, ctypes.byref(tid)) != 0
    assert L.shs_texture_release(gpu_ctx._h, 0) != 0
    from shs_gpu import scene_lib
    frame, draws, _, _, _ = scene_lib.c5_scene(64, 48, textured=True)
    arr = gpu_ctx.prepare_lib(frame, draws)
    bad = arr[2][0].base_color_tex + 1000
    arr[2][0].base_color_tex = bad
    with pytest.raises(shs_gpu.ShsError):
        gpu_ctx.render_pbr_forward_prepared(arr)
