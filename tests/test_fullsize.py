"""BASELINE configs 4 and 5 at their stated sizes against the CPU oracle (the parity tests
stopped at 512x288; the oracle does a full C5 frame in ~0.6 s and a full C4 frame in a few seconds).

C5: PassShadowMap 2048^2 + PassPBRForward (PBR, PCF, motion) at 3840x2160, the bench's exact draws.
C4: Forward+ light lists (256 lights, 16-px tiles, max 128) + the per-pixel point-light pass over 1M
triangles at 3840x2160.  Shadow map, light camera, depth, coverage counts and light lists: bit-exact;
HDR colour and motion: within 1e-5 per channel, absolute (helpers.assert_float_close)."""
import numpy as np
import pytest

from helpers import assert_depth_bitexact, assert_float_close

pytestmark = pytest.mark.gpu


def test_c5_full_size_exact(gpu_ctx, oracle_mod):
    from shs_gpu import scene_lib
    frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160, 2048)
    lvp = gpu_ctx.render_shadow_map(S, sun, casters)
    sm_gpu = gpu_ctx.resolve_shadow_map()
    sm_ref, lvp_ref = oracle_mod.shadow_map(S, sun, casters)
    assert np.array_equal(lvp.view(np.uint32), lvp_ref.view(np.uint32)), "light camera differs"
    assert_depth_bitexact(sm_gpu, sm_ref)
    assert (sm_ref < 1.0).sum() > 100_000
    scene_lib.wire_shadow(draws, lvp)
    gpu_ctx.render_pbr_forward(frame, draws)
    gh, gd, gm = gpu_ctx.resolve_lib()
    st = gpu_ctx.lib_stats()
    rh, rd, rm, rst = oracle_mod.pbr_forward(frame, draws, sm_ref)
    for k in ("tri_input", "tri_after_clip", "tri_raster"):
        assert st[k] == rst[k], (k, st[k], rst[k])
    assert_depth_bitexact(gd, rd)
    assert st["covered_pixels"] == int((rd < 1.0).sum()) > 1_000_000
    assert_float_close(gm, rm, what="motion")
    n = assert_float_close(gh, rh, what="hdr")
    print(f"c5 4K: {st['covered_pixels']} covered px, {n} HDR channels not bit-identical (within 1e-5)")


def test_c4_full_size_exact(gpu_ctx, oracle_mod):
    from shs_gpu import scene_lib
    frame, draws, lights, cull = scene_lib.c4_scene()
    gpu_ctx.upload_lights(lights)
    gpu_ctx.light_cull(cull)
    gc, gi, _ = gpu_ctx.resolve_light_lists()
    rc, ri = oracle_mod.light_cull(cull, lights)[:2]
    assert np.array_equal(gc, rc), "list counts differ"
    for l in np.nonzero(rc)[0]:
        n = int(rc[l])
        assert np.array_equal(gi[l, :n], ri[l, :n]), f"list {l} differs"
    assert rc.sum() > 0 and rc.max() <= cull.max_per_tile
    gpu_ctx.render_pbr_forward(frame, draws)
    gh, gd, gm = gpu_ctx.resolve_lib()
    st = gpu_ctx.lib_stats()
    assert st["tri_input"] == 1_000_000
    rh, rd, rm, rst = oracle_mod.forward_plus(frame, draws, lights, cull, (rc, ri))
    assert_depth_bitexact(gd, rd)
    assert st["covered_pixels"] == int((rd < 1.0).sum()) > 500_000
    assert_float_close(gm, rm, what="motion")
    n = assert_float_close(gh, rh, what="forward+ hdr")
    print(f"c4 4K: {st['covered_pixels']} covered px, {n} HDR channels not bit-identical (within 1e-5)")
