"""Profiling hooks (SHS_OPT_TIMELINE): the library raster's workgroup timeline of the camera pass (1) or
of the shadow pass (2, round 6), read with shs_lib_debug_timeline.  The hooks only add stores of
s_memrealtime stamps and counts: the images stay the oracle's (the other tests), so this checks the
records themselves -- every busy tile counted once, in the pass that was asked for."""
import numpy as np
import pytest


def _run(ctx, frame, draws, casters, sun, S, prep):
    ctx.render_shadow_map(S, sun, casters)
    ctx.render_pbr_forward_prepared(prep)
    ctx.synchronize_lib()
    t = ctx.lib_debug_timeline().astype(np.int64)
    F = {k: i for i, k in enumerate(ctx.LIB_TIMELINE_FIELDS)}
    return t, F


@pytest.mark.gpu
def test_camera_and_shadow_raster_timelines():
    import shs_gpu
    from shs_gpu import scene_lib
    frame, draws, casters, sun, S = scene_lib.c5_scene(640, 360, 256)
    ctx = shs_gpu.Context(0)
    try:
        lvp = ctx.render_shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)
        prep = ctx.prepare_lib(frame, draws)
        ctx.render_pbr_forward_prepared(prep)
        ctx.synchronize_lib()
        ctx.set_timeline(True)
        cam, F = _run(ctx, frame, draws, casters, sun, S, prep)
        ctx.set_timeline(True, shadow=True)
        sh, _ = _run(ctx, frame, draws, casters, sun, S, prep)
        ctx.set_timeline(False)
        for t in (cam, sh):
            live = t[:, F["start"]] > 0
            assert live.any()
            assert (t[live, F["end"]] >= t[live, F["start"]]).all()
            assert t[:, F["n_busy"]].sum() > 0
        # the shadow map's raster tiles: 256 x 256 texels in 32 x 8 tiles; a workgroup renders or
        # clears each owned tile once
        n_sm = (S // 32) * (S // 8)
        assert sh[:, F["n_busy"]].sum() + sh[:, F["n_clear"]].sum() <= n_sm
        assert cam[:, F["n_busy"]].sum() <= ((640 + 31) // 32) * ((360 + 7) // 8)
    finally:
        ctx.close()
