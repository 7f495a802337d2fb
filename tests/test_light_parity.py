"""GPU parity of the Forward+ light-list binning (fp_stress_depth_reduce.comp / fp_stress_light_cull.comp
semantics) and the per-pixel point-light program against the CPU oracle (oracle/shs_oracle_light.c).

Lists (counts and the ascending light indices) and depth ranges: exact.  Shaded HDR: within 1e-5."""
import numpy as np
import pytest

from helpers import assert_depth_bitexact, assert_float_close

pytestmark = pytest.mark.gpu


def _small_c4(mode=1, max_per_tile=128, tile=16, W=480, H=270, n_lights=64):
    from shs_gpu import scene_lib
    return scene_lib.c4_scene(W, H, n_objects=60, tris_per_object=200, n_lights=n_lights, mode=mode, tile_size=tile,
                              max_per_tile=max_per_tile)


def _prepass(draws):
    """Depth prepass: the same draws with a program that reads no light lists (depth is program
    independent; the reference's make_depth_prepass_program, pass_adapters.hpp:335-353)."""
    return [type(d)(**{**d.__dict__, "program": 2}) for d in draws]


def _check_lists(gpu_ctx, oracle_mod, cull, lights, depth=None):
    gc, gi, gr = gpu_ctx.resolve_light_lists()
    rc, ri, rr = oracle_mod.light_cull(cull, lights, depth)
    assert np.array_equal(gc, rc), f"{int((gc != rc).sum())} list counts differ"
    for l in np.nonzero(rc)[0]:
        n = int(rc[l])
        assert np.array_equal(gi[l, :n], ri[l, :n]), f"list {l} differs"
    if cull.mode == 2:
        assert np.array_equal(gr.view(np.uint32), rr.view(np.uint32))
    return gc


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_light_lists_exact(gpu_ctx, oracle_mod, mode):
    frame, draws, lights, cull = _small_c4(mode)
    gpu_ctx.upload_lights(lights)
    gpu_ctx.render_pbr_forward(frame, _prepass(draws))
    _, depth, _ = gpu_ctx.resolve_lib()
    gpu_ctx.light_cull(cull)
    counts = _check_lists(gpu_ctx, oracle_mod, cull, lights, depth)
    assert counts.max() > 0


@pytest.mark.parametrize("mode,tile,maxp", [(1, 16, 128), (2, 16, 128), (1, 8, 4), (3, 32, 16)])
def test_forward_plus_frame(gpu_ctx, oracle_mod, mode, tile, maxp):
    """Depth prepass -> (depth reduce) -> light cull -> Forward+ shading, GPU vs oracle."""
    frame, draws, lights, cull = _small_c4(mode, max_per_tile=maxp, tile=tile)
    gpu_ctx.upload_lights(lights)
    gpu_ctx.render_pbr_forward(frame, _prepass(draws))
    _, depth, _ = gpu_ctx.resolve_lib()
    gpu_ctx.light_cull(cull)
    lists = _check_lists(gpu_ctx, oracle_mod, cull, lights, depth)
    gpu_ctx.render_pbr_forward(frame, draws)
    gh, gd, _ = gpu_ctx.resolve_lib()
    rc, ri, _ = oracle_mod.light_cull(cull, lights, depth)
    rh, rd, _, _ = oracle_mod.forward_plus(frame, draws, lights, cull, (rc, ri))
    assert_depth_bitexact(gd, rd)
    assert_float_close(gh, rh, what="forward+ hdr")
    if maxp == 4:
        assert (lists >= 4).any(), "no saturated list: the full-loop fallback is not exercised"


@pytest.mark.parametrize("mode", [1, 2])
def test_forward_plus_resize_sequence(gpu_ctx, oracle_mod, mode):
    """One context through frame sizes that keep / change the bin-tile grid, the raster-tile rows and
    the light-tile grid (each cached per geometry on the device side): every frame vs the oracle."""
    for W, H in [(480, 270), (480, 262), (470, 262), (200, 130), (17, 9), (480, 270)]:
        frame, draws, lights, cull = _small_c4(mode, W=W, H=H, n_lights=32)
        gpu_ctx.upload_lights(lights)
        gpu_ctx.render_pbr_forward(frame, _prepass(draws))
        _, depth, _ = gpu_ctx.resolve_lib()
        gpu_ctx.light_cull(cull)
        _check_lists(gpu_ctx, oracle_mod, cull, lights, depth)
        gpu_ctx.render_pbr_forward(frame, draws)
        gh, gd, _ = gpu_ctx.resolve_lib()
        rc, ri, _ = oracle_mod.light_cull(cull, lights, depth)
        rh, rd, _, _ = oracle_mod.forward_plus(frame, draws, lights, cull, (rc, ri))
        assert_depth_bitexact(gd, rd)
        assert_float_close(gh, rh, what=f"forward+ hdr {W}x{H}")


def test_light_lists_sharded(gpu_ctx, oracle_mod):
    """Lists of a tile shard equal the full lists on the owned 32x32 tiles and are empty elsewhere."""
    frame, draws, lights, cull = _small_c4(1)
    gpu_ctx.upload_lights(lights)
    gpu_ctx.light_cull(cull)
    full_c, full_i, _ = gpu_ctx.resolve_light_lists()
    tx, ty = cull.tiles
    for rank in range(3):
        cull.shard_rank, cull.shard_count = rank, 3
        gpu_ctx.light_cull(cull)
        c, i, _ = gpu_ctx.resolve_light_lists()
        for l in range(tx * ty):
            x, y = l % tx, l // tx
            row_up = frame.height - 1 - y * cull.tile_size
            owned = ((row_up // 32) * ((frame.width + 31) // 32) + (x * cull.tile_size) // 32) % 3 == rank
            if owned:
                assert c[l] == full_c[l] and np.array_equal(i[l, :c[l]], full_i[l, :c[l]])
            else:
                assert c[l] == 0


def test_c4_full_size_properties(gpu_ctx):
    """1M triangles, 256 lights, 3840x2160 (beyond the oracle's reach here): lists bounded and
    ascending, frame deterministic, depth finite where covered."""
    from shs_gpu import scene_lib
    frame, draws, lights, cull = scene_lib.c4_scene()
    gpu_ctx.upload_lights(lights)
    gpu_ctx.light_cull(cull)
    counts, idx, _ = gpu_ctx.resolve_light_lists()
    assert counts.max() <= cull.max_per_tile and counts.sum() > 0
    for l in np.nonzero(counts)[0][:2000]:
        n = int(counts[l])
        assert np.all(np.diff(idx[l, :n].astype(np.int64)) > 0) and idx[l, n - 1] < len(lights)
    gpu_ctx.render_pbr_forward(frame, draws)
    h1, d1, _ = gpu_ctx.resolve_lib()
    st = gpu_ctx.lib_stats()
    assert st["tri_input"] == 1_000_000
    gpu_ctx.render_pbr_forward(frame, draws)
    h2, d2, _ = gpu_ctx.resolve_lib()
    assert np.array_equal(h1.view(np.uint32), h2.view(np.uint32)) and np.array_equal(d1.view(np.uint32), d2.view(np.uint32))
    cov = d1 < 1.0
    assert cov.sum() > 500_000 and np.isfinite(h1[cov]).all() and (h1[cov][:, :3] <= 1.0).all()


def test_tiled_depth_cull_sharded(oracle_mod):
    """tiled-depth-range culling (mode 2) reads the previous camera pass's depth.  Sharded over
    3 ranks with the interleaved layout (static ownership: a rank keeps the depth of every tile it owns)
    for 3 frames, each rank's own lists equal the oracle's lists over the same depth; the region layout,
    whose rectangles move between passes, is refused instead of reading stale depth."""
    import shs_gpu
    from test_shipped_frames import _owned_light_lists
    count = 3
    frame, draws, lights, cull = _small_c4(2, W=480, H=272)   # 272 % 32 = 16: light tiles inside one bin row
    ref = shs_gpu.Context(0)
    ctxs = [shs_gpu.Context(0) for _ in range(count)]
    try:
        ref.render_pbr_forward(frame, _prepass(draws))
        _, depth, _ = ref.resolve_lib()                      # the depth prepass every frame re-renders
        rc, ri, _ = oracle_mod.light_cull(cull, lights, depth)
        for c in ctxs:
            c.upload_lights(lights)
        for it in range(3):
            for r, c in enumerate(ctxs):
                frame.shard_rank, frame.shard_count = r, count
                cull.shard_rank, cull.shard_count = r, count
                c.render_pbr_forward(frame, _prepass(draws))   # the rank's owned tiles of the prepass
                c.light_cull(cull)
                gc, gi, _ = c.resolve_light_lists()
                own = _owned_light_lists(cull, r, count)
                assert own.any()
                assert np.array_equal(gc[own], rc[own]), f"frame {it} rank {r}: counts differ"
                for l in np.nonzero(own & (rc > 0))[0]:
                    assert np.array_equal(gi[l, :rc[l]], ri[l, :rc[l]]), f"frame {it} rank {r}: list {l}"
        regional = ctxs[0]
        regional.set_shard_layout(True)
        frame.shard_rank, frame.shard_count = 0, count
        cull.shard_rank, cull.shard_count = 0, count
        regional.render_pbr_forward(frame, _prepass(draws))
        with pytest.raises(shs_gpu.ShsError):
            regional.light_cull(cull)
        # at 480x270 a 16-px light tile straddles two bin rows (two ranks' depth): refused as well
        frame2, draws2, _, cull2 = _small_c4(2, W=480, H=270)
        c = ctxs[1]
        frame2.shard_rank, frame2.shard_count = 1, count
        cull2.shard_rank, cull2.shard_count = 1, count
        c.render_pbr_forward(frame2, _prepass(draws2))
        with pytest.raises(shs_gpu.ShsError):
            c.light_cull(cull2)
    finally:
        for c in ctxs + [ref]:
            c.close()
        frame.shard_rank, frame.shard_count = 0, 1
        cull.shard_rank, cull.shard_count = 0, 1
