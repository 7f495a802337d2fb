"""Frame batches (shs_render_legacy_batch): one k_setup + k_raster pair renders n_frames independent
frames; every frame must be bit-identical to the frame shs_render_legacy renders from the same draws
(and hence to the oracle).  Covers scan mode (C2 poses), bin mode with spill (C3 + tiny bin
capacity), ghost fragments of unbounded slivers in both modes, shards, and the validation rules."""
import numpy as np
import pytest

from helpers import FLT_MAX, assert_color_parity, assert_depth_bitexact
from test_gpu_parity import _hair_soup, _identity_draw, _ndc_soup

pytestmark = pytest.mark.gpu


def _poses(n, shading=3, width=1920, height=1080):
    from shs_gpu import scene
    out = []
    for k in range(n):
        frame, draws = scene.monkey_scene(width, height, shading, yaw=-20.0 + 5.5 * k, pitch=-4.0 + 1.5 * k,
                                          rotation=13.0 * k)
        out.append(draws)
    return frame, out


def _singles(ctx, frame, frames_draws):
    res = []
    for d in frames_draws:
        ctx.render(frame, d)
        c, z = ctx.resolve()
        res.append((c, z, ctx.stats()))
    return res


def _owned_mask(frame):
    """Screen-row mask of the pixels a shard owns (32x32 tiles, tile % count == rank)."""
    T = 32
    ty, tx = np.mgrid[0:frame.height, 0:frame.width] // T
    tiles_x = (frame.width + T - 1) // T
    return (ty * tiles_x + tx) % frame.shard_count == frame.shard_rank


def _assert_batch_equals_singles(ctx, frame, frames_draws, before_batch=None):
    singles = _singles(ctx, frame, frames_draws)
    if before_batch is not None:
        before_batch(ctx)
    ctx.render_batch(frame, frames_draws)
    st = ctx.stats()
    m = _owned_mask(frame)   # a shard writes only its own tiles; the rest of the buffer is stale
    for k, (c1, z1, _) in enumerate(singles):
        c, z = ctx.resolve_frame(k)
        if frame.shard_count > 1:
            z, z1 = np.where(m, z, 0.0), np.where(m, z1, 0.0)
            mc = m[::-1][..., None]   # colour is in canvas rows
            c, c1 = np.where(mc, c, 0), np.where(mc, c1, 0)
        assert np.array_equal(z.view(np.uint32), z1.view(np.uint32)), f"frame {k}: depth differs from the single render"
        assert np.array_equal(c, c1), f"frame {k}: colour differs from the single render"
    assert st["tri_input"] == sum(s["tri_input"] for _, _, s in singles)
    assert st["covered_pixels"] == sum(s["covered_pixels"] for _, _, s in singles)
    return singles, st


@pytest.mark.parametrize("n_frames", [1, 2, 7, 16])
def test_batch_c2_poses_match_single_frames(gpu_ctx, n_frames):
    frame, fd = _poses(n_frames)
    _assert_batch_equals_singles(gpu_ctx, frame, fd)


def test_batch_geometry_sequence(gpu_ctx):
    """One context through batches whose frame size (inside and across the bin-tile grid), frame
    count and shard change from call to call: every frame equals its single render."""
    for W, H, n, rank, count in [(322, 181, 3, 0, 1), (322, 176, 5, 0, 1), (33, 17, 2, 0, 1), (322, 181, 4, 1, 3),
                                 (322, 181, 1, 0, 1), (1, 1, 3, 0, 1), (322, 181, 6, 0, 1)]:
        frame, fd = _poses(n, width=W, height=H)
        frame.shard_rank, frame.shard_count = rank, count
        _assert_batch_equals_singles(gpu_ctx, frame, fd)


def test_batch_frames_match_oracle(gpu_ctx, oracle_mod):
    """Every frame of a mixed-shading 640x480 batch against the CPU oracle directly (colour with each
    frame's own pre-truncation floats)."""
    from shs_gpu import scene
    fds = []
    for k, sh in enumerate([3, 2, 1, 0, 3]):
        frame, draws = scene.monkey_scene(640, 480, sh, yaw=7.0 * k - 10.0, pitch=2.0 * k, rotation=31.0 * k,
                                          cam_pos=(0.0, 5.0, -12.0))
        fds.append(draws)
    frame.prequant = True
    gpu_ctx.render_batch(frame, fds)
    for k in range(len(fds)):
        c, z = gpu_ctx.resolve_frame(k)
        pq = gpu_ctx.resolve_prequant(k)
        rc, rd, rpq = oracle_mod.render_legacy(frame.width, frame.height, fds[k], threads=8, prequant=True)
        assert_depth_bitexact(z, rd)
        assert_color_parity(c, rc, pq, rpq)


@pytest.mark.parametrize("mode", [1, 2], ids=["scan", "bins"])
def test_batch_shared_varyings_static_scene(oracle_mod, mode):
    """A static scene under a batch of camera poses (same meshes, shading and model matrices in every
    frame) stores its corner varyings once for the batch (RF_SHARED_VARY); each frame still shades with
    its own draw uniforms -- here a moving camera position and light -- so every frame is checked
    against the oracle directly.  Both raster modes."""
    import shs_gpu
    from shs_gpu import scene
    fds = []
    for k in range(5):
        cam = (0.8 * k - 1.5, 5.0 - 0.4 * k, -18.0 + 0.7 * k)
        frame, draws = scene.monkey_scene(480, 320, 3 if mode == 1 else 2, yaw=4.0 * k - 8.0, pitch=1.5 * k - 3.0,
                                          rotation=25.0, cam_pos=cam)
        for d in draws:
            d.light_dir = np.asarray([0.3 * k - 0.6, -1.0, 0.5 + 0.1 * k], np.float32)
        fds.append(draws)
    frame.prequant = True
    ctx = shs_gpu.Context(0)
    try:
        ctx.set_raster_mode(mode)
        ctx.render_batch(frame, fds)
        for k in range(len(fds)):
            c, z = ctx.resolve_frame(k)
            pq = ctx.resolve_prequant(k)
            rc, rd, rpq = oracle_mod.render_legacy(frame.width, frame.height, fds[k], threads=8, prequant=True)
            assert_depth_bitexact(z, rd)
            assert_color_parity(c, rc, pq, rpq)
    finally:
        ctx.close()


def test_batch_c3_bins_with_spill(oracle_mod):
    """C3 grid (bin mode) at 960x540, three poses, bin capacity 4: most entries spill to the shared
    spill list whose entries carry the frame's bin tile."""
    import shs_gpu
    from shs_gpu import scene
    fds = []
    for k in range(3):
        frame, draws = scene.grid_scene(960, 540, n=4, yaw=-6.0 + 6.0 * k)
        fds.append(draws)
    ctx = shs_gpu.Context(0)
    try:
        ctx.set_raster_mode(2)
        # the context grows the capacity to the fullest tile it has seen: shrink it again for the batch
        _, st = _assert_batch_equals_singles(ctx, frame, fds, before_batch=lambda c: c.set_bin_capacity(4))
        assert st["spilled"] > 0
        c, z = ctx.resolve_frame(2)
        rc, rd, _ = oracle_mod.render_legacy(frame.width, frame.height, fds[2], threads=8)
        assert_depth_bitexact(z, rd)
    finally:
        ctx.close()


@pytest.mark.parametrize("mode", [1, 2], ids=["scan", "bins"])
def test_batch_hair_slivers_ghost_fragments(mode):
    """Unbounded slivers emit ghost fragments tagged with their frame (ghost waves in scan mode, the
    sliver list + k_ghost in bin mode); frames with different slivers must not see each other's."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    W, H = 400, 300
    fds = []
    for seed in (99, 100, 101):
        rng = np.random.default_rng(seed)
        pos, nrm = _hair_soup(rng, W, H, 1500)
        fds.append([_identity_draw(Mesh(pos, nrm), 3)])
    ctx = shs_gpu.Context(0)
    try:
        ctx.set_raster_mode(mode)
        _, st = _assert_batch_equals_singles(ctx, shs_gpu.Frame(W, H), fds)
        assert st["ghost_fragments"] > 0
    finally:
        ctx.close()


def test_batch_sharded_frames(gpu_ctx):
    """Shard ownership applies to every frame of the batch."""
    import shs_gpu
    _, fd = _poses(3, width=640, height=480)
    frame = shs_gpu.Frame(640, 480, shard_rank=1, shard_count=3)
    _assert_batch_equals_singles(gpu_ctx, frame, fd)


def test_batch_soup_multi_draw_device_table(gpu_ctx):
    """2 draws x 4 frames = 8 draws: the device draw table (more than fit in kernel arguments)."""
    import shs_gpu
    from shs_gpu.scene import Mesh
    W, H = 333, 241
    fds = []
    for seed in range(4):
        rng = np.random.default_rng(40 + seed)
        pos, nrm = _ndc_soup(rng, W, H, 600)
        fds.append([_identity_draw(Mesh(pos[:300], nrm[:300]), seed % 4), _identity_draw(Mesh(pos[300:], nrm[300:]), 3)])
    _assert_batch_equals_singles(gpu_ctx, shs_gpu.Frame(W, H), fds)


def test_batch_validation(gpu_ctx):
    import shs_gpu
    from shs_gpu import ShsError
    from shs_gpu.scene import Mesh
    frame, fd = _poses(2, width=320, height=240)
    rng = np.random.default_rng(1)
    pos, nrm = _ndc_soup(rng, 320, 240, 50)
    with pytest.raises(ShsError):   # unequal triangle counts across frames
        gpu_ctx.render_batch(frame, [fd[0], [_identity_draw(Mesh(pos, nrm))]])
    gpu_ctx.render_batch(frame, fd)
    with pytest.raises(ShsError):
        gpu_ctx.resolve_frame(2)
    c, z = gpu_ctx.resolve_frame(1)
    assert (z < FLT_MAX).sum() > 0


def test_legacy_pipeline_matches_unpipelined():
    """SHS_OPT_LEGACY_PIPELINE (k_pipe: batch k's raster in batch k + 1's launch, the last one at the
    flush): a sequence of C2-sized batches -- consecutive batches, a resolve between two of them (a
    flush), a frame-size change (the framebuffers grow: the pending raster is flushed first), a
    single-frame render in between (not pipelined) -- resolves to byte-identical frames, and the
    statistics of the last batch agree."""
    import shs_gpu
    import bench
    frame, sets = bench.batch_poses("c2", 16)
    small, ssets = bench.batch_poses("c1", 16)
    ref, pip = shs_gpu.Context(0), shs_gpu.Context(0)
    try:
        pip.set_legacy_pipeline(True)
        plan = [(frame, sets[0]), (frame, sets[1]), "resolve", (frame, sets[2]), (frame, sets[3]), (small, ssets[0]),
                "resolve", (small, ssets[1]), ("single", sets[0][3]), (frame, sets[1]), (frame, sets[2]),
                (frame, sets[3])]
        for step in plan:
            if step == "resolve":
                for k in (0, 7, 15):
                    a, b = ref.resolve_frame(k), pip.resolve_frame(k)
                    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32)), k
                continue
            if step[0] == "single":
                ref.render(frame, step[1])
                pip.render(frame, step[1])
                continue
            fr, fds = step
            ref.render_batch_prepared(ref.prepare_batch(fr, fds))
            pip.render_batch_prepared(pip.prepare_batch(fr, fds))
        # the framebuffers grow (32 frames) while the previous batch's raster is pending --
        # enqueue_frame flushes it before the reallocation
        frame32, sets32 = bench.batch_poses("c2", 32)
        ref.render_batch_prepared(ref.prepare_batch(frame32, sets32[0]))
        pip.render_batch_prepared(pip.prepare_batch(frame32, sets32[0]))
        for k in range(32):
            a, b = ref.resolve_frame(k), pip.resolve_frame(k)
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32)), k
        assert ref.stats() == pip.stats()
    finally:
        ref.close()
        pip.close()


def test_legacy_pipeline_unpack_after_pending_raster():
    """peers' tiles unpacked into a pipelined legacy frame whose raster is still pending land
    after that raster (shs_tiles_unpack flushes it first), so the raster's clear strips cannot overwrite
    them: the owned pixels of rank 1 of 2 hold the unpacked words, the others the rendered frame."""
    import torch
    import shs_gpu
    import bench
    frame, sets = bench.batch_poses("c2", 16)
    ref, pip = shs_gpu.Context(0), shs_gpu.Context(0)
    try:
        pip.set_legacy_pipeline(True)
        ref.render_batch_prepared(ref.prepare_batch(frame, sets[0]))
        rc, rd = ref.resolve_frame(0)
        pip.render_batch_prepared(pip.prepare_batch(frame, sets[0]))   # its raster is pending now
        words = pip.tiles_rank_words(pip.TARGET_LEGACY, 1, 2)
        buf = torch.full((words,), 0x5A5A5A5A, dtype=torch.int32, device="cuda:0")
        torch.cuda.synchronize()
        pip.tiles_unpack(pip.TARGET_LEGACY, 1, 2, buf.data_ptr())
        gc, gd = pip.resolve_frame(0)
        W, H = frame.width, frame.height
        tx = (W + 31) // 32
        owned = int(((np.arange(H)[:, None] // 32 * tx + np.arange(W)[None, :] // 32) % 2 == 1).sum())
        cw = np.ascontiguousarray(gc).view(np.uint32).reshape(H, W)
        dw = gd.view(np.uint32)
        assert int((cw == 0x5A5A5A5A).sum()) == owned and int((dw == 0x5A5A5A5A).sum()) == owned
        rcw = np.ascontiguousarray(rc).view(np.uint32).reshape(H, W)
        assert np.array_equal(cw[cw != 0x5A5A5A5A], rcw[cw != 0x5A5A5A5A])
        assert np.array_equal(dw[dw != 0x5A5A5A5A], rd.view(np.uint32)[dw != 0x5A5A5A5A])
    finally:
        ref.close()
        pip.close()
