"""Oracle checks of exactly what bench.py times and ships.

* C2: the bench's timed steps are batches of bench.LEGACY_FRAMES['c2'] (128) camera poses at 1920x1080 (bench.batch_poses); pose
  sets 0 and 3 are rendered as one batch each, exactly as the timed loop does (prepare_batch +
  render_batch_prepared), and every frame is compared with the oracle: depth bit-exact, colour under
  the pre-truncation rule with that frame's own prequant floats.  The same batches rendered without
  the prequant plane (the bench's flags) are byte-identical.
* C4 / C5 at N = 8: the frame bench.py --gpus 8 ships is 8 tile shards, each rendered with the fused
  tonemap into the present staging, composed by shs_tiles_pack / shs_tiles_unpack.  Rendered here as
  8 shards in turn on one GPU, composed, and compared with the oracle frames: depth and light lists
  bit-exact, HDR and motion within 1e-5, present bytes equal to the oracle's PassTonemap of the GPU HDR
  and to that of the oracle HDR except where the two HDR values differ (a tonemap threshold between
  two values 1e-5 apart)."""
import numpy as np
import pytest

from helpers import assert_color_parity, assert_depth_bitexact, assert_float_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pose_set", [0, 3])
def test_c2_bench_batch_every_frame_vs_oracle(oracle_mod, pose_set):
    import dataclasses
    import bench
    import shs_gpu
    F = bench.LEGACY_FRAMES["c2"]
    frame, sets = bench.batch_poses("c2", F)
    fds = sets[pose_set]
    assert (frame.width, frame.height) == (1920, 1080) and len(fds) == F
    ctx = shs_gpu.Context(0)
    try:
        ctx.render_batch_prepared(ctx.prepare_batch(frame, fds))          # the bench's flags
        plain = [ctx.resolve_frame(k) for k in range(F)]
        pframe = dataclasses.replace(frame, prequant=True)
        ctx.render_batch_prepared(ctx.prepare_batch(pframe, fds))
        boundary = 0
        for k in range(F):
            c, z = ctx.resolve_frame(k)
            pq = ctx.resolve_prequant(k)
            assert np.array_equal(c, plain[k][0]) and np.array_equal(z.view(np.uint32), plain[k][1].view(np.uint32)), \
                f"frame {k}: the prequant plane changed the image"
            rc, rd, rpq = oracle_mod.render_legacy(1920, 1080, fds[k], threads=16, prequant=True)
            assert_depth_bitexact(z, rd)
            boundary += assert_color_parity(c, rc, pq, rpq)
        print(f"pose set {pose_set}: {F} frames exact, {boundary} truncation-boundary bytes")
    finally:
        ctx.close()


def _owned_light_lists(cull, rank, count):
    """Light tiles (cull.tile_size px, rows down) covering a pixel of one of rank's 32x32 GPU tiles (rows
    up, tile % count == rank): a light tile straddling two bin rows belongs to both owners."""
    tx, ty = cull.tiles
    ts, H = cull.tile_size, cull.height
    ly, lx = np.mgrid[0:ty, 0:tx]
    top = H - 1 - ly * ts
    bot = np.maximum(top - ts + 1, 0)
    bw = (cull.width + 31) // 32
    own = ((top // 32) * bw + lx * ts // 32) % count == rank
    own |= ((bot // 32) * bw + lx * ts // 32) % count == rank
    return own.reshape(-1)


@pytest.mark.parametrize("cfg", ["c4", "c5"])
def test_sharded_4k_frame_composes_to_oracle(oracle_mod, cfg):
    import torch
    import shs_gpu
    from shs_gpu import scene_lib
    count = 8
    if cfg == "c4":
        frame, draws, lights, cull = scene_lib.c4_scene(3840, 2160)
        rcounts, ridx = oracle_mod.light_cull(cull, lights)[:2]
        rh, rd, rm, _ = oracle_mod.forward_plus(frame, draws, lights, cull, (rcounts, ridx))
    else:
        frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160, 2048)
        sm_ref, lvp_ref = oracle_mod.shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp_ref)
        rh, rd, rm, _ = oracle_mod.pbr_forward(frame, draws, sm_ref)
    ctxs, lib_bufs, pres_bufs = [], [], []
    got_counts = np.zeros(cull.n_lists, np.uint32) if cfg == "c4" else None
    got_idx = np.zeros((cull.n_lists, cull.max_per_tile), np.uint32) if cfg == "c4" else None
    try:
        for r in range(count):
            ctx = shs_gpu.Context(0)
            frame.shard_rank, frame.shard_count = r, count
            if cfg == "c4":
                cull.shard_rank, cull.shard_count = r, count
                ctx.upload_lights(lights)
                ctx.light_cull(cull)
                c, i, _ = ctx.resolve_light_lists()
                own = _owned_light_lists(cull, r, count)
                assert (c[~own] == 0).all(), "a rank built lists of tiles it does not own"
                got_counts[own] = c[own]
                got_idx[own] = i[own]
            else:
                lvp = ctx.render_shadow_map(S, sun, casters)
                assert np.array_equal(lvp.view(np.uint32), lvp_ref.view(np.uint32))
            ctx.fuse_tonemap(1.0, 2.2, ldr=False, present=True)    # bench.py's N > 1 frame
            ctx.render_pbr_forward(frame, draws)
            for target, keep in ((ctx.TARGET_LIB, lib_bufs), (ctx.TARGET_LIB_PRESENT, pres_bufs)):
                buf = torch.zeros(ctx.tiles_packed_words(target, count), dtype=torch.int32, device="cuda:0")
                torch.cuda.synchronize()   # torch's fill runs on its own stream: done before the pack
                ctx.tiles_pack(target, r, count, buf.data_ptr())
                keep.append(buf)
            ctx.synchronize_lib()
            if r == 0:
                ctxs.append(ctx)      # rank 0 composes
            else:
                ctx.close()
        frame.shard_rank, frame.shard_count = 0, 1
        root = ctxs[0]
        for r in range(1, count):
            root.tiles_unpack(root.TARGET_LIB, r, count, lib_bufs[r].data_ptr())
            root.tiles_unpack(root.TARGET_LIB_PRESENT, r, count, pres_bufs[r].data_ptr())
        gh, gd, gm = root.resolve_lib()
        _, gp = root.resolve_ldr()
    finally:
        for c in ctxs:
            c.close()
    if cfg == "c4":
        assert np.array_equal(got_counts, rcounts), "composed light-list counts differ"
        for l in np.nonzero(rcounts)[0]:
            assert np.array_equal(got_idx[l, :rcounts[l]], ridx[l, :rcounts[l]]), f"light list {l} differs"
    assert_depth_bitexact(gd, rd)
    assert_float_close(gm, rm, what="motion")
    n = assert_float_close(gh, rh, what="hdr")
    _, p_gpu_hdr = oracle_mod.tonemap(gh)
    assert np.array_equal(gp, p_gpu_hdr), "present staging is not PassTonemap of the composed HDR"
    _, p_ref = oracle_mod.tonemap(rh)
    differ = (gp != p_ref).any(axis=2)
    hdr_differ = (gh.view(np.uint32) != rh.view(np.uint32)).any(axis=2)[::-1]   # present rows are top-down
    assert not (differ & ~hdr_differ).any(), "present bytes differ where the HDR is bit-identical"
    assert np.abs(gp.astype(np.int16) - p_ref.astype(np.int16)).max() <= 1
    print(f"{cfg} 8 shards composed: {n} HDR channels not bit-identical, {int(differ.sum())} present px at a threshold")
