"""Region layout of tile-sharded library frames (SHS_OPT_SHARD_LAYOUT = SHS_SHARD_REGIONS, shs_shard.hpp):
every rank owns one rectangle of 32x32 bin tiles from a cost-balanced bisection that each rank derives
from its own previous camera pass.  The composed frame must equal the oracle exactly as the interleaved
layout's does -- depth and light lists bit-exact, HDR / motion within 1e-5, present bytes exact -- on
the first frame (pixel-only split) and on later ones (split from the previous pass's block bounds), and
the rectangles must tile the bin grid with every rank agreeing on them."""
import numpy as np
import pytest

from helpers import assert_depth_bitexact, assert_float_close

pytestmark = pytest.mark.gpu

T = 32


def _tiles(w, h):
    return (w + T - 1) // T, (h + T - 1) // T


def _check_layout(regions, w, h):
    tx, ty = _tiles(w, h)
    cover = np.zeros((ty, tx), np.int32)
    for x0, y0, x1, y1 in regions:
        if x1 >= x0 and y1 >= y0:
            assert 0 <= x0 and x1 < tx and 0 <= y0 and y1 < ty, (x0, y0, x1, y1)
            cover[y0:y1 + 1, x0:x1 + 1] += 1
    assert (cover == 1).all(), "regions do not tile the bin grid exactly"


def _mask(w, h, rect):
    x0, y0, x1, y1 = rect
    m = np.zeros((h, w), bool)
    if x1 >= x0 and y1 >= y0:
        m[y0 * T:(y1 + 1) * T, x0 * T:(x1 + 1) * T] = True
    return m


def _owned_lists(cull, rect, h):
    """The light-list tiles a rank builds: list tile (lx, ly) (rows top-down in list space) is built by
    the owners of the bin tiles its top and bottom pixel rows (y up) fall in (light_list_owned)."""
    x0, y0, x1, y1 = rect
    ts = cull.tile_size
    ltx = (cull.width + ts - 1) // ts
    lty = (cull.height + ts - 1) // ts
    own = np.zeros(ltx * lty, bool)
    for ly in range(lty):
        top_up = h - 1 - ly * ts
        bot_up = max(top_up - ts + 1, 0)
        for lx in range(ltx):
            bx = lx * ts // T
            own[ly * ltx + lx] = x0 <= bx <= x1 and (y0 <= top_up // T <= y1 or y0 <= bot_up // T <= y1)
    return own


@pytest.mark.parametrize("count", [2, 3, 8])
def test_region_shards_forward_plus_match_oracle(oracle_mod, count):
    """A C4-like Forward+ frame (light cull + PassPBRForward, fused tonemap into the present staging),
    region-sharded over `count` contexts for three frames: the composed depth / HDR / motion / present
    bytes and every rank's own light lists equal the oracle's."""
    import shs_gpu
    from shs_gpu import scene_lib
    W, H = 640, 360
    frame, draws, lights, cull = scene_lib.c4_scene(W, H, n_objects=80, tris_per_object=600)
    rc, ri = oracle_mod.light_cull(cull, lights)[:2]
    rh, rd, rm, _ = oracle_mod.forward_plus(frame, draws, lights, cull, (rc, ri))
    ctxs = [shs_gpu.Context(0) for _ in range(count)]
    layouts = []
    try:
        for c in ctxs:
            c.set_shard_layout(True)
            c.upload_lights(lights)
            c.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
        for it in range(3):
            gh, gd, gm = np.zeros_like(rh), np.zeros_like(rd), np.zeros_like(rm)
            gp = None
            regs = []
            for r, c in enumerate(ctxs):
                frame.shard_rank, frame.shard_count = r, count
                cull.shard_rank, cull.shard_count = r, count
                c.light_cull(cull)
                c.render_pbr_forward(frame, draws)
                h, d, m = c.resolve_lib()
                _, pres = c.resolve_ldr()
                reg = c.shard_regions(count)
                regs.append(reg)
                own = _mask(W, H, reg[r])
                gh[own], gd[own], gm[own] = h[own], d[own], m[own]
                if gp is None:
                    gp = np.zeros_like(pres)
                own_p = own[::-1]   # present staging rows top-down
                gp[own_p] = pres[own_p]
                counts, idx, _ = c.resolve_light_lists()
                lo = _owned_lists(cull, reg[r], H)
                assert np.array_equal(counts[lo], rc[lo]), f"rank {r}: light counts differ"
                for li in np.nonzero(lo)[0]:
                    n = int(rc[li])
                    assert np.array_equal(idx[li, :n], ri[li, :n]), f"rank {r}: light list {li} differs"
            assert all(g == regs[0] for g in regs), "ranks disagree on the layout"
            _check_layout(regs[0], W, H)
            layouts.append(regs[0])
            assert_depth_bitexact(gd, rd)
            assert_float_close(gm, rm, what="motion")
            assert_float_close(gh, rh, what="hdr")
            # present bytes: PassTonemap of the composed HDR exactly; against the oracle's, different only
            # where the HDR itself differs within its 1e-5 (test_shipped_frames' rule)
            assert np.array_equal(gp, oracle_mod.tonemap(gh)[1]), "present staging is not PassTonemap of the HDR"
            differ = (gp != oracle_mod.tonemap(rh)[1]).any(axis=2)
            hdr_differ = (gh.view(np.uint32) != rh.view(np.uint32)).any(axis=2)[::-1]
            assert not (differ & ~hdr_differ).any(), "present bytes differ where the HDR is bit-identical"
    finally:
        for c in ctxs:
            c.close()
        frame.shard_rank, frame.shard_count = 0, 1
        cull.shard_rank, cull.shard_count = 0, 1
    # the same frame again: the balanced layout is stable from the second frame on
    assert layouts[1] == layouts[2]


def test_region_gather_device_present(oracle_mod):
    """shard.gather_frame_device over a region layout (ranks of different packed sizes, point-to-point
    receives of exactly each rank's size): the composed present staging equals the unsharded frame's,
    for two frames (the second with the balanced layout)."""
    import torch
    import shs_gpu
    from shs_gpu import scene_lib, shard
    from test_gather_gpu import _RankZeroDist
    count = 4
    ctxs = [shs_gpu.Context(0) for _ in range(count)]
    full = shs_gpu.Context(0)
    out = None
    try:
        for c in ctxs:
            c.set_shard_layout(True)
            c.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
        root = ctxs[0]
        sizes_seen = set()
        for yaw in (0.0, 0.0, 25.0):
            frame, draws, _, _, _ = scene_lib.c5_scene(352, 200, yaw=yaw)
            full.render_pbr_forward(frame, draws)
            full.tonemap(1.0, 2.2, ldr=False, present=True)
            _, want = full.resolve_ldr()
            packed = [None]
            for r in range(1, count):
                c = ctxs[r]
                frame.shard_rank, frame.shard_count = r, count
                c.render_pbr_forward(frame, draws)
                b = torch.zeros(c.tiles_packed_words(c.TARGET_LIB_PRESENT, count), dtype=torch.int32, device="cuda:0")
                torch.cuda.synchronize()   # torch's fill runs on its own stream: done before the pack
                c.tiles_pack(c.TARGET_LIB_PRESENT, r, count, b.data_ptr())
                c.synchronize_lib()
                packed.append(b)
                sizes_seen.add(c.tiles_rank_words(c.TARGET_LIB_PRESENT, r, count))
            frame.shard_rank, frame.shard_count = 0, count
            root.render_pbr_forward(frame, draws)
            out = shard.gather_frame_device(_RankZeroDist(count, packed), root, root.TARGET_LIB_PRESENT, out=out)
            torch.cuda.synchronize()
            _, got = root.resolve_ldr()
            assert np.array_equal(got, want), f"yaw {yaw}: composed frame differs"
        assert len(sizes_seen) > 1, "region ranks all had the same size"
    finally:
        for c in ctxs + [full]:
            c.close()


def test_region_more_ranks_than_tiles():
    """A 40x20 frame (2 x 1 bin tiles) over 5 region ranks: ranks without tiles render and pack
    nothing, and the two owners compose the unsharded frame."""
    import shs_gpu
    from shs_gpu import scene_lib
    count = 5
    frame, draws, _, _, _ = scene_lib.c5_scene(40, 20)
    full = shs_gpu.Context(0)
    ctxs = [shs_gpu.Context(0) for _ in range(count)]
    try:
        full.render_pbr_forward(frame, draws)
        fh, fd, fm = full.resolve_lib()
        for _ in range(2):
            gh, gd = np.zeros_like(fh), np.zeros_like(fd)
            for r, c in enumerate(ctxs):
                c.set_shard_layout(True)
                frame.shard_rank, frame.shard_count = r, count
                c.render_pbr_forward(frame, draws)
                h, d, _ = c.resolve_lib()
                reg = c.shard_regions(count)
                _check_layout(reg, 40, 20)
                own = _mask(40, 20, reg[r])
                gh[own], gd[own] = h[own], d[own]
                words = c.tiles_rank_words(c.TARGET_LIB, r, count)
                assert (words == 0) == (not own.any())
            assert np.array_equal(gd.view(np.uint32), fd.view(np.uint32))
            assert np.array_equal(gh.view(np.uint32), fh.view(np.uint32))
    finally:
        for c in ctxs + [full]:
            c.close()
