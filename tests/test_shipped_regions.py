"""Oracle checks of the region-sharded 4K frames `bench.py --config c4|c5 --gpus N` ships (VERDICT r3,
next-round item 1).  The bench's N > 1 default is the REGION layout (SHS_OPT_SHARD_LAYOUT regions,
root share 0.85): every rank owns one rectangle of 32x32 bin tiles and its camera-pass setup skips the
256-triangle blocks whose projected bounds miss it.  At C4's 1M triangles / 4096 setup blocks that skip
predicate does real work, so it is checked here at full size against the oracle:

* 8 contexts on device 0 play the 8 ranks, two consecutive frames each: the first with the pixel-only
  split (no previous pass), the second balanced from the first pass's block bounds;
* each frame is composed on rank 0 through shs_tiles_pack / shs_tiles_unpack (what the RCCL gather
  moves), and compared with the oracle frame: depth and every rank's light lists bit-exact, HDR and
  motion within 1e-5, present bytes equal to PassTonemap of the composed HDR (and to the oracle's
  except where the two HDR values differ within their 1e-5);
* one full-size C4 frame through shs_group (8 contexts, one process, peer-copy gather) in the region
  layout, against the same oracle frame.

References: passes/pass_pbr_forward.hpp:49-214, shaders/vulkan/fp_stress_light_cull.comp:148-266."""
import numpy as np
import pytest

from helpers import assert_depth_bitexact, assert_float_close
from test_regions import _check_layout, _mask, _owned_lists

pytestmark = pytest.mark.gpu

RANKS = 8
ROOT_SHARE = 0.85     # bench.py --root-share default


@pytest.fixture(scope="module")
def c4_ref(oracle_mod):
    from shs_gpu import scene_lib
    frame, draws, lights, cull = scene_lib.c4_scene(3840, 2160)
    rc, ri = oracle_mod.light_cull(cull, lights)[:2]
    rh, rd, rm, _ = oracle_mod.forward_plus(frame, draws, lights, cull, (rc, ri))
    return (frame, draws, lights, cull), (rc, ri), (rh, rd, rm)


@pytest.fixture(scope="module")
def c5_ref(oracle_mod):
    from shs_gpu import scene_lib
    frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160, 2048)
    sm_ref, lvp_ref = oracle_mod.shadow_map(S, sun, casters)
    scene_lib.wire_shadow(draws, lvp_ref)
    rh, rd, rm, _ = oracle_mod.pbr_forward(frame, draws, sm_ref)
    return (frame, draws, casters, sun, S), lvp_ref, (rh, rd, rm)


def _check_composed(oracle_mod, got, ref, present):
    gh, gd, gm = got
    rh, rd, rm = ref
    assert_depth_bitexact(gd, rd)
    assert_float_close(gm, rm, what="motion")
    n = assert_float_close(gh, rh, what="hdr")
    assert np.array_equal(present, oracle_mod.tonemap(gh)[1]), "present staging is not PassTonemap of the composed HDR"
    differ = (present != oracle_mod.tonemap(rh)[1]).any(axis=2)
    hdr_differ = (gh.view(np.uint32) != rh.view(np.uint32)).any(axis=2)[::-1]   # present rows are top-down
    assert not (differ & ~hdr_differ).any(), "present bytes differ where the HDR is bit-identical"
    return n


@pytest.mark.parametrize("cfg", ["c4", "c5"])
def test_region_sharded_4k_frames_compose_to_oracle(oracle_mod, c4_ref, c5_ref, cfg):
    import torch
    import shs_gpu
    if cfg == "c4":
        (frame, draws, lights, cull), (rc, ri), ref = c4_ref
    else:
        (frame, draws, casters, sun, S), lvp_ref, ref = c5_ref
    W, H = frame.width, frame.height
    ctxs = [shs_gpu.Context(0) for _ in range(RANKS)]
    layouts = []
    try:
        for c in ctxs:
            c.set_shard_layout(True)
            c.set_shard_root_share(ROOT_SHARE)
            c.fuse_tonemap(1.0, 2.2, ldr=False, present=True)     # bench.py's N > 1 frame
            if cfg == "c4":
                c.upload_lights(lights)
            else:
                c.set_shadow_footprint(True)   # bench.py's C5: each rank's shadow pass covers its own footprint
        for it in range(2):
            lib_bufs, pres_bufs, regs, shadow_tiles = [None] * RANKS, [None] * RANKS, [], []
            got_counts = np.zeros_like(rc) if cfg == "c4" else None
            listed = np.zeros(rc.shape[0], bool) if cfg == "c4" else None
            for r, c in enumerate(ctxs):
                frame.shard_rank, frame.shard_count = r, RANKS
                if cfg == "c4":
                    cull.shard_rank, cull.shard_count = r, RANKS
                    c.light_cull(cull)
                else:
                    lvp = c.render_shadow_map(S, sun, casters)
                    assert np.array_equal(lvp.view(np.uint32), lvp_ref.view(np.uint32))
                c.render_pbr_forward(frame, draws)
                if cfg == "c5":
                    sx0, sy0, sx1, sy1 = c.shadow_region()
                    shadow_tiles.append(max(0, sx1 - sx0 + 1) * max(0, sy1 - sy0 + 1))
                reg = c.shard_regions(RANKS)
                regs.append(reg)
                if cfg == "c4":
                    counts, idx, _ = c.resolve_light_lists()
                    own = _owned_lists(cull, reg[r], H)
                    assert np.array_equal(counts[own], rc[own]), f"frame {it} rank {r}: light counts differ"
                    for li in np.nonzero(own & (rc > 0))[0]:
                        assert np.array_equal(idx[li, :rc[li]], ri[li, :rc[li]]), f"frame {it} rank {r}: list {li}"
                    got_counts[own] = counts[own]
                    listed |= own
                if r > 0:
                    for target, keep in ((c.TARGET_LIB, lib_bufs), (c.TARGET_LIB_PRESENT, pres_bufs)):
                        words = c.tiles_packed_words(target, RANKS)
                        assert c.tiles_rank_words(target, r, RANKS) <= words
                        buf = torch.zeros(max(words, 1), dtype=torch.int32, device="cuda:0")
                        torch.cuda.synchronize()   # torch's fill runs on its own stream: done before the pack
                        c.tiles_pack(target, r, RANKS, buf.data_ptr())
                        keep[r] = buf
                c.synchronize_lib()
            assert all(g == regs[0] for g in regs), f"frame {it}: ranks disagree on the layout"
            _check_layout(regs[0], W, H)
            layouts.append(regs[0])
            root = ctxs[0]
            for r in range(1, RANKS):
                if root.tiles_rank_words(root.TARGET_LIB, r, RANKS) > 0:
                    root.tiles_unpack(root.TARGET_LIB, r, RANKS, lib_bufs[r].data_ptr())
                    root.tiles_unpack(root.TARGET_LIB_PRESENT, r, RANKS, pres_bufs[r].data_ptr())
            got = root.resolve_lib()
            _, present = root.resolve_ldr()
            n = _check_composed(oracle_mod, got, ref, present)
            if cfg == "c4":
                assert listed.all(), "some light list has no owner"
                assert np.array_equal(got_counts, rc)
            owned = [int(_mask(W, H, reg).sum()) for reg in regs[0]]
            print(f"{cfg} frame {it}: layout {regs[0]}, owned px {owned}, shadow tiles {shadow_tiles}, "
                  f"{n} HDR channels not bit-identical")
            if cfg == "c5":
                assert max(shadow_tiles) < 64 * 64, "a rank rendered the whole shadow map"
    finally:
        for c in ctxs:
            c.close()
        frame.shard_rank, frame.shard_count = 0, 1
        if cfg == "c4":
            cull.shard_rank, cull.shard_count = 0, 1
    # the first frame splits by pixels only; the second is balanced from the block bounds
    assert layouts[0] != layouts[1], "the second frame did not rebalance"


def test_group_gather_region_c4_4k_matches_oracle(oracle_mod, c4_ref):
    """shs_group (one host process, 8 contexts on device 0, peer-copy gather into rank 0), region layout,
    two frames: the gathered full-size C4 frame (HDR + depth + motion, and the present staging) equals
    the oracle frame."""
    from shs_gpu.group import Group
    (frame, draws, lights, cull), (rc, ri), ref = c4_ref
    g = Group([0] * RANKS)
    try:
        g.set_shard_layout(True, ROOT_SHARE)
        g.upload_lights(lights)
        g.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
        for it in range(2):
            g.light_cull(cull)
            g.render_pbr_forward(frame, draws)
            g.gather(g.root.TARGET_LIB)
            g.gather(g.root.TARGET_LIB_PRESENT)
            got = g.root.resolve_lib()
            _, present = g.root.resolve_ldr()
            n = _check_composed(oracle_mod, got, ref, present)
            print(f"group c4 frame {it}: {n} HDR channels not bit-identical")
    finally:
        g.close()
