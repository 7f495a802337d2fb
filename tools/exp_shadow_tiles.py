"""The C5 shadow pass's raster at shard r of N (region layout, shadow footprint on; SHS_OPT_TIMELINE 2):
span, busy tiles, candidates and pairs, and per workgroup its longest tile -- bin-list entries, rounds,
staging passes, staged candidates, pairs, gather time -- what bounds the shadow raster of a rank.
usage (GPU box): python tools/exp_shadow_tiles.py [N] [ranks, e.g. 3,0] [top]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
RANKS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [3]
TOP = int(sys.argv[3]) if len(sys.argv) > 3 else 6
for R in RANKS:
    frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160, 2048)
    ctx = shs_gpu.Context(0)
    if N > 1:
        ctx.set_shard_layout(True)
        frame.shard_rank, frame.shard_count = R, N
    ctx.set_shadow_footprint(True)
    lvp = ctx.render_shadow_map(S, sun, casters)
    scene_lib.wire_shadow(draws, lvp)
    prep = ctx.prepare_lib(frame, draws)
    ctx.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
    for _ in range(6):
        ctx.render_shadow_map(S, sun, casters)
        ctx.render_pbr_forward_prepared(prep)
    ctx.synchronize_lib()
    ctx.set_timeline(True, shadow=True)
    for rep in range(2):
        ctx.render_shadow_map(S, sun, casters)
        ctx.render_pbr_forward_prepared(prep)
        ctx.synchronize_lib()
        t = ctx.lib_debug_timeline().astype(np.int64)
        F = {k: i for i, k in enumerate(ctx.LIB_TIMELINE_FIELDS)}
        live = t[:, F["start"]] > 0
        t = t[live]
        st = t[:, F["start"]] - t[:, F["start"]].min()
        en = t[:, F["end"]] - t[:, F["start"]].min()
        dur = en - st
        mt = t[:, F["max_tile"]]
        print(f"C5 shadow rank {R}/{N} rep {rep}: {len(t)} raster workgroups, span {en.max() / 100:.1f} us; busy tiles "
              f"{t[:, F['n_busy']].sum()}, candidates {t[:, F['n_cand']].sum()}, pairs {t[:, F['n_pairs']].sum()}, "
              f"passes {t[:, F['chunks']].sum()}", flush=True)
        print(f"  workgroup us: median {np.median(dur) / 100:.1f} p90 {np.percentile(dur, 90) / 100:.1f} max {dur.max() / 100:.1f}; "
              f"longest tile per wg: median {np.median(mt) / 100:.1f} p90 {np.percentile(mt, 90) / 100:.1f} "
              f"max {mt.max() / 100:.1f}", flush=True)
        tw = S // 32
        for i in np.argsort(-mt)[:TOP]:
            r = t[i]
            rt = int(r[F["mt_rt"]])
            print(f"  wg {i:4d}: tile {rt} (x {rt % tw * 32}, y {rt // tw * 8}) {mt[i] / 100:.1f} us; entries {r[F['mt_items']]}, rounds "
                  f"{r[F['mt_rounds']]}, passes {r[F['mt_passes']]} (early ends {r[F['mt_breaks']]}), staged "
                  f"{r[F['mt_staged']]}, pairs {r[F['mt_pairs']]}, gather {r[F['mt_gather']] / 100:.1f} us; wg {dur[i] / 100:.1f} us, "
                  f"busy {r[F['n_busy']]}", flush=True)
    ctx.close()
