"""Library camera-pass raster, per-workgroup timeline (SHS_OPT_TIMELINE, shs_lib_debug_timeline) for C4
at shard r of N: how long the workgroups run, and what the slowest ones spend (gather / stage + pairs /
resolve ticks summed over their tiles, candidates, longest busy tile).
usage (GPU box): python tools/exp_raster_timeline.py [N] [rank]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
R = int(sys.argv[2]) if len(sys.argv) > 2 else 0
frame, draws, lights, cull = scene_lib.c4_scene(3840, 2160)
ctx = shs_gpu.Context(0)
ctx.upload_lights(lights)
frame.shard_rank, frame.shard_count = R, N
cull.shard_rank, cull.shard_count = R, N
ctx.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
prep = ctx.prepare_lib(frame, draws)
for _ in range(5):
    ctx.light_cull(cull)
    ctx.render_pbr_forward_prepared(prep)
ctx.synchronize_lib()
ctx.set_timeline(True)
ctx.light_cull(cull)
ctx.render_pbr_forward_prepared(prep)
ctx.synchronize_lib()
t = ctx.lib_debug_timeline().astype(np.int64)
F = {k: i for i, k in enumerate(ctx.LIB_TIMELINE_FIELDS)}
st = t[:, F["start"]] - t[:, F["start"]].min()
en = t[:, F["end"]] - t[:, F["start"]].min()
dur = en - st
print(f"C4 shard {R}/{N}: {len(t)} raster workgroups, span {en.max() / 100:.1f} us; busy tiles {t[:, F['n_busy']].sum()}, "
      f"cleared {t[:, F['n_clear']].sum()}, candidates {t[:, F['n_cand']].sum()}, pairs {t[:, F['n_pairs']].sum()}")
print(f"  workgroup duration us: median {np.median(dur) / 100:.1f} p90 {np.percentile(dur, 90) / 100:.1f} max {dur.max() / 100:.1f}")
print(f"  longest single busy tile us: median {np.median(t[:, F['max_tile']]) / 100:.1f} max {t[:, F['max_tile']].max() / 100:.1f}")
for i in np.argsort(-dur)[:8]:
    row = t[i]
    print(f"  wg {i}: {dur[i] / 100:.1f} us, busy {row[F['n_busy']]}, cand {row[F['n_cand']]}, pairs {row[F['n_pairs']]}, "
          f"chunks {row[F['chunks']]}, gather {row[F['gather']] / 100:.1f} pairs {row[F['pairs']] / 100:.1f} "
          f"shade {row[F['shade']] / 100:.1f} clear {row[F['clear']] / 100:.1f}, longest tile {row[F['max_tile']] / 100:.1f}")
tot = {k: t[:, F[k]].sum() / 100 for k in ("gather", "pairs", "shade", "clear")}
print("  summed phase us over all workgroups:", {k: round(v, 1) for k, v in tot.items()}, "sum of durations", round(dur.sum() / 100, 1))
ctx.close()
