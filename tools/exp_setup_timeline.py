"""Library camera-pass setup, per-workgroup timeline (SHS_OPT_TIMELINE, shs_lib_debug_setup_timeline):
start / triangles-done / deferred-marks-done / end per workgroup, for C4 at shard r of N.
usage (GPU box): python tools/exp_setup_timeline.py [N] [rank]   (env SPLIT_REGIONS=1: region layout)"""
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
if os.environ.get("SPLIT_REGIONS") == "1":
    ctx.set_shard_layout(True)
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
t = ctx.lib_debug_setup_timeline().astype(np.int64)
t0 = t[:, 0].min()
st, a, b, e = (t[:, k] - t0 for k in range(4))
dur = e - st
live = (a - st) > 0 if os.environ.get("SPLIT_REGIONS") == "1" else np.ones(len(t), bool)
if os.environ.get("SPLIT_REGIONS") == "1":   # skipped blocks record start == triangles-done
    live = t[:, 1] != t[:, 3]
    print(f"  surviving blocks {int(live.sum())} of {len(t)}; their duration median {np.median(dur[live]) / 100:.2f} us, "
          f"triangles phase {np.median((a - st)[live]) / 100:.2f}, skipped blocks' duration median {np.median(dur[~live]) / 100:.2f} us")
print(f"C4 shard {R}/{N}: {len(t)} setup workgroups, span {(e.max()) / 100:.1f} us (10 ns ticks / 100)")
print(f"  per-workgroup duration us: median {np.median(dur) / 100:.2f} p90 {np.percentile(dur, 90) / 100:.2f} max {dur.max() / 100:.2f}")
print(f"  triangles phase us: median {np.median(a - st) / 100:.2f}; deferred marks median {np.median(b - a) / 100:.2f}; "
      f"flush median {np.median(e - b) / 100:.2f}")
order = np.argsort(st)
for q in (0, 0.1, 0.25, 0.5, 0.75, 0.9, 1.0):
    i = order[min(int(q * (len(order) - 1)), len(order) - 1)]
    print(f"  start quantile {q:.2f}: start {st[i] / 100:.1f} us end {e[i] / 100:.1f} us")
conc = []
for ts in np.linspace(0, e.max(), 20):
    conc.append(int(((st <= ts) & (e > ts)).sum()))
print("  concurrent workgroups over the span:", conc)
ctx.close()
