"""k_lib_setup per-workgroup timeline (SHS_OPT_TIMELINE) of the camera pass: where the setup's time
goes per block -- triangle setup (t1 - t0), deferred small-primitive marks (t2 - t1), the block's large
primitives' busy marks / bin appends (t3 - t2) -- and the launch span.
usage (GPU box): python tools/timeline_setup.py [c4|c5] [shard_count]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
    count = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    ctx = shs_gpu.Context(0)
    ctx.set_timeline(True)
    if cfg == "c4":
        frame, draws, lights, cull = scene_lib.c4_scene(3840, 2160)
        ctx.upload_lights(lights)
        ctx.light_cull(cull)
    else:
        frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160, 2048)
        lvp = ctx.render_shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)
    frame.shard_rank, frame.shard_count = 0, count
    prep = ctx.prepare_lib(frame, draws)
    for _ in range(5):
        ctx.render_pbr_forward_prepared(prep)
    ctx.synchronize_lib()
    ctx.render_pbr_forward_prepared(prep)
    ctx.synchronize_lib()
    t = ctx.lib_debug_setup_timeline().reshape(-1, 8).astype(np.int64)
    t = t[t[:, 0] != 0]   # a listed (tile-sharded) setup runs fewer workgroups than setup blocks
    t0 = t[:, 0].min()
    span = (t[:, 3].max() - t0) / 100.0
    tri = (t[:, 1] - t[:, 0]) / 100.0
    dfr = (t[:, 2] - t[:, 1]) / 100.0
    big = (t[:, 3] - t[:, 2]) / 100.0
    start = (t[:, 0] - t0) / 100.0
    print(f"{cfg} shards={count}: {len(t)} blocks, launch span {span:.1f} us; start offsets p50 {np.median(start):.1f} "
          f"max {start.max():.1f} us")
    for name, v in (("triangles", tri), ("deferred marks", dfr), ("large prims", big), ("total", tri + dfr + big)):
        print(f"  {name:15s} p50 {np.median(v):7.2f}  p90 {np.percentile(v, 90):7.2f}  max {v.max():7.2f} us")
    print(f"  large prims per block: mean {t[:, 4].mean():.1f} max {t[:, 4].max()}; union w*h mean {t[:, 5].mean():.1f}")
    if t[:, 6].any():
        fe = (t[:, 6] - t[:, 0]) / 100.0
        print(f"  cull front end  p50 {np.median(fe):7.2f}  p90 {np.percentile(fe, 90):7.2f}  max {fe.max():7.2f} us; "
              f"kept per block mean {t[:, 7].mean():.1f} max {t[:, 7].max()}")
    w = np.argmax(tri + dfr + big)
    print(f"  slowest block {w}: start {start[w]:.1f} tri {tri[w]:.1f} deferred {dfr[w]:.1f} big {big[w]:.1f} us, "
          f"nbig {t[w, 4]}")


if __name__ == "__main__":
    main()
