"""Per-workgroup timeline of the library camera pass (SHS_OPT_TIMELINE): where k_lib_raster's time goes.

usage (GPU box): [SPLIT_REGIONS=1] python tools/timeline_lib.py [c4|c5] [n_objects] [tris_per_object] [shard_count] [rank]
Per workgroup: duration, summed phase times over its busy tiles (gather / stage + pairs / resolve +
shade), clear time, tile / chunk / pair / candidate counts; distribution over workgroups and the
slowest workgroup."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    ctx = shs_gpu.Context(0)
    ctx.set_timeline(True)
    if cfg == "c4":
        n_obj = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
        tpo = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
        frame, draws, lights, cull = scene_lib.c4_scene(n_objects=n_obj, tris_per_object=tpo)
        ctx.upload_lights(lights)

        def one():
            ctx.light_cull(cull)
            ctx.render_pbr_forward_prepared(prepared)
        ctx.light_cull(cull)
    else:
        frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160)
        lvp = ctx.render_shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)

        def one():
            ctx.render_pbr_forward_prepared(prepared)
    count = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    rank = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    if count > 1 and os.environ.get("SPLIT_REGIONS") == "1":   # the region layout (balanced on this context's passes)
        ctx.set_shard_layout(True)
    frame.shard_rank, frame.shard_count = rank, count
    if cfg == "c4":
        cull.shard_rank, cull.shard_count = rank, count
        ctx.light_cull(cull)
    prepared = ctx.prepare_lib(frame, draws)
    for _ in range(5):
        one()
    ctx.synchronize_lib()
    names = ctx.LIB_TIMELINE_FIELDS
    for rep in range(2):
        one()
        ctx.synchronize_lib()
        t = ctx.lib_debug_timeline().astype(np.int64)
        f = {n: t[:, i] for i, n in enumerate(names)}
        t0 = f["start"].min()
        dur = (f["end"] - f["start"]) / 100.0
        print(f"{cfg} frame {rep}: {len(t)} workgroups, span {(f['end'].max() - t0) / 100:.1f} us, "
              f"start spread {(f['start'].max() - t0) / 100:.1f} us")

        def dist(name, v):
            print(f"  {name:10s} med {np.median(v):9.2f} p90 {np.percentile(v, 90):9.2f} max {v.max():9.2f} "
                  f"sum {v.sum():12.1f}")
        dist("wg us", dur)
        for n in ("gather", "pairs", "stage", "seg", "shade", "clear", "max_tile", "tiles"):
            dist(n + " us", f[n] / 100.0)
        dist("after us", (f["end"] - f["last"]) / 100.0)
        dist("between us", ((f["end"] - f["start"]) - f["tiles"] - (f["end"] - f["last"])) / 100.0)
        for n in ("n_busy", "n_clear", "chunks", "n_pairs", "n_cand"):
            dist(n, f[n].astype(np.float64))
        st = ctx.lib_debug_setup_timeline().astype(np.int64)
        s0 = st[:, 0].min()
        sd = (st[:, 3] - st[:, 0]) / 100.0
        ks = int(np.argmax(sd))
        print(f"  setup: {len(st)} workgroups, span {(st[:, 3].max() - s0) / 100:.1f} us, start spread "
              f"{(st[:, 0].max() - s0) / 100:.1f} us; wg dur med {np.median(sd):.2f} p90 {np.percentile(sd, 90):.2f} "
              f"max {sd.max():.2f}; phases (tri/defer/big) med {np.median((st[:, 1] - st[:, 0]) / 100):.2f}/"
              f"{np.median((st[:, 2] - st[:, 1]) / 100):.2f}/{np.median((st[:, 3] - st[:, 2]) / 100):.2f}; "
              f"slowest wg {ks}: {(st[ks, 1] - st[ks, 0]) / 100:.2f}/{(st[ks, 2] - st[ks, 1]) / 100:.2f}/"
              f"{(st[ks, 3] - st[ks, 2]) / 100:.2f} big={st[ks, 4]} union={st[ks, 5]}; blocks with big prims "
              f"{int((st[:, 4] > 0).sum())}, no-agg unions {int((st[:, 5] > 256).sum())}")
        k = int(np.argmax(dur))
        print("  slowest wg %d: %s" % (k, " ".join(
            "%s=%s" % (n, ("%.1f" % (f[n][k] / 100.0)) if n in ("gather", "pairs", "stage", "seg", "shade", "clear", "max_tile", "tiles")
                       else int(f[n][k])) for n in names[2:])))
    ctx.close()


if __name__ == "__main__":
    main()
