#!/usr/bin/env python3
"""Debug aid: the region-sharded 4K C4 frames of tests/test_shipped_regions.py, rank by rank, two
frames; for every rank the owned pixels' HDR / depth are compared with the oracle frame and the worst
mismatches printed with the rank's rectangle, the pixel's light-list tile and its list count.

  SHS_GPU_LIB=leisure-software-renderer_amd/shs_gpu/libshs_gpu_exp.so SHS_LIB_EXP=16 python tools/dbg_regions_c4.py     # with the wave light-list culling disabled"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]


def main():
    import shs_gpu
    from shs_gpu import scene_lib
    from oracle import oracle
    ranks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    frame, draws, lights, cull = scene_lib.c4_scene(3840, 2160)
    rc, ri = oracle.light_cull(cull, lights)[:2]
    rh, rd, rm, _ = oracle.forward_plus(frame, draws, lights, cull, (rc, ri))
    W, H = frame.width, frame.height
    ctxs = [shs_gpu.Context(0) for _ in range(ranks)]
    for c in ctxs:
        c.set_shard_layout(True)
        c.set_shard_root_share(0.85)
        c.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
        c.upload_lights(lights)
    for it in range(2):
        for r, c in enumerate(ctxs):
            frame.shard_rank, frame.shard_count = r, ranks
            cull.shard_rank, cull.shard_count = r, ranks
            c.light_cull(cull)
            c.render_pbr_forward(frame, draws)
            x0, y0, x1, y1 = c.shard_regions(ranks)[r]
            h, d, _ = c.resolve_lib()
            sl = (slice(y0 * 32, (y1 + 1) * 32), slice(x0 * 32, (x1 + 1) * 32))
            err = np.abs(h[sl].astype(np.float64) - rh[sl].astype(np.float64)).max(axis=2)
            derr = (d[sl].view(np.uint32) != rd[sl].view(np.uint32))
            bad = np.argwhere(err > 1e-5)
            counts, _, _ = c.resolve_light_lists()
            print(f"frame {it} rank {r} rect {(x0, y0, x1, y1)}: {len(bad)} px HDR off, {int(derr.sum())} depth off", flush=True)
            for by, bx in bad[:6]:
                py, px = y0 * 32 + by, x0 * 32 + bx
                lt = ((H - 1 - py) // 16) * ((W + 15) // 16) + px // 16
                print(f"   px ({px},{py}) gpu {h[py, px]} ref {rh[py, px]} depth {d[py, px]}/{rd[py, px]} "
                      f"list {lt} gpu count {counts[lt]} ref count {rc[lt]}", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
