"""Debug: C4 small through shs_group with N ranks -- per frame count of differing present pixels
against the unsharded context, one gather per frame and back to back."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402
from shs_gpu.group import Group  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
frame, draws, lights, cull = scene_lib.c4_scene(960, 540, n_objects=60, tris_per_object=500)
single = shs_gpu.Context(0)
single.upload_lights(lights)
single.light_cull(cull)
single.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
single.render_pbr_forward(frame, draws)
_, want = single.resolve_ldr()
wh, wd, wm = single.resolve_lib()
g = Group([0] * n)
g.upload_lights(lights)
g.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
for mode in ("sync", "b2b"):
    for k in range(3):
        g.light_cull(cull)
        g.render_pbr_forward(frame, draws)
        g.gather(single.TARGET_LIB_PRESENT)
        if mode == "sync":
            _, got = g.root.resolve_ldr()
            bad = (got != want).any(axis=2)
            ys, xs = np.nonzero(bad)
            tiles = sorted(set(((y // 32) * ((960 + 31) // 32) + x // 32) for y, x in zip(ys, xs)))
            print(mode, k, "bad px", int(bad.sum()), "tiles", tiles[:20], "owners", sorted(set(t % n for t in tiles)))
    if mode == "b2b":
        _, got = g.root.resolve_ldr()
        print(mode, "bad px", int((got != want).any(axis=2).sum()))
g.gather(single.TARGET_LIB)
gh, gd, gm = g.root.resolve_lib()
print("lib target: hdr bad", int((gh.view(np.uint32) != wh.view(np.uint32)).any(axis=2).sum()), "depth bad",
      int((gd.view(np.uint32) != wd.view(np.uint32)).sum()))
for r in range(n):
    c = g.ranks[r]
    print("rank", r, c.lib_stats())
print("single", single.lib_stats())

# the same shards rendered one context at a time (no group), and the per-rank light lists
wc, wi, _ = single.resolve_light_lists()
seq = np.zeros_like(wh)
for r in range(n):
    c = shs_gpu.Context(0)
    frame.shard_rank, frame.shard_count = r, n
    cull.shard_rank, cull.shard_count = r, n
    c.upload_lights(lights)
    c.light_cull(cull)
    lc, li, _ = c.resolve_light_lists()
    c.render_pbr_forward(frame, draws)
    h, d, m = c.resolve_lib()
    ty, tx = np.mgrid[0:540, 0:960] // 32
    own = ((ty * 30 + tx) % n) == r
    seq[own] = h[own]
    gl = g.ranks[r].resolve_light_lists()
    ltx, lty = cull.tiles
    ly, lx = np.mgrid[0:lty, 0:ltx]
    lown = ((((ly * 16) // 32) * 30 + (lx * 16) // 32) % n == r).reshape(-1)
    print("rank", r, "seq lists vs single (owned) bad", int((lc[lown] != wc[lown]).sum()),
          "group lists vs single (owned) bad", int((gl[0][lown] != wc[lown]).sum()), "owned", int(lown.sum()))
    c.close()
frame.shard_rank, frame.shard_count = 0, 1
print("sequential composed hdr bad", int((seq.view(np.uint32) != wh.view(np.uint32)).any(axis=2).sum()))
