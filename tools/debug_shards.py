"""Diagnose shard-compose mismatches: prints differing pixels between full and sharded renders."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu
from shs_gpu import scene
from oracle import oracle

frame, draws = scene.monkey_scene(640, 480, 3, cam_pos=(0.0, 5.0, -12.0))
ctx = shs_gpu.Context(0)
ctx.render(frame, draws); fc, fd = ctx.resolve(); print("full stats", ctx.stats())
oc, od, _ = oracle.render_legacy(640, 480, draws)
print("full vs oracle depth diff", int((fd.view(np.uint32) != od.view(np.uint32)).sum()),
      "colour diff", int((fc != oc).any(-1).sum()))
T = shs_gpu.lib().shs_gpu_tile_size(); tx = (640 + T - 1) // T
for rank in range(3):
    f = shs_gpu.Frame(640, 480, shard_rank=rank, shard_count=3)
    ctx.render(f, draws); c, d = ctx.resolve(); print("rank", rank, ctx.stats())
    own = np.zeros((480, 640), bool)
    for ty in range((480 + T - 1) // T):
        for t in range(tx):
            if (ty * tx + t) % 3 == rank:
                own[ty * T:(ty + 1) * T, t * T:(t + 1) * T] = True
    dd = (d.view(np.uint32) != fd.view(np.uint32)) & own
    cd = (c != fc).any(-1) & own[::-1]
    print("  depth diffs", int(dd.sum()), "colour diffs", int(cd.sum()))
    ys, xs = np.nonzero(cd)
    for y, x in list(zip(ys, xs))[:8]:
        print("   canvas", y, x, "shard", c[y, x], "full", fc[y, x], "depth s/f", d[479 - y, x], fd[479 - y, x])
