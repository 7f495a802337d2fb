"""Tiny C4-style frames (few triangles) for per-kernel trace timing (run under rocprofv3 --kernel-trace)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402

n_obj = int(sys.argv[1]) if len(sys.argv) > 1 else 1
tpo = int(sys.argv[2]) if len(sys.argv) > 2 else 100
n_draws = int(sys.argv[3]) if len(sys.argv) > 3 else 1
frame, draws, lights, cull = scene_lib.c4_scene(n_objects=n_obj, tris_per_object=tpo, n_draws=n_draws)
ctx = shs_gpu.Context(0)
ctx.upload_lights(lights)
prepared = ctx.prepare_lib(frame, draws)
for _ in range(30):
    ctx.light_cull(cull)
    ctx.render_pbr_forward_prepared(prepared)
ctx.synchronize_lib()
ctx.close()
print("done")
