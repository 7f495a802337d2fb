"""C4 cost breakdown (GPU box): kernel times of the library path under scene variants.

usage: python tools/exp_c4.py [frames]
Each variant prints mean k_lib_setup / k_lib_raster ms over `frames` frames and the pass stats."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import lib_path, scene_lib  # noqa: E402


def run(label, n_objects=1000, tpo=1000, program=None, width=3840, height=2160, frames=20, shard=(0, 1), n_lights=256,
        lists=False):
    frame, draws, lights, cull = scene_lib.c4_scene(width, height, n_objects=n_objects, tris_per_object=tpo,
                                                    n_lights=n_lights)
    frame.shard_rank, frame.shard_count = shard
    cull.shard_rank, cull.shard_count = shard
    if program is not None:
        for d in draws:
            d.program = program
    ctx = shs_gpu.Context(0)
    ctx.upload_lights(lights)
    ctx.light_cull(cull)
    prepared = ctx.prepare_lib(frame, draws)
    for _ in range(3):
        ctx.light_cull(cull)
        ctx.render_pbr_forward_prepared(prepared)
    ctx.synchronize_lib()
    st = ctx.lib_stats()
    ctx.enable_timing(True)
    ctx.lib_timing_reset()
    t0 = time.perf_counter()
    for _ in range(frames):
        ctx.light_cull(cull)
        ctx.render_pbr_forward_prepared(prepared)
    ctx.synchronize_lib()
    dt = (time.perf_counter() - t0) / frames * 1e3
    _, kms = ctx.lib_timing_read()
    if lists:
        counts = ctx.resolve_light_lists()[0]
        print(f"  light lists: mean {counts.mean():.1f}  p90 {sorted(counts.ravel())[int(0.9 * counts.size)]}  max {counts.max()}")
    ctx.close()
    print(f"{label:28s} frame {dt:7.3f} ms  setup {kms['setup']:7.3f}  raster {kms['raster']:7.3f}  "
          f"clip {st['tri_after_clip']} rast {st['tri_raster']} cov {st['covered_pixels']} maxbin {st['max_tile_bin']} "
          f"spill {st['spilled']} extra {st['clipped_extra']}", flush=True)


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    if len(sys.argv) > 2 and sys.argv[2] == "shade":
        run("c4", frames=frames, lists=True)
        for n in (1, 16, 64):
            run(f"c4 {n} lights", frames=frames, n_lights=n)
        run("c4 debug-albedo", program=lib_path.PROGRAM_DEBUG_ALBEDO, frames=frames)
        return
    run("c4", frames=frames)
    run("c4 debug-albedo", program=lib_path.PROGRAM_DEBUG_ALBEDO, frames=frames)
    run("c4 250k tris", n_objects=250, frames=frames)
    run("c4 100 obj x 100", n_objects=100, tpo=100, frames=frames)
    run("c4 1080p", width=1920, height=1080, frames=frames)
    for n in (2, 4, 8):
        run(f"c4 rank 0 of {n}", frames=frames, shard=(0, n))


if __name__ == "__main__":
    main()
