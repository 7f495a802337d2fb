"""Host enqueue rate vs GPU rate of the C4 / C5 frame (one rank's shard): is the per-frame time set by
the GPU or by the host's API calls?  usage (GPU box): python tools/exp_host_rate.py [c4|c5] [N] [frames]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    ctx = shs_gpu.Context(0)
    if cfg == "c4":
        frame, draws, lights, cull = scene_lib.c4_scene(3840, 2160)
        ctx.upload_lights(lights)
        cull.shard_rank, cull.shard_count = 0, N
    else:
        frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160, 2048)
        lvp = ctx.render_shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)
    frame.shard_rank, frame.shard_count = 0, N
    prep = ctx.prepare_lib(frame, draws)

    def one():
        if cfg == "c4":
            ctx.light_cull(cull)
        else:
            ctx.render_shadow_map(S, sun, casters)
        ctx.render_pbr_forward_prepared(prep)
        ctx.tonemap(1.0, 2.2, ldr=False, present=True)

    for _ in range(5):
        one()
    ctx.synchronize_lib()
    for rep in range(3):
        t0 = time.perf_counter()
        calls = []
        for _ in range(nf):
            a = time.perf_counter()
            one()
            calls.append(time.perf_counter() - a)
        t1 = time.perf_counter()
        ctx.synchronize_lib()
        t2 = time.perf_counter()
        calls.sort()
        print(f"{cfg} N={N}: enqueue {(t1 - t0) / nf * 1e3:.4f} ms/frame (median call {calls[nf // 2] * 1e3:.4f}, "
              f"max {calls[-1] * 1e3:.4f}), total {(t2 - t0) / nf * 1e3:.4f} ms/frame", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
