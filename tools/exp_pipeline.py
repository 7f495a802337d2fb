"""Frames in flight: per-rank throughput of the tile-sharded C4 / C5 frame when D contexts (each with
its own stream and workspace) render consecutive frames round-robin, so frame k+1's kernels can run
while frame k's are still in flight.  Measured on ONE GPU, each rank's shard in turn (as
exp_shard_split.py), without the gather.
usage (GPU box): python tools/exp_pipeline.py [c4|c5] [frames] [N list] [depth list, e.g. 1,2,3]
(env SPLIT_CULL / SPLIT_PART / SPLIT_REGIONS as exp_shard_split.py; SPLIT_ONLY=r: rank r's shard only)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402


def make_ctx(cfg):
    ctx = shs_gpu.Context(0)
    if os.environ.get("SPLIT_CULL") is not None:
        ctx.set_shard_cull(os.environ["SPLIT_CULL"] == "1")
    if os.environ.get("SPLIT_PART") is not None:
        ctx.set_lib_part(int(os.environ["SPLIT_PART"]))
    if os.environ.get("SPLIT_REGIONS") == "1":
        ctx.set_shard_layout(True)
    if cfg == "c4":
        frame, draws, lights, cull = scene_lib.c4_scene(3840, 2160)
        ctx.upload_lights(lights)
        extra = cull
    else:
        frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160, 2048)
        # SPLIT_FOOTPRINT (default 1, bench.py's C5): the shadow pass over the camera pass's PCF footprint
        ctx.set_shadow_footprint(os.environ.get("SPLIT_FOOTPRINT", "1") == "1")
        lvp = ctx.render_shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)
        extra = (casters, sun, S)
    ctx.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
    return ctx, frame, draws, extra


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    ns = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 8]
    depths = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [1, 2, 3]
    pool = [make_ctx(cfg) for _ in range(max(depths))]
    for N in ns:
        for D in depths:
            per_rank, host_ms, sh_regs = [], [], []
            only = os.environ.get("SPLIT_ONLY")
            for r in ([int(only)] if only is not None and N > 1 else range(N)):
                ones = []
                for ctx, frame, draws, extra in pool[:D]:
                    frame.shard_rank, frame.shard_count = r, N
                    if cfg == "c4":
                        extra.shard_rank, extra.shard_count = r, N
                    prep = ctx.prepare_lib(frame, draws)

                    def one(ctx=ctx, prep=prep, extra=extra):
                        if cfg == "c4":
                            ctx.light_cull(extra)
                        else:
                            ctx.render_shadow_map(extra[2], extra[1], extra[0])
                        ctx.render_pbr_forward_prepared(prep)
                    ones.append(one)
                for i in range(3 * D):
                    ones[i % D]()
                for ctx, *_ in pool[:D]:
                    ctx.synchronize_lib()
                t0 = time.perf_counter()
                host = 0.0
                for i in range(nf):
                    h0 = time.perf_counter()
                    ones[i % D]()
                    host += time.perf_counter() - h0
                for ctx, *_ in pool[:D]:
                    ctx.synchronize_lib()
                per_rank.append((time.perf_counter() - t0) / nf * 1e3)
                host_ms.append(host / nf * 1e3)
                if cfg == "c5" and N > 1:
                    sh_regs.append(tuple(pool[0][0].shadow_region()))
            ms = np.array(per_rank)
            print(f"{cfg} N={N} frames in flight {D}: per-rank ms/frame max {ms.max():.4f} mean {ms.mean():.4f}"
                  f" | " + " ".join(f"{x:.4f}" for x in ms) + f" | host enqueue ms/frame {np.mean(host_ms):.4f}", flush=True)
            if N > 1 and os.environ.get("SPLIT_REGIONS") == "1":
                print(f"   regions {pool[0][0].shard_regions(N)}", flush=True)
            if sh_regs:
                print(f"   shadow-map tiles per rank {sh_regs}", flush=True)
    for ctx, *_ in pool:
        ctx.close()


if __name__ == "__main__":
    main()
