"""Rank 0 of an N-way region-sharded C4 / C5 frame with the gather's device work included: D contexts
render rank 0's shard round-robin (frames in flight), and after each frame rank 0 unpacks the N - 1
peers' packed present tiles (shs_tiles_unpack, what gather_frame_device / shs_group_gather run on rank
0 after the xGMI transfers).  The peers' buffers are packed once beforehand by contexts rendering
their shards (the transfer itself runs on the copy engines / RCCL and is not in this figure).  Prints
rank 0's ms/frame without and with the unpacks, and every rank's ms/frame for comparison.
usage (GPU box): python tools/exp_root.py [c4|c5] [N] [root_share] [frames] [D]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import torch  # noqa: E402
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402


def make(cfg, share):
    ctx = shs_gpu.Context(0)
    ctx.set_shard_layout(True)
    ctx.set_shard_root_share(share)
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


def frame_fn(cfg, ctx, prep, extra):
    def one():
        if cfg == "c4":
            ctx.light_cull(extra)
        else:
            ctx.render_shadow_map(extra[2], extra[1], extra[0])
        ctx.render_pbr_forward_prepared(prep)
    return one


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    share = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    nf = int(sys.argv[4]) if len(sys.argv) > 4 else 60
    D = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    T = shs_gpu.Context.TARGET_LIB_PRESENT
    pool = [make(cfg, share) for _ in range(D)]
    times = {}
    packed = {}
    for r in range(N):
        ones = []
        for ctx, frame, draws, extra in pool:
            frame.shard_rank, frame.shard_count = r, N
            if cfg == "c4":
                extra.shard_rank, extra.shard_count = r, N
            ones.append(frame_fn(cfg, ctx, ctx.prepare_lib(frame, draws), extra))
        for i in range(3 * D):
            ones[i % D]()
        for ctx, *_ in pool:
            ctx.synchronize_lib()
        t0 = time.perf_counter()
        for i in range(nf):
            ones[i % D]()
        for ctx, *_ in pool:
            ctx.synchronize_lib()
        times[r] = (time.perf_counter() - t0) / nf * 1e3
        if r > 0:   # this rank's packed present tiles, for rank 0's unpacks
            ctx = pool[0][0]
            b = torch.zeros(max(ctx.tiles_rank_words(T, r, N), 1), dtype=torch.int32, device="cuda:0")
            torch.cuda.synchronize()   # torch's fill (its own stream) before the pack
            ctx.tiles_pack(T, r, N, b.data_ptr())
            ctx.synchronize_lib()
            packed[r] = b
    regs = pool[0][0].shard_regions(N)
    # rank 0 again, each frame followed by the N - 1 unpacks on its context's stream
    ones = []
    for ctx, frame, draws, extra in pool:
        frame.shard_rank, frame.shard_count = 0, N
        if cfg == "c4":
            extra.shard_rank, extra.shard_count = 0, N
        f = frame_fn(cfg, ctx, ctx.prepare_lib(frame, draws), extra)

        def with_unpack(f=f, ctx=ctx):
            f()
            ctx.tiles_unpack_ranks(T, N, [0] + [packed[r].data_ptr() for r in range(1, N)])
        ones.append(with_unpack)
    for i in range(3 * D):
        ones[i % D]()
    for ctx, *_ in pool:
        ctx.synchronize_lib()
    t0 = time.perf_counter()
    for i in range(nf):
        ones[i % D]()
    for ctx, *_ in pool:
        ctx.synchronize_lib()
    root_gather = (time.perf_counter() - t0) / nf * 1e3
    ms = np.array([times[r] for r in range(N)])
    print(f"{cfg} N={N} D={D} root share {share}: per-rank ms/frame " + " ".join(f"{x:.4f}" for x in ms)
          + f" | rank 0 with {N - 1} unpacks {root_gather:.4f} | worst {max(ms[1:].max(), root_gather):.4f}", flush=True)
    print(f"   regions {regs}", flush=True)
    for ctx, *_ in pool:
        ctx.close()


if __name__ == "__main__":
    main()
