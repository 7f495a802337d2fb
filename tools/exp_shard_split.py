"""Per-rank work of the tile-sharded C4 / C5 frame, measured on ONE GPU by rendering each rank's shard
in turn (shard_rank / shard_count): the Amdahl inputs for the N-GPU projection.
usage (GPU box): python tools/exp_shard_split.py [c4|c5] [frames] [N list, e.g. 1,2,4,8]
(env SPLIT_CULL=0|1: SHS_OPT_SHARD_CULL, SPLIT_PART=-1|0|n: SHS_OPT_LIB_PART, SPLIT_REGIONS=1: region layout)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ns = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 4, 8]
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
    else:
        frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160, 2048)
        lvp = ctx.render_shadow_map(S, sun, casters)
        scene_lib.wire_shadow(draws, lvp)
    ctx.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
    for N in ns:
        per_rank = []
        for r in range(N):
            frame.shard_rank, frame.shard_count = r, N
            if cfg == "c4":
                cull.shard_rank, cull.shard_count = r, N
            prep = ctx.prepare_lib(frame, draws)

            def one():
                if cfg == "c4":
                    ctx.light_cull(cull)
                else:
                    ctx.render_shadow_map(S, sun, casters)
                ctx.render_pbr_forward_prepared(prep)
                pass  # tonemap fused into the camera pass (ctx.fuse_tonemap)

            for _ in range(3):
                one()
            ctx.synchronize_lib()
            ctx.enable_timing(True)
            ctx.lib_timing_reset()
            t0 = time.perf_counter()
            for _ in range(nf):
                one()
            ctx.synchronize_lib()
            el = (time.perf_counter() - t0) / nf * 1e3
            _, kms = ctx.lib_timing_read()
            ctx.enable_timing(False)
            per_rank.append((el, kms))
        worst = max(per_rank, key=lambda x: x[0])
        ms = np.array([p[0] for p in per_rank])
        k = worst[1]
        print(f"{cfg} N={N}: per-rank ms/frame max {ms.max():.4f} mean {ms.mean():.4f} | worst rank kernels: "
              + " ".join(f"{a}={b:.4f}" for a, b in k.items()), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
