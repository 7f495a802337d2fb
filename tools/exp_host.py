"""Host cost of enqueueing one tile-sharded C4 frame (light cull + camera pass), per call, with D
contexts round-robin: Python-side desc building, the shs_light_cull call, the shs_render_pbr_forward
call, and a host-only ctypes call for scale.
usage (GPU box): python tools/exp_host.py [N] [rank] [D] [frames]   (env SPLIT_REGIONS=1: region layout)"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rank = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    D = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    nf = int(sys.argv[4]) if len(sys.argv) > 4 else 200
    frame, draws, lights, cull = scene_lib.c4_scene(3840, 2160)
    frame.shard_rank, frame.shard_count = rank, N
    cull.shard_rank, cull.shard_count = rank, N
    ctxs = []
    for _ in range(D):
        c = shs_gpu.Context(0)
        if os.environ.get("SPLIT_REGIONS") == "1":
            c.set_shard_layout(True)
        c.upload_lights(lights)
        c.fuse_tonemap(1.0, 2.2, ldr=False, present=True)
        ctxs.append((c, c.prepare_lib(frame, draws)))
    cdesc = cull.desc()
    t = {"desc": 0.0, "cull": 0.0, "render": 0.0, "ctypes_noop": 0.0}
    words = ctypes.c_int64()
    for i in range(nf + 3 * D):
        c, prep = ctxs[i % D]
        a = time.perf_counter()
        cull.desc()
        b = time.perf_counter()
        c._check(c._lib.shs_light_cull(c._h, ctypes.byref(cdesc)))
        c._cull = cull
        d = time.perf_counter()
        c.render_pbr_forward_prepared(prep)
        e = time.perf_counter()
        c._lib.shs_tiles_rank_words(c._h, 1, rank, N, ctypes.byref(words))
        f = time.perf_counter()
        if i >= 3 * D:
            t["desc"] += b - a
            t["cull"] += d - b
            t["render"] += e - d
            t["ctypes_noop"] += f - e
    for c, _ in ctxs:
        c.synchronize_lib()
    print(f"N={N} rank {rank} D={D}: host us per frame " + " ".join(f"{k} {v / nf * 1e6:.1f}" for k, v in t.items()), flush=True)
    for c, _ in ctxs:
        c.close()


if __name__ == "__main__":
    main()
