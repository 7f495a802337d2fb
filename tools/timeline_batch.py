"""Per-workgroup timeline of one legacy BATCH (SHS_OPT_TIMELINE): the bench's C2 / C3 step, one
k_setup + one k_raster over F frames, run with the setup on its own stream as in the bench.

usage (GPU box): python tools/timeline_batch.py [c2|c3] [frames]
Prints the setup and raster workgroups' start / end offsets and durations (us, relative to the first
setup workgroup), the setup phase marks, and the raster's start after the setup's end."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT, os.path.join(ROOT, "tools")]
import shs_gpu  # noqa: E402
import bench  # noqa: E402
from timeline import phases, summarize  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n_frames = int(sys.argv[2]) if len(sys.argv) > 2 else bench.LEGACY_FRAMES[cfg]
    frame, sets = bench.batch_poses(cfg, n_frames)
    ctx = shs_gpu.Context(0)
    ctx.set_timeline(True)
    prepared = [ctx.prepare_batch(frame, fds) for fds in sets]
    for i in range(20):
        ctx.render_batch_prepared(prepared[i % len(prepared)])
    ctx.synchronize()
    for rep in range(3):
        ctx.render_batch_prepared(prepared[rep % len(prepared)])
        ctx.synchronize()
        head, s, r = ctx.debug_timeline()
        t0 = int(s[:, 0].min())
        print(f"{cfg} batch of {n_frames} frames, step {rep}: {head}")
        # (batches: ghost waves inline or in k_ghost, so every k_setup workgroup is a setup block)
        summarize("setup", s, t0)
        summarize("raster", r, t0)
        phases(s, ["draw", "setup_tri", "busy", "bins", "make_rec", "stats"], "setup")
        phases(r, ["busy_list", "gather", "staged", "rastered", "shaded", "written"], "raster first tile")
        st = (s[:, 0].astype(np.int64) - t0) / 100.0
        en = (s[:, 1].astype(np.int64) - t0) / 100.0
        for q in (0.25, 0.5, 0.75, 0.9, 1.0):
            print(f"  setup workgroups started by {np.quantile(st, q):7.2f} us ({q:.0%}), ended by {np.quantile(en, q):7.2f} us")
        print(f"  setup span {en.max():.2f} us; raster first start {(int(r[:, 0].min()) - t0) / 100:.2f} us "
              f"(gap {(int(r[:, 0].min()) - int(s[:, 1].max())) / 100:.2f} us)")
    ctx.close()


if __name__ == "__main__":
    main()
