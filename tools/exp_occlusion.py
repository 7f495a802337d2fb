"""Software occlusion pass timing (GPU box): shs_occlusion_pass vs the CPU restatement (1 thread)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402
from oracle import oracle  # noqa: E402   (CPU baseline only)

for n, (W, H) in ((300, (300, 225)), (2000, (300, 225)), (2000, (1200, 900))):
    objs, view, vp, _, _ = scene_lib.occlusion_scene(n_objects=n, seed=7, width=W, height=H)
    fv = np.arange(len(objs), dtype=np.uint32)
    ctx = shs_gpu.Context(0)
    for _ in range(3):
        got = ctx.occlusion_pass(W, H, view, vp, objs, fv)
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        got = ctx.occlusion_pass(W, H, view, vp, objs, fv)
    gpu_ms = (time.perf_counter() - t0) / reps * 1e3
    ctx.close()
    t0 = time.perf_counter()
    want = oracle.occlusion_pass(W, H, view, vp, objs, fv)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    same = np.array_equal(got[0], want[0]) and np.array_equal(got[2].view(np.uint32), want[2].view(np.uint32))
    print(f"occlusion {len(objs)} objects {W}x{H}: gpu {gpu_ms:.2f} ms/pass (synchronous, incl. host sort + copies), "
          f"cpu restatement {cpu_ms:.2f} ms (1 thread), occluded {int(want[0].sum())}, exact {same}", flush=True)
