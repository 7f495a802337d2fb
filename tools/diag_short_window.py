#!/usr/bin/env python3
"""Why the driver's short C2 bench window (--steps 20 --warmup 5) reads ~8 % below a 200-step run
(VERDICT r3, next-round item 2): the bench's exact C2 loop, timed as consecutive windows of 20 steps
(barrier + synchronize around each window, as bench.py does around its one window), with the mean
k_raster / k_setup event times of each window.  A slow first window that speeds up afterwards is a
warm-up effect (clocks, caches, first-touch); a flat series means the short window is just noise.

  python tools/diag_short_window.py [--windows 15] [--warmup 5] [--pre-legs]

--pre-legs runs bench.py's auxiliary legs (single-frame latency, Seam-1 PCIe) before the windows,
the order bench.py uses from round 4 on."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "leisure-software-renderer_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=15)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pre-legs", action="store_true")
    a = ap.parse_args()
    import bench
    import shs_gpu
    F = 64
    frame, sets = bench.batch_poses("c2", F)
    ctx = shs_gpu.Context(0)
    prepared = [ctx.prepare_batch(frame, fds) for fds in sets]
    t_start = time.perf_counter()
    if a.pre_legs:
        one = ctx.prepare(frame, sets[0][0])
        for _ in range(90):
            ctx.render_prepared(one)
        ctx.synchronize()
    for i in range(a.warmup):
        ctx.render_batch_prepared(prepared[i % 4])
    ctx.synchronize()
    ctx.render_batch_prepared(prepared[0])
    ctx.synchronize()
    out = []
    for w in range(a.windows):
        ctx.enable_timing(True)
        ctx.timing_reset()
        ctx.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            ctx.render_batch_prepared(prepared[i % 4])
        ctx.synchronize()
        el = time.perf_counter() - t0
        _, kms = ctx.timing_read()
        ctx.enable_timing(False)
        row = {"window": w, "t_since_start_ms": round((t0 - t_start) * 1e3, 1),
               "ms_per_step": round(el / a.steps * 1e3, 4), "mtri_s": round(967 * F * a.steps / el / 1e6, 1),
               "raster_ms": round(kms["raster"], 4), "setup_ms": round(kms["setup"], 4)}
        out.append(row)
        print(json.dumps(row), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
