"""Canvas-API extras timing on device-resident buffers: combined_motion_blur_pass at
hello_pbr's 1200x900 and the DoF step (3 blur iterations, autofocus, composite) at the same size, against
the oracle's sequential restatement on one host thread.  Kernel times: rocprofv3 around this script."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "leisure-software-renderer_amd")


def main():
    import torch
    import shs_gpu
    from shs_gpu.scene_lib import look_at_lh, perspective_lh_no
    no_cpu = "--no-cpu" in sys.argv
    W, H, iters = 1200, 900, 50
    rng = np.random.default_rng(0)
    src = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    depth = rng.uniform(0.5, 80.0, size=(H, W)).astype(np.float32)
    vel = rng.normal(0.0, 8.0, size=(H, W, 2)).astype(np.float32)
    proj = perspective_lh_no(np.float32(np.deg2rad(60.0)), np.float32(W) / np.float32(H), np.float32(0.1), np.float32(1000.0))
    view = look_at_lh((0.0, 2.0, -6.0), (0.0, 1.0, 10.0))
    pview = look_at_lh((0.4, 2.1, -5.7), (0.3, 1.0, 10.0))
    ctx = shs_gpu.Context(0)
    stream = torch.cuda.Stream()          # a real stream: the events and the passes share it
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    t_src, t_depth, t_vel = (torch.from_numpy(a).cuda() for a in (src, depth, vel))
    t_dst = torch.empty_like(t_src)
    t_col = t_src.clone()
    t_blur = torch.empty_like(t_src)
    out = {"W": W, "H": H}
    for name, fn in (("motion_blur", lambda: ctx.canvas_motion_blur(t_src, t_depth, t_vel, view, proj, pview, proj, dst=t_dst)),
                     ("dof", lambda: (t_col.copy_(t_src), ctx.canvas_dof(t_col, t_depth, blur=t_blur)))):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[f"{name}_ms"] = round(e0.elapsed_time(e1) / iters, 4)
    if not no_cpu:
        from oracle import oracle
        t0 = time.perf_counter()
        oracle.canvas_motion_blur(src, depth, vel, view, proj, pview, proj)
        out["motion_blur_cpu_1thread_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
        t0 = time.perf_counter()
        oracle.canvas_dof(src, depth)
        out["dof_cpu_1thread_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
