"""Tonemap kernel throughput at 4K (GPU box): C5 HDR frame -> PassTonemap (LDR + present)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "leisure-software-renderer_amd"), ROOT]
import torch  # noqa: E402
import shs_gpu  # noqa: E402
from shs_gpu import scene_lib  # noqa: E402

frame, draws, casters, sun, S = scene_lib.c5_scene(3840, 2160)
ctx = shs_gpu.Context(0)
stream = torch.cuda.Stream()          # a real stream: torch's default one is the null stream
torch.cuda.set_stream(stream)
ctx.set_stream(stream.cuda_stream)
ctx.render_pbr_forward(frame, draws)
for flags in ((True, True), (True, False)):
    for _ in range(10):
        ctx.tonemap(1.0, 2.2, *flags)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 200
    a.record()
    for _ in range(n):
        ctx.tonemap(1.0, 2.2, *flags)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / n
    px = frame.width * frame.height
    by = px * (16 + 4 * (int(flags[0]) + int(flags[1])))
    print(f"tonemap ldr={flags[0]} present={flags[1]}: {ms * 1e3:.1f} us/launch, {by / ms / 1e6:.0f} GB/s "
          f"({by / ms / 1e6 / 8000:.3f} of 8 TB/s), {px / ms / 1e3:.0f} Mpix/s", flush=True)
ctx.close()

# PassMotionBlur after a tonemap (RT_ColorLDR): default parameters
ctx = shs_gpu.Context(0)
ctx.set_stream(stream.cuda_stream)
ctx.render_pbr_forward(frame, draws)
ctx.tonemap(1.0, 2.2, ldr=True, present=False)
for present in (False, True):
    for _ in range(10):
        ctx.motion_blur(present=present)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 200
    a.record()
    for _ in range(n):
        ctx.motion_blur(present=present)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / n
    px = frame.width * frame.height
    by = px * (4 + 4 + 8 + 4 + 4 * int(present))   # src + depth + motion read, dst (+ present) written
    print(f"motion blur present={present}: {ms * 1e3:.1f} us/launch, {by / ms / 1e6:.0f} GB/s algorithmic "
          f"({by / ms / 1e6 / 8000:.3f} of 8 TB/s)", flush=True)
ctx.close()
